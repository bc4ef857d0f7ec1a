#!/bin/bash
# tools/profile_round.sh over several workloads in one GPU call:
#   tools/profile_all.sh TAG WL...
set -eo pipefail
TAG=$1; shift
for wl in "$@"; do bash tools/profile_round.sh "$TAG" "$wl" 2>&1 | tail -1; done
