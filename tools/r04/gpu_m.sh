#!/bin/bash
# round 4: the MGS gather change first, then the bordered / netlist / grid-partition runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/r04/gpu_l.sh && bash tools/r04/gpu_k.sh
