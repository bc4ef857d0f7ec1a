#!/bin/bash
# C5 many-RHS batch: rocprofv3 kernel traces at several batch sizes (one call)
#   bash tools/c5_batch_prof.sh TAG STEPS S... (an item S:ENV=V runs S with that environment)
set -o pipefail
TAG=$1; ST=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for item in "$@"; do
  S=${item%%:*}; E=""; [ "$item" != "$S" ] && E=${item#*:}
  t=$(echo "s$S${E:+_$E}" | tr '=' '-')
  env $E timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$t -o run -- python3 -u bench.py --workload c5 --c5-mode batch \
      --c5-scenarios $S --c5-steps $ST --steps 1 --warmup 0 --cpu-iters 0 --no-profile > $O/$t.json 2> $O/$t.err || exit 1
done
