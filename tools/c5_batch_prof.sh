#!/bin/bash
# C5 many-RHS batch: rocprofv3 kernel traces at several batch sizes (one call)
#   bash tools/c5_batch_prof.sh TAG STEPS S...
set -o pipefail
TAG=$1; ST=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for S in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s$S -o run -- python3 -u bench.py --workload c5 --c5-mode batch \
      --c5-scenarios $S --c5-steps $ST --steps 1 --warmup 0 --cpu-iters 0 --no-profile > $O/s$S.json 2> $O/s$S.err || exit 1
done
