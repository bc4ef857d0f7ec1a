#!/bin/bash
# the batch's SpMV inside the forward solve's launch (default) vs its own launch
# (GG_BATCH_FUSE=0): the batch GPU tests, then C5 with 8 scenarios, alternating
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-bfuse}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 1 0; do
    GG_BATCH_FUSE=$v timeout -k 10 300 python -u bench.py --workload c5 --c5-scenarios 8 --c5-mode batch --c5-steps 300 \
        --steps 1 --warmup 1 --cpu-iters 0 > $O/c5b8_f${v}_$rep.json 2> $O/c5b8_f${v}_$rep.err
    python3 -c "
import json; d=json.loads(open('$O/c5b8_f${v}_$rep.json').read().strip().splitlines()[-1]); print('fuse=$v', $rep, d['value'])" | tee -a $O/summary.txt
  done
done
