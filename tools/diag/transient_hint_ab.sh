#!/bin/bash
# transient steps: the hinted short first chunk (default) vs two speculative cycles
# (GG_TRANSIENT_HINT=0): the transient GPU tests, then the C5 line under each
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-thint}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_netlist.py \
    -x -q --timeout 300 --timeout-method thread -m gpu -k "transient or c5" > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 1 0; do
    GG_TRANSIENT_HINT=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --cpu-iters 0 \
        > $O/c5_h${v}_$rep.json 2> $O/c5_h${v}_$rep.err
    python3 -c "
import json; d=json.loads(open('$O/c5_h${v}_$rep.json').read().strip().splitlines()[-1]); print('hint=$v', $rep, d['value'], d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
