#!/bin/bash
# fused rows on skewed ILU(k) grids: the FMA / ILU(k) GPU tests, then C2 with
# ILU(1) / ILU(2) under GG_FMA_SKEW=1 (default) and 0 (GG_DIV_RCP's multiply)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-fskew}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fastdiv.py tests/test_gpu_parity.py -x -q --timeout 240 \
    --timeout-method thread -k "fma or iluk or skew" > $O/tests.log 2>&1
tail -1 $O/tests.log
for k in 1 2; do
  for v in 1 0; do
    GG_FMA_SKEW=$v timeout -k 10 300 python -u bench.py --ilu-level $k --steps 2 --warmup 1 --cpu-iters 0 \
        > $O/c2_ilu${k}_s$v.json 2> $O/c2_ilu${k}_s$v.err
    python3 -c "
import json; d=json.loads(open('$O/c2_ilu${k}_s$v.json').read().strip().splitlines()[-1]); k=d['kernels']
print('ilu$k skew_fma=$v', d['value'], d['ms_per_step'], {n: k[n]['avg_us'] for n in k})" | tee -a $O/summary.txt
  done
done
