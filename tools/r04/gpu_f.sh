#!/bin/bash
# round 4: MGS prefetch A/B (GG_MGS_PREFETCH 1 / 0) x gather form (0 / 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
GG_MGS_PREFETCH=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_c2_history.py "tests/test_gpu_parity.py::test_gmres_left_c1_parity" > gpurun_out/r04f_tests.log 2>&1 || { tail -30 gpurun_out/r04f_tests.log; exit 1; }
tail -1 gpurun_out/r04f_tests.log
for r in 1 2; do
  for cfg in "1 2" "0 2" "0 0"; do
    set -- $cfg
    GG_MGS_PREFETCH=$1 GG_MGS_GATHER=$2 timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 --cpu-iters 0 \
      > gpurun_out/r04f_pf$1_xg$2_$r.json 2> /dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04f_pf$1_xg$2_$r.json').read().strip().splitlines()[-1])
k=d['kernels']; print('pf=$1 xg=$2 run $r', d['value'], {n:k[n]['avg_us'] for n in k})"
  done
done
