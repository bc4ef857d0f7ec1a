#!/bin/bash
# round 4: static tiles + fallback; parity + residency + C4 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_residency.py "tests/test_gpu_parity.py::test_tile3d_edges_and_ranges" \
  "tests/test_gpu_fastdiv.py::test_fma_c4_first_iterations" tests/test_gpu_dd.py \
  > gpurun_out/r04i_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/r04i_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r04i_tests.log | tail -2
timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-iters 0 > gpurun_out/r04i_c4.json 2> /dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r04i_c4.json').read().strip().splitlines()[-1])
k=d['kernels']; print('C4', d['value'], {n:k[n]['avg_us'] for n in k})"
