#!/bin/bash
# round 4: XCD-local MGS gather -- parity, then C2 A/B (GG_MGS_GATHER 0 / 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_c2_history.py tests/test_gpu_residency.py \
  "tests/test_gpu_parity.py::test_gmres_left_c1_parity" "tests/test_gpu_fastdiv.py::test_fma_gmres_parity" \
  > gpurun_out/r04c_tests.log 2>&1 || { tail -30 gpurun_out/r04c_tests.log; exit 1; }
tail -3 gpurun_out/r04c_tests.log
for r in 1 2; do
  for xg in 0 2; do
    GG_MGS_GATHER=$xg timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-iters 0 \
      > gpurun_out/r04c_bench_xg${xg}_$r.json 2> gpurun_out/r04c_bench_xg${xg}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r04c_bench_xg${xg}_$r.json').read().strip().splitlines()[-1])
k=d['kernels']; print('xg=$xg run $r', d['value'], 'it/s', {n:k[n]['avg_us'] for n in k})"
  done
done
