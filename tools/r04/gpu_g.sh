#!/bin/bash
# round 4: padding skip (UnitMap) -- parity, then C2 / C4 A/B (GG_NO_PADSKIP)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_c2_history.py tests/test_gpu_residency.py tests/test_golden.py \
  "tests/test_gpu_parity.py::test_gmres_left_c1_parity" "tests/test_gpu_parity.py::test_gmres_wide_orthogonalization_parity" \
  "tests/test_gpu_parity.py::test_wave3d_apply_and_gmres" "tests/test_gpu_parity.py::test_gmres_split_parity" \
  "tests/test_gpu_parity.py::test_gmres_split_wavefront_parity" "tests/test_gpu_parity.py::test_gmres_iluk_grid_parity" \
  "tests/test_gpu_fastdiv.py::test_fma_c4_first_iterations" "tests/test_gpu_fastdiv.py::test_fma_gmres_parity" \
  > gpurun_out/r04g_tests.log 2>&1 || { tail -30 gpurun_out/r04g_tests.log; exit 1; }
tail -1 gpurun_out/r04g_tests.log
for r in 1 2; do
  for ps in 0 1; do
    GG_NO_PADSKIP=$ps timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 --cpu-iters 0 \
      > gpurun_out/r04g_c2_ps$ps_$r.json 2> /dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04g_c2_ps$ps_$r.json').read().strip().splitlines()[-1])
k=d['kernels']; print('C2 no_padskip=$ps run $r', d['value'], {n:k[n]['avg_us'] for n in k})"
  done
done
for ps in 0 1; do
  GG_NO_PADSKIP=$ps timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-iters 0 \
    > gpurun_out/r04g_c4_ps$ps.json 2> /dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04g_c4_ps$ps.json').read().strip().splitlines()[-1])
k=d['kernels']; print('C4 no_padskip=$ps', d['value'], {n:k[n]['avg_us'] for n in k})"
done
