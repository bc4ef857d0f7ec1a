#!/bin/bash
# round 4, first GPU check: the residency / queue / engine-cache changes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_residency.py tests/test_gpu_boundary.py "tests/test_gpu_fastdiv.py::test_fused_spmv_same_bits" \
  > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r04a_tests.log
exit $rc
