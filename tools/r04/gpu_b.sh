#!/bin/bash
# round 4: the C2 full-history parity, golden FMA, engine cache test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_c2_history.py tests/test_golden.py "tests/test_gpu_boundary.py::test_engine_abi_tran_keeps_its_solver" \
  > gpurun_out/r04b_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|C2 full|GMRES_GPU_tran" gpurun_out/r04b_tests.log | tail -40
exit $rc
