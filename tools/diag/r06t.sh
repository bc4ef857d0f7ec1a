set -eo pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd_modes.py tests/test_gpu_dd_ranks.py tests/test_gpu_dd.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06t_dd_tests.log 2>&1
tail -2 gpurun_out/r06t_dd_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "spmv or sell or stream or panel" > gpurun_out/r06t_spmv_tests.log 2>&1
tail -1 gpurun_out/r06t_spmv_tests.log
bash tools/diag/dd_loop.sh r06t "c2 c4" "8" "cgs2"
GG_DD_HALO_FUSED=0 bash tools/diag/dd_loop.sh r06t_nf "c2 c4" "8" "cgs2"
