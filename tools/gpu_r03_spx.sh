set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spmv" --timeout 300 --timeout-method thread > $O/r03_spx_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_spx_c4new.json 2> $O/r03_spx.err &&
GGMRES_LIB=variants/libggmres_spx0.so timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_spx_c4old.json 2>> $O/r03_spx.err &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 2 --cpu-iters 0 > $O/r03_spx_c2new.json 2>> $O/r03_spx.err &&
GGMRES_LIB=variants/libggmres_spx0.so timeout -k 10 300 python -u bench.py --workload c2 --steps 2 --cpu-iters 0 > $O/r03_spx_c2old.json 2>> $O/r03_spx.err
