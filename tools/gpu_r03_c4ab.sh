set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "c4_single" --timeout 250 --timeout-method thread > $O/r03_c4_test.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_c4_stash.json 2> $O/r03_c4.err &&
GGMRES_LIB=variants/libggmres_nostash.so timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_c4_nostash.json 2>> $O/r03_c4.err &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_c4_stash2.json 2>> $O/r03_c4.err
