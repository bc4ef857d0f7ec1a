# round-3 GPU batch: one-barrier block sums in the one-launch orthogonalization kernels
# (bit-identical): the GMRES parity tests, then C2 / C4 A/B against the previous kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastdiv.py -x -q --timeout 200 --timeout-method thread > $O/r03_pp_tests.log 2>&1 &&
B="python -u bench.py --cpu-iters 0"
timeout -k 10 200 $B > $O/r03_pp_new.json 2> $O/r03_pp.err &&
GGMRES_LIB=variants/libggmres_prev.so timeout -k 10 200 $B > $O/r03_pp_prev.json 2>> $O/r03_pp.err &&
timeout -k 10 200 $B > $O/r03_pp_new2.json 2>> $O/r03_pp.err &&
GGMRES_LIB=variants/libggmres_prev.so timeout -k 10 200 $B > $O/r03_pp_prev2.json 2>> $O/r03_pp.err &&
timeout -k 10 300 $B --workload c4 > $O/r03_pp_c4_new.json 2>> $O/r03_pp.err &&
GGMRES_LIB=variants/libggmres_prev.so timeout -k 10 300 $B --workload c4 > $O/r03_pp_c4_prev.json 2>> $O/r03_pp.err
