set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python -u bench.py --workload c2 --steps 2 --cpu-iters 0"
D="python -u bench.py --workload dd --dd-grid c2 --steps 1 --warmup 1"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py -x -q -k "cgs2" --timeout 300 --timeout-method thread > $O/r03_ab2_tests.log 2>&1 &&
timeout -k 10 300 $D --dd-parts 4 > $O/r03_ab2_p4.json 2> $O/r03_ab2.err &&
timeout -k 10 300 $D --dd-parts 8 > $O/r03_ab2_p8.json 2>> $O/r03_ab2.err &&
timeout -k 10 300 $B > $O/r03_ab2_c2a.json 2>> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_lxcd.so timeout -k 10 300 $B > $O/r03_ab2_lxcd1.json 2>> $O/r03_ab2.err &&
timeout -k 10 300 $B > $O/r03_ab2_c2b.json 2>> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_lxcd.so timeout -k 10 300 $B > $O/r03_ab2_lxcd2.json 2>> $O/r03_ab2.err
