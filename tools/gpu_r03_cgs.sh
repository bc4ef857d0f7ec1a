set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
D="python -u bench.py --workload dd --dd-grid c2 --steps 1 --warmup 1"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_dd_ranks.py -x -q --timeout 300 --timeout-method thread > $O/r03_cgs_tests.log 2>&1 &&
timeout -k 10 300 $D --dd-parts 2 > $O/r03_cgs_p2.json 2> $O/r03_cgs.err &&
timeout -k 10 300 $D --dd-parts 4 > $O/r03_cgs_p4.json 2>> $O/r03_cgs.err &&
timeout -k 10 300 $D --dd-parts 8 > $O/r03_cgs_p8.json 2>> $O/r03_cgs.err &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cgsprof -o sf -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --steps 1 --warmup 0 --no-profile > $O/r03_cgsprof.json 2> $O/r03_cgsprof.err &&
find /tmp/cgsprof -name "*kernel_stats.csv" -exec cp {} $O/r03_kernel_stats_dd_c2_local2_cgsreg.csv \;
