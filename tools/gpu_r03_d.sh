# round-3 GPU batch D: sharded-solve tests (division mode), the IPC exchange
# latency probe, sharded bench lines with the reciprocal-multiply division
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_dd_ranks.py -x -q --timeout 300 --timeout-method thread > $O/r03_dd_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ipc_exchange_probe.py 1000 > $O/r03_ipc_exchange.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 > $O/r03_dd_c2_p2_cgs2_rcp.json 2> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 4 > $O/r03_dd_c2_p4_cgs2_rcp.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 8 > $O/r03_dd_c2_p8_cgs2_rcp.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-parts 8 > $O/r03_dd_c4_p8_cgs2_rcp.json 2>> $O/r03_dd.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_dd4 -o run -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 4 --steps 1 --warmup 0 > $O/r03_dd_prof4.json 2> $O/r03_dd_prof4.err &&
find /tmp/prof_dd4 -name '*kernel_stats.csv' -exec cp {} $O/r03_kernel_stats_dd_c2_local4_cgs2_rcp.csv \; &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_dd8 -o run -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 8 --steps 1 --warmup 0 > $O/r03_dd_prof8.json 2> $O/r03_dd_prof8.err &&
find /tmp/prof_dd8 -name '*kernel_stats.csv' -exec cp {} $O/r03_kernel_stats_dd_c2_local8_cgs2_rcp.csv \; &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_dd2 -o run -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --steps 1 --warmup 0 > $O/r03_dd_prof2.json 2> $O/r03_dd_prof2.err &&
find /tmp/prof_dd2 -name '*kernel_stats.csv' -exec cp {} $O/r03_kernel_stats_dd_c2_local2_cgs2_rcp.csv \;
