set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/sfprof -o sf -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 4 --steps 1 --warmup 0 --no-profile > $O/r03_sfprof.json 2> $O/r03_sfprof.err &&
find /tmp/sfprof -name "*kernel_stats.csv" -exec cp {} $O/r03_kernel_stats_dd_c2_local4_sepflow.csv \;
