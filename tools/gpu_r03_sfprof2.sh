set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/sfprof2 -o sf -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --steps 1 --warmup 0 --no-profile > $O/r03_sfprof2.json 2> $O/r03_sfprof2.err &&
find /tmp/sfprof2 -name "*kernel_stats.csv" -exec cp {} $O/r03_kernel_stats_dd_c2_local2_r03.csv \;
