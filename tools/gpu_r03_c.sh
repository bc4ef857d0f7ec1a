# round-3 GPU batch C: the whole GPU suite (incl. the split wavefront cases),
# bench lines (C2, PG engine, sharded solves), a kernel-stats profile of the
# sharded C2 solve (the trace itself is deleted: gpurun_out must stay < 64 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/r03_bench_c2.json 2> $O/r03_bench.err &&
timeout -k 10 300 python -u bench.py --workload pg > $O/r03_bench_pg.json 2>> $O/r03_bench.err &&
timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --max-iter 600 > $O/r03_bench_pg_random.json 2>> $O/r03_bench.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 > $O/r03_dd_c2_p2_cgs2.json 2> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --dd-orth mgs > $O/r03_dd_c2_p2_mgs.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 4 > $O/r03_dd_c2_p4_cgs2.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-parts 8 > $O/r03_dd_c4_p8_cgs2.json 2>> $O/r03_dd.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_dd -o run -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --steps 1 --warmup 0 > $O/r03_dd_prof.json 2> $O/r03_dd_prof.err &&
find /tmp/prof_dd -name '*kernel_stats.csv' -exec cp {} $O/r03_kernel_stats_dd_c2_local2_cgs2.csv \;
