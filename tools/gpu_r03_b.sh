# round-3 GPU batch: latency probe (contraction off), the whole GPU suite, sharded-solve bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 ./tools/lat_probe > $O/r03_lat_probe.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 > $O/r03_dd_c2_p2_cgs2.json 2> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --dd-orth mgs > $O/r03_dd_c2_p2_mgs.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 4 > $O/r03_dd_c2_p4_cgs2.json 2>> $O/r03_dd.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-parts 8 > $O/r03_dd_c4_p8_cgs2.json 2>> $O/r03_dd.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dd_c2_p2 -o run -f csv -- python3 -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --steps 1 --warmup 0 > $O/r03_dd_prof.json 2> $O/r03_dd_prof.err
