set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python -u bench.py --workload dd --dd-grid c2 --steps 1 --warmup 1"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd.py tests/test_gpu_dd_ranks.py tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > $O/r03_sf_tests.log 2>&1 &&
timeout -k 10 300 $B --dd-parts 4 > $O/r03_sf_p4_new.json 2> $O/r03_sf.err &&
GG_DD_SEPFLOW=0 timeout -k 10 300 $B --dd-parts 4 > $O/r03_sf_p4_old.json 2>> $O/r03_sf.err &&
timeout -k 10 300 $B --dd-parts 8 > $O/r03_sf_p8_new.json 2>> $O/r03_sf.err &&
GG_DD_SEPFLOW=0 timeout -k 10 300 $B --dd-parts 8 > $O/r03_sf_p8_old.json 2>> $O/r03_sf.err &&
timeout -k 10 300 $B --dd-parts 2 > $O/r03_sf_p2_new.json 2>> $O/r03_sf.err &&
GG_DD_SEPFLOW=0 timeout -k 10 300 $B --dd-parts 2 > $O/r03_sf_p2_old.json 2>> $O/r03_sf.err
