# round-3 GPU check: latency probe, new-mode parity tests, bench lines (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/lat_probe > gpurun_out/r03_lat_probe.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_fastdiv.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_fastdiv.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_dd_ranks.py tests/test_gpu_dd.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_dd.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03_bench_rcp.json 2> gpurun_out/r03_bench_rcp.err &&
timeout -k 10 300 python -u bench.py --division exact > gpurun_out/r03_bench_exact.json 2> gpurun_out/r03_bench_exact.err
