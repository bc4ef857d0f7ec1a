# round-3 GPU batch: the fast-division tests (GG_DIV_FMA incl. 3D tiles), C4 A/B,
# the C2 wavefront trace under GG_DIV_FMA, the whole GPU suite, local-shard C2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fastdiv.py -x -q --timeout 200 --timeout-method thread > $O/r03_gpu_fma_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 --division fma > $O/r03_bench_c4_fma.json 2> $O/r03_bench_c4.err &&
timeout -k 10 300 python -u bench.py --workload c4 --division rcp > $O/r03_bench_c4_rcp_ab.json 2>> $O/r03_bench_c4.err &&
timeout -k 10 120 python -u tools/wave_trace.py --division fma > $O/r03_wave_trace_fma.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03_gpu_tests_head.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 2 --division fma > $O/r03_dd_c2_p2_fma.json 2> $O/r03_dd_fma.err &&
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 4 --division fma > $O/r03_dd_c2_p4_fma.json 2>> $O/r03_dd_fma.err
