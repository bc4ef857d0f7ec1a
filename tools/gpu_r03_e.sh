# round-3 GPU batch: GG_DIV_FMA on the split (PG) engine -- tests, PG bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fastdiv.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/r03_gpu_fma_split_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload pg --division fma --cpu-iters 0 > $O/r03_bench_pg_fma.json 2> $O/r03_bench_pg.err &&
timeout -k 10 300 python -u bench.py --workload pg --division rcp --cpu-iters 0 > $O/r03_bench_pg_rcp_ab.json 2>> $O/r03_bench_pg.err
