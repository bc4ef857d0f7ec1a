# round-3 GPU batch: GG_DIV_FMA -- C2 bench A/B (fma, rcp, fma)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u bench.py --division fma --cpu-iters 0 > $O/r03_bench_c2_fma.json 2> $O/r03_bench_fma.err &&
timeout -k 10 300 python -u bench.py --division rcp --cpu-iters 0 > $O/r03_bench_c2_rcp_ab.json 2>> $O/r03_bench_fma.err &&
timeout -k 10 300 python -u bench.py --division fma --cpu-iters 0 > $O/r03_bench_c2_fma2.json 2>> $O/r03_bench_fma.err
