# round-3 closing batch (fused SpMV kernels): the GPU suite, then profiles with
# PMC traffic for C2 / PG / C4 (each step time-limited, chained)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03_gpu_tests_fused.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs c2 > $O/prof_c2.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs pg > $O/prof_pg.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs c4 > $O/prof_c4.log 2>&1
