# round-3 final measurement batch: the GPU suite, profiles with PMC traffic for
# C2 / C4 / PG, bench lines for every workload (each step time-limited, chained)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03_gpu_tests_final.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03 c2 > $O/prof_c2.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03 c4 > $O/prof_c4.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03 pg > $O/prof_pg.log 2>&1
