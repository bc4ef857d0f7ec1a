# fused SpMV with 2-slice groups: bit-identity tests, then C2 / PG / C4 profiles with PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastdiv.py -x -v -k "fused or fma" --timeout 200 --timeout-method thread > $O/fsg2_tests.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs2 c2 > $O/prof_c2.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs2 pg > $O/prof_pg.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs2 c4 > $O/prof_c4.log 2>&1
