# round-3 GPU batch: final profiles with GG_DIV_FMA (C2, PG, C4 kernel stats + PMC traffic), C5 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile_round.sh r03fma c2 &&
bash tools/profile_round.sh r03fma pg &&
bash tools/profile_round.sh r03fma c4 &&
timeout -k 10 300 python -u bench.py --workload c5 > gpurun_out/r03_bench_c5_fma.json 2> gpurun_out/r03_c5.err
