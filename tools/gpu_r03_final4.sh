# round-3 closing batch, part 2: PG and C4 profiles with PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 bash tools/profile_round.sh r03fs pg > $O/prof_pg.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs c4 > $O/prof_c4.log 2>&1
