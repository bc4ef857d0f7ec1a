#!/bin/bash
# Refresh the committed profile set on a GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh TAG [WORKLOAD]        (WORKLOAD: c2 (default), c4, pg, pgr, netlist, c5, c3, c3s,
#                                                 c2_ilu1, c3s_ilu1)
# writes gpurun_out/prof_TAG[_WORKLOAD]/{bench.json, kernel_stats.csv, pmc_traffic.json}
# Each GPU step has its own time limit; the steps are chained with && so the
# script ends at the first failure.
set -eo pipefail
TAG=${1:-r02}
WL=${2:-c2}
OUT=gpurun_out/prof_${TAG}_${WL}
ARGS=""
[ "$WL" = c2 ] || ARGS="--workload $WL"
[ "$WL" = pgr ] && ARGS="--workload pg --pg-perm random"      # the split on the flow kernel
[ "$WL" = c2_ilu1 ] && ARGS="--ilu-level 1"                     # ILU(1) grid factors (skewed wavefront)
[ "$WL" = c3s_ilu1 ] && ARGS="--workload c3s --ilu-level 1"     # C3's own preconditioner on the stand-in
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run -f csv -- \
    python3 -u bench.py $ARGS --steps 1 --warmup 1 --cpu-iters 0 > $OUT/bench_under_rocprof.json 2> $OUT/stats.err
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -f csv -- \
    python3 -u bench.py $ARGS --steps 1 --warmup 0 --cpu-iters 0 --max-iter 600 --no-profile > /dev/null 2> $OUT/fetch.err
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -f csv -- \
    python3 -u bench.py $ARGS --steps 1 --warmup 0 --cpu-iters 0 --max-iter 600 --no-profile > /dev/null 2> $OUT/write.err
python3 profiles/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json
find $OUT -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
# the per-dispatch traces are tens of MB at C2 (gpurun_out comes back only under 64 MiB)
rm -rf $OUT/fetch $OUT/write $OUT/stats
echo "profile $TAG $WL done"
