#!/bin/bash
# Round 5: per-rank sharded solve (loopback, P = 8) -- the CGS2 exchanges inside
# the kernels (GG_DD_XK) and the SpMV's interface exchange in line on the
# solver's stream (GG_DD_HALO_INLINE) against the launch-per-step path: the dd
# GPU tests first (the IPC ranks test runs the in-kernel CGS2 exchange), then
# alternating variants, then per-kernel times of the chosen one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05n}
GG_DD_HALO_INLINE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dd_ranks.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_ddtests.log 2>&1 || { tail -30 gpurun_out/${T}_ddtests.log; exit 1; }
tail -1 gpurun_out/${T}_ddtests.log
for g in c2 c4; do
    for rep in 1 2; do
        for v in "0 0" "1 0" "1 1"; do
            set -- $v
            f=gpurun_out/${T}_xk$1_hi$2_${g}_$rep
            GG_DD_XK=$1 GG_DD_HALO_INLINE=$2 timeout -k 10 300 python -u bench.py --workload dd --dd-grid $g \
                --dd-part grid --dd-parts 8 --dd-comm loopback --dd-rank 0 --max-iter 300 --steps 2 --warmup 1 \
                > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
            python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_per_rank"][0]["kernels"]
print(sys.argv[1], d["value"], "it/s;", {n: v["avg_us_per_shard"] for n, v in k.items()})
PY
        done
    done
done
# per-kernel times of the per-rank solve (C4/8 and C2/8 loopback)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for g in c4 c2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$g -o run -f csv -- \
        python3 -u bench.py --workload dd --dd-grid $g --dd-part grid --dd-parts 8 --dd-comm loopback --dd-rank 0 \
        --max-iter 300 --steps 2 --warmup 1 > gpurun_out/${T}_prof_$g.log 2>&1 || { tail -20 gpurun_out/${T}_prof_$g.log; exit 1; }
    f=$(find gpurun_out/${T}_prof_$g -name '*kernel_stats.csv' | head -1)
    cp "$f" gpurun_out/${T}_kstats_$g.csv
    head -25 gpurun_out/${T}_kstats_$g.csv | cut -c1-160
    rm -rf gpurun_out/${T}_prof_$g
done
