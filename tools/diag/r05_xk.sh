#!/bin/bash
# Round 5: the sharded solve's in-kernel exchanges (GG_DD_XK) -- the IPC ranks
# test both ways, loopback P = 8 per-rank timing alternating xk 0 / 1 (halo in
# line), then per-kernel times of both at C2/8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dd_ranks.py -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_ddtests.log 2>&1; rc=$?
grep -E "^E  |passed|failed" gpurun_out/${T}_ddtests.log | head -20
[ $rc -le 1 ] || exit 1
for g in c2 c4; do
    for rep in 1 2; do
        for xk in 0 1; do
            f=gpurun_out/${T}_xk${xk}_${g}_$rep
            GG_DD_XK=$xk timeout -k 10 300 python -u bench.py --workload dd --dd-grid $g \
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
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
for xk in 0 1; do
    g=c2
    GG_DD_XK=$xk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$xk -o run -f csv -- \
        python3 -u bench.py --workload dd --dd-grid $g --dd-part grid --dd-parts 8 --dd-comm loopback --dd-rank 0 \
        --max-iter 300 --steps 2 --warmup 1 > gpurun_out/${T}_prof_$xk.log 2>&1 || { tail -20 gpurun_out/${T}_prof_$xk.log; exit 1; }
    f=$(find gpurun_out/${T}_prof_$xk -name '*kernel_stats.csv' | head -1)
    cp "$f" gpurun_out/${T}_kstats_xk$xk.csv
    rm -rf gpurun_out/${T}_prof_$xk
done
