#!/bin/bash
# Round 5: per-rank timing of the sharded solve -- one shard alone on this GPU
# with loopback exchanges (GG_DD_LOOPBACK), a fixed iteration count, C2 on
# rectangles and C4 on boxes, P = 2 / 4 / 8 (rank 0: it counts the separator
# replica in its dots).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05h}
for g in c2 c4; do
    for P in 2 4 8; do
        f=gpurun_out/${T}_loop_${g}_$P
        timeout -k 10 300 python -u bench.py --workload dd --dd-grid $g --dd-part grid --dd-parts $P --dd-comm loopback \
            --dd-rank 0 --max-iter 300 --steps 2 --warmup 1 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_per_rank"][0]["kernels"]
print(sys.argv[1], d["value"], "it/s;", {n: v["avg_us_per_shard"] for n, v in k.items()}, "xch", d["config"]["exchange_latency"])
PY
    done
done
