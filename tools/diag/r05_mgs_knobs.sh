#!/bin/bash
# Round 5: the persistent MGS's runtime knobs re-checked after the DPP wave sums --
# GG_MGS_GATHER (0 every block gathers, 2 XCD-local reducers = default, 3 reducer-only
# blocks) x GG_MGS_PREFETCH (1 default, 0); C2 at a fixed iteration count, two runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05ac}
for rep in 1 2; do
    for v in "2 1" "0 1" "3 1" "2 0"; do
        set -- $v
        f=gpurun_out/${T}_g$1p$2_$rep
        GG_MGS_GATHER=$1 GG_MGS_PREFETCH=$2 timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 \
            --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
    done
done
