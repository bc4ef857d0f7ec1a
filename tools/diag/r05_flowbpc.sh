#!/bin/bash
# Round 5: flow-kernel blocks per CU (GG_FLOW_BPC; unset = the heuristic) on the
# RCM-placed permuted PG split, fixed 1,200 iterations, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05aa}
for rep in 1 2; do
    for b in def 1 2 3 4; do
        f=gpurun_out/${T}_pgr_bpc${b}_$rep
        if [ $b = def ]; then unset GG_FLOW_BPC; else export GG_FLOW_BPC=$b; fi
        timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --steps 3 --warmup 1 \
            --cpu-iters 0 --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {n: v["avg_us"] for n, v in r.items()})
PY
    done
done
