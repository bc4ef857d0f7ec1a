#!/bin/bash
# Round 5 end: round 4's bench/binding with round 4's library (r04tree) against
# round 4's bench/binding with THIS round's library (r04mix) on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
    for t in r04tree r04mix; do
        (cd variants/$t && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200) \
            > gpurun_out/r05ak_${t}_$rep.json 2> gpurun_out/r05ak_${t}_$rep.err || { tail -20 gpurun_out/r05ak_${t}_$rep.err; exit 1; }
        python3 - gpurun_out/r05ak_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v.get("avg_us") for n, v in k.items()})
PY
    done
done
