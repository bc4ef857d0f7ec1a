#!/bin/bash
# Round 5: the flow kernel's s_sleep between poll rounds (GG_FLOW_SLEEP) on the
# randomly permuted PG split -- fixed 1,200 iterations, two runs per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=$1; shift
for rep in 1 2; do
    for v in "$@"; do
        f=gpurun_out/${T}_$v$rep
        GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 240 python -u bench.py --workload pg --pg-perm random \
            --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
    done
done
