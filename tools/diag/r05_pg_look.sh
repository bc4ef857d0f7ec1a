#!/bin/bash
# Round 5: look-ahead 4 for the split engine's fused (non-unit) forward solve too
# (variant fsall) vs the default (base: unit fused L only) -- PG on the C2 grid,
# the split parity tests for the variant first, fixed 1,200 iterations, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05af}
GGMRES_LIB=variants/libggmres_fsall.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k split \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
    for v in fsall base; do
        f=gpurun_out/${T}_pg_${v}_$rep
        GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 300 python -u bench.py --workload pg --steps 3 --warmup 1 \
            --cpu-iters 0 --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
    done
done
