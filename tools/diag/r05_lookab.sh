#!/bin/bash
# Round 5 end: redundant compute waves forward look-ahead 4 (default) vs 3 and backward XCD spread 4 (default) vs 8 re-measured on
# the per-wave compute loop, C2, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
A="--steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200"
for rep in 1 2; do
    for t in base lookl3 xcd8; do
        L=""; [ $t = base ] || L=variants/libggmres_$t.so
        GGMRES_LIB=$L timeout -k 10 300 python -u bench.py $A \
            > gpurun_out/r05ao_${t}_$rep.json 2> gpurun_out/r05ao_${t}_$rep.err || { tail -20 gpurun_out/r05ao_${t}_$rep.err; exit 1; }
        python3 - gpurun_out/r05ao_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v.get("avg_us") for n, v in k.items() if n in ("trsv_L", "trsv_U", "mgs_givens")})
PY
    done
done
