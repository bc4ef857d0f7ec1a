#!/bin/bash
# Round 5 end: where round 4 -> 5's wavefront difference comes from, on ONE box:
# round 4's tree, this round's tree, and this round's tree with round 4's wavefront
# configuration (variant v1: GG_WAVE_NC=1, GG_WAVE_XCD=8, GG_WAVE_LOOK_L=3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
    (cd variants/r04tree && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200) \
        > gpurun_out/r05aj_r04_$rep.json 2> gpurun_out/r05aj_r04_$rep.err || { tail -20 gpurun_out/r05aj_r04_$rep.err; exit 1; }
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200 \
        > gpurun_out/r05aj_r05_$rep.json 2> gpurun_out/r05aj_r05_$rep.err || { tail -20 gpurun_out/r05aj_r05_$rep.err; exit 1; }
    GGMRES_LIB=variants/libggmres_v1.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 \
        --max-iter 1200 > gpurun_out/r05aj_v1_$rep.json 2> gpurun_out/r05aj_v1_$rep.err || { tail -20 gpurun_out/r05aj_v1_$rep.err; exit 1; }
    for t in r04 r05 v1; do
        python3 - gpurun_out/r05aj_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v.get("avg_us") for n, v in k.items()})
PY
    done
done
