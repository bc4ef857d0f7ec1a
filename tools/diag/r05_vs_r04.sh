#!/bin/bash
# Round 5 end: round 4's final tree (git archive b43908d, built in variants/r04tree)
# against this round's final tree on ONE box -- the C2 bench line, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$(pwd)
for rep in 1 2 3; do
    (cd variants/r04tree && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0) \
        > gpurun_out/r05ai_r04_$rep.json 2> gpurun_out/r05ai_r04_$rep.err || { tail -20 gpurun_out/r05ai_r04_$rep.err; exit 1; }
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 \
        > gpurun_out/r05ai_r05_$rep.json 2> gpurun_out/r05ai_r05_$rep.err || { tail -20 gpurun_out/r05ai_r05_$rep.err; exit 1; }
    for t in r04 r05; do
        python3 - gpurun_out/r05ai_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], d["ms_per_step"], {n: v.get("avg_us") for n, v in k.items()})
PY
    done
done
