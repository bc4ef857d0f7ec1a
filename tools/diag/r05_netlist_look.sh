#!/bin/bash
# Round 5: the unit forward solve's look-ahead (GG_WAVE_LOOK_L 4 vs 3) on the netlist
# (unfused, bordered) and C2 (fused), fixed 1,200 iterations, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05ae}
for rep in 1 2; do
    for wl in netlist c2; do
        for v in l4 l3; do
            f=gpurun_out/${T}_${wl}_${v}_$rep
            GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 \
                --cpu-iters 0 --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
            python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
        done
    done
done
