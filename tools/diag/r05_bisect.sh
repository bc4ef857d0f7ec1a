#!/bin/bash
# Round 5 end: round 4's bench/binding (variants/r04tree) driving the library
# built at successive round-5 commits, on one box (GGMRES_LIB selects it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
    for t in r04 f289add 1814861 head; do
        case $t in
            r04) L=$R/variants/r04tree/gpu-gmres_amd/lib/libggmres.so ;;
            head) L=$R/gpu-gmres_amd/lib/libggmres.so ;;
            *) L=$R/variants/libggmres_$t.so ;;
        esac
        (cd variants/r04tree && GGMRES_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200) \
            > gpurun_out/r05al_${t}_$rep.json 2> gpurun_out/r05al_${t}_$rep.err || { tail -20 gpurun_out/r05al_${t}_$rep.err; exit 1; }
        python3 - gpurun_out/r05al_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v.get("avg_us") for n, v in k.items()})
PY
    done
done
