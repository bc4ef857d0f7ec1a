#!/bin/bash
# A/B of the wavefront solve's x staging (round 5): variants/libggmres_<v>.so
# for each v given -- C2 full-history parity (bit-exact), then C2 at a fixed
# iteration count twice, plus the wave trace.
#   tools/diag/r05_stage_ab.sh TAG v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=$1; shift
for v in "$@"; do
    if [ "$v" != nostage ]; then
        GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_history.py -x -q \
            --timeout 240 --timeout-method thread > gpurun_out/${T}_hist_$v.log 2>&1 || { tail -30 gpurun_out/${T}_hist_$v.log; exit 1; }
        echo "$v: $(tail -1 gpurun_out/${T}_hist_$v.log)"
    fi
    for rep in 1 2; do
        GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 \
            --tol 1e-30 --max-iter 1200 > gpurun_out/${T}_$v$rep.json 2> gpurun_out/${T}_$v$rep.err || { tail -20 gpurun_out/${T}_$v$rep.err; exit 1; }
        python3 - gpurun_out/${T}_$v$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
    done
    [ "${TRACE:-1}" = 1 ] || continue
    GGMRES_LIB=variants/libggmres_$v.so timeout -k 10 120 python -u tools/wave_trace.py > gpurun_out/${T}_trace_$v.txt 2>&1 || { tail -20 gpurun_out/${T}_trace_$v.txt; exit 1; }
    grep -E "total|phase|publish|seen" gpurun_out/${T}_trace_$v.txt
done
