#!/bin/bash
# Round 5: the split engine's k_mul folded into the persistent MGS (GG_SPLIT_MULFOLD)
# -- the split / border / fast-division GPU suites, then pg and netlist A/B at a
# fixed iteration count, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05w}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_border.py tests/test_gpu_fastdiv.py \
    tests/test_gpu_residency.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
    || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
    for wl in pg netlist; do
        for mf in 1 0; do
            f=gpurun_out/${T}_${wl}_mf${mf}_$rep
            GG_SPLIT_MULFOLD=$mf timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-iters 0 \
                --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
            python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
        done
    done
done
