#!/bin/bash
# Round 5: the split engine's D_r^-1 pass folded into the fused SpMV's gathers
# (GG_SPLIT_DIVFOLD) -- the split suites, then PG (grid order) A/B and a C2 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05x}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_border.py tests/test_gpu_fastdiv.py \
    tests/test_gpu_c2_history.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
    || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
    for df in 1 0; do
        f=gpurun_out/${T}_pg_df${df}_$rep
        GG_SPLIT_DIVFOLD=$df timeout -k 10 300 python -u bench.py --workload pg --steps 3 --warmup 1 --cpu-iters 0 \
            --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
    done
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err \
    || { tail -20 gpurun_out/${T}_c2.err; exit 1; }
python3 - gpurun_out/${T}_c2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
print(sys.argv[1], d["value"], {k: v["avg_us"] for k, v in r.items()})
PY
