#!/bin/bash
# Round 5: the flow solves' sentinel fills moved into the MGS / SpMV launches (GG_FLOW_FILLFOLD)
# -- the split suites, then permuted-PG A/B at a fixed iteration count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05z}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_border.py tests/test_gpu_fastdiv.py \
    tests/test_abi.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
    || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
    for xd in 1 0; do
        f=gpurun_out/${T}_pgr_ff${xd}_$rep
        GG_FLOW_FILLFOLD=$xd timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --steps 3 --warmup 1 \
            --cpu-iters 0 --tol 1e-30 --max-iter 1200 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("rooflines") or {}
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v["avg_us"] for n, v in r.items()}, "spmv", (k.get("spmv") or {}).get("avg_us"))
PY
    done
done
