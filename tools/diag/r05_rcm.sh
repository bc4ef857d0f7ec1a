#!/bin/bash
# Round 5: the split engine's flow path in an RCM layout -- parity tests, then
# the randomly permuted PG split (bench --workload pg --pg-perm random) with the
# RCM layout and with the natural one (GG_FLOW_RCM=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastdiv.py tests/test_gpu_border.py \
    tests/test_gpu_boundary.py -k "split or border or pg_classes" -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for rcm in 1 0; do
    GG_FLOW_RCM=$rcm timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --steps 3 --warmup 1 \
        --cpu-iters 0 > gpurun_out/${T}_pgr_rcm$rcm.json 2> gpurun_out/${T}_pgr_rcm$rcm.err || { tail -20 gpurun_out/${T}_pgr_rcm$rcm.err; exit 1; }
    python3 - gpurun_out/${T}_pgr_rcm$rcm.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["config"]["iters_per_solve"], {k: v.get("avg_us") for k, v in d["kernels"].items()})
PY
done
