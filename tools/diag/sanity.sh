#!/bin/bash
# quick end-of-round sanity on the in-tree library: smoke, batch + C2 history tests, the default line
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
T=${1:-sanity}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_c2_history.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err
