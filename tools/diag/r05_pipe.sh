#!/bin/bash
# Round 5: the pipelined restart-cycle loop (GG_CYCLE_PIPE) -- the GPU suite, then
# C2 with and without it, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
    for pipe in 1 0; do
        f=gpurun_out/${T}_c2_pipe${pipe}_$rep
        GG_CYCLE_PIPE=$pipe timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-iters 0 > $f.json 2> $f.err \
            || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["config"]["iters_per_solve"], d["ms_per_step"])
PY
    done
done
