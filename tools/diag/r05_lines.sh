#!/bin/bash
# Round 5 end: C5 (1 and 8 scenarios) and C2 with ILU(1)/ILU(2) on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
    local t=$1; shift
    timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r05ap_$t.json 2> gpurun_out/r05ap_$t.err || { tail -20 gpurun_out/r05ap_$t.err; exit 1; }
    python3 - gpurun_out/r05ap_$t.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["config"].get("iters_per_solve"), d["ms_per_step"])
PY
}
run c2_ilu1 --ilu-level 1
run c2_ilu2 --ilu-level 2
run c5 --workload c5
run c5_s8 --workload c5 --c5-scenarios 8
