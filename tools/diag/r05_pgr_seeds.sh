#!/bin/bash
# Round 5: iterations to 1e-8 of the randomly permuted PG split in the natural and
# the RCM layout, for three seeds (the reduction order's effect on GMRES(30))
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r05l}
for seed in 1 2 3; do
    for rcm in 1 0; do
        f=gpurun_out/${T}_pgr_s${seed}_rcm$rcm
        GG_FLOW_RCM=$rcm timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --pg-seed $seed \
            --steps 1 --warmup 1 --cpu-iters 0 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
        python3 - $f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], "it/s", d["config"]["iters_per_solve"], "iterations", d["ms_per_step"], "ms/solve")
PY
    done
done
