#!/bin/bash
# round 4: flow-kernel grid size on the randomly permuted PG split (GG_FLOW_BPC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for bpc in 1 2 4 8; do
  GG_FLOW_BPC=$bpc timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --steps 1 --warmup 1 --cpu-iters 0 --max-iter 600 \
    > gpurun_out/r04s_pgr_bpc$bpc.json 2> gpurun_out/r04s_pgr_bpc$bpc.err || { tail -20 gpurun_out/r04s_pgr_bpc$bpc.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04s_pgr_bpc$bpc.json').read().strip().splitlines()[-1])
k=d['kernels']; print('pgr bpc=$bpc', d['value'], {n:k[n]['avg_us'] for n in k}, d['config'].get('iters_per_solve'))"
done
