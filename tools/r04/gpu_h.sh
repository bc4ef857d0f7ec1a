#!/bin/bash
# round 4: C4 A/B -- tile queue vs static, after the wide-kernel spill fix
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for st in 0 1; do
    GG_TILE_STATIC=$st timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-iters 0 \
      > gpurun_out/r04h_c4_st${st}_r$r.json 2> /dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04h_c4_st${st}_r$r.json').read().strip().splitlines()[-1])
k=d['kernels']; print('C4 static=$st run $r', d['value'], {n:k[n]['avg_us'] for n in k})"
  done
done
