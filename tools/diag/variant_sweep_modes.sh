#!/bin/bash
# variants across division modes / workloads: tools/diag/variant_sweep_modes.sh TAG NAME...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="variants/libggmres_$v.so"; fi
  for args in "--division fma" "--division exact" "--workload pg" "--workload netlist"; do
    tagx=$(echo "$args" | tr -d ' -')
    GGMRES_LIB=$lib timeout -k 10 300 python -u bench.py $args --steps 2 --warmup 1 --cpu-iters 0 \
      > gpurun_out/${TAG}_${v}_$tagx.json 2> gpurun_out/${TAG}_${v}_$tagx.err || { tail -20 gpurun_out/${TAG}_${v}_$tagx.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_${v}_$tagx.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$v $tagx', d['value'], {n:k[n]['avg_us'] for n in k if n.startswith('trsv')})"
  done
done
