#!/bin/bash
# A/B of kernel variants (tools/build_variant.sh) on the C2 bench, one box:
#   tools/diag/variant_sweep.sh TAG NAME...   (NAME "base" = the main library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="variants/libggmres_$v.so"; fi
  GGMRES_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 \
    > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_$v.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$v', d['value'], {n:k[n]['avg_us'] for n in k})"
done
