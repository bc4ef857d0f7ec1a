#!/bin/bash
# D_r^-1 folded into the split engine's SpMV: the suite, an A/B on the netlist
# and the permuted PG split (GG_SPMV_XDIV=1 / 0), then the round's profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash tools/gpu_round.sh r04p tests || exit 1
for wl in "netlist" "pg --pg-perm random"; do
  nm=${wl%% *}
  for e in 1 0; do
    GG_SPMV_XDIV=$e timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-iters 0 \
      > gpurun_out/r04p_${nm}_x$e.json 2> gpurun_out/r04p_${nm}_x$e.err || { tail -20 gpurun_out/r04p_${nm}_x$e.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04p_${nm}_x$e.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$nm xdiv=$e', d['value'], {n:k[n].get('avg_us') for n in k if isinstance(k[n], dict)})"
  done
done
bash tools/gpu_round.sh r04p prof:c2 prof:netlist prof:c4 smoke || exit 1
