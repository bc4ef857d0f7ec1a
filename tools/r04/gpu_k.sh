#!/bin/bash
# round 4: bordered-grid wavefront (netlist) parity + netlist bench, bordered vs flow-only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_border.py \
  > gpurun_out/r04k_border_tests.log 2>&1 || { tail -40 gpurun_out/r04k_border_tests.log; exit 1; }
tail -8 gpurun_out/r04k_border_tests.log
for g in 300 1000; do
  for nb in 0 1; do
    GG_NO_BORDER=$nb timeout -k 10 400 python -u bench.py --workload netlist --grid $g --steps 1 --warmup 1 --cpu-iters 60 \
      > gpurun_out/r04k_netlist_${g}_nb$nb.json 2> gpurun_out/r04k_netlist_${g}_nb$nb.err || { tail -20 gpurun_out/r04k_netlist_${g}_nb$nb.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04k_netlist_${g}_nb$nb.json').read().strip().splitlines()[-1])
k=d['kernels']; c=d['config']; print('netlist $g nb=$nb', d['value'], c['iters_per_solve'], c['relres'], c['netlist'], {n:k[n]['avg_us'] for n in k}); print(d['roofline']); print(d.get('latency_roofline')); print(d['cpu_baseline'])"
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dd.py -k "grid" \
  > gpurun_out/r04k_dd_grid_tests.log 2>&1 || { tail -40 gpurun_out/r04k_dd_grid_tests.log; exit 1; }
tail -4 gpurun_out/r04k_dd_grid_tests.log
for P in 4 8; do
  for part in slabs grid; do
    timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts $P --dd-part $part --steps 2 --warmup 1 \
      > gpurun_out/r04k_dd_${P}_$part.json 2> gpurun_out/r04k_dd_${P}_$part.err || { tail -20 gpurun_out/r04k_dd_${P}_$part.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04k_dd_${P}_$part.json').read().strip().splitlines()[-1])
print('dd P=$P $part', d['value'], d['config'].get('iters_per_solve'), d.get('roofline'), d.get('kernels'))"
  done
done
