#!/bin/bash
# round 4: netlist workload (baseline, split engine on the dataflow solves)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for g in 300 1000; do
  timeout -k 10 400 python -u bench.py --workload netlist --grid $g --steps 1 --warmup 1 --cpu-iters 60 \
    > gpurun_out/r04j_netlist_$g.json 2> gpurun_out/r04j_netlist_$g.err || { tail -20 gpurun_out/r04j_netlist_$g.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04j_netlist_$g.json').read().strip().splitlines()[-1])
k=d['kernels']; c=d['config']; print('netlist $g', d['value'], c['iters_per_solve'], c['relres'], c['netlist'], {n:k[n]['avg_us'] for n in k}); print(d['roofline']); print(d['latency_roofline']); print(d['cpu_baseline'])"
done
