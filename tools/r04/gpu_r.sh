#!/bin/bash
# round 4: narrow-level flow solves on one XCD (GG_FLOW_XCD) -- parity subset + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_border.py \
  tests/test_gpu_dd.py > gpurun_out/r04r_tests.log 2>&1 || { tail -40 gpurun_out/r04r_tests.log; exit 1; }
tail -2 gpurun_out/r04r_tests.log
for fx in 1 0; do
  GG_FLOW_XCD=$fx timeout -k 10 300 python -u bench.py --workload pg --pg-perm random --steps 1 --warmup 1 --cpu-iters 0 --max-iter 600 \
    > gpurun_out/r04r_pgr_fx$fx.json 2> gpurun_out/r04r_pgr_fx$fx.err || { tail -20 gpurun_out/r04r_pgr_fx$fx.err; exit 1; }
  GG_NO_BORDER=1 GG_FLOW_XCD=$fx timeout -k 10 300 python -u bench.py --workload netlist --grid 300 --steps 1 --warmup 1 --cpu-iters 0 \
    > gpurun_out/r04r_net300_fx$fx.json 2> gpurun_out/r04r_net300_fx$fx.err || { tail -20 gpurun_out/r04r_net300_fx$fx.err; exit 1; }
  for f in pgr net300; do
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04r_${f}_fx$fx.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$f fx=$fx', d['value'], {n:k[n]['avg_us'] for n in k}, d.get('latency_roofline'))"
  done
done
for P in 4 8; do
  timeout -k 10 300 python -u bench.py --workload dd --dd-grid c4 --dd-part grid --dd-parts $P --steps 1 --warmup 1 \
    > gpurun_out/r04r_dd_c4grid_$P.json 2> gpurun_out/r04r_dd_c4grid_$P.err || { tail -20 gpurun_out/r04r_dd_c4grid_$P.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04r_dd_c4grid_$P.json').read().strip().splitlines()[-1])
print('dd c4 grid P=$P', d['value'], d['config'].get('iters_per_solve'), json.dumps(d.get('kernels_per_rank'))[:900])"
done
timeout -k 10 300 python -u bench.py --workload netlist --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/r04r_netlist.json 2> gpurun_out/r04r_netlist.err || { tail -20 gpurun_out/r04r_netlist.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04r_netlist.json').read().strip().splitlines()[-1])
k=d['kernels']; print('netlist', d['value'], {n:k[n]['avg_us'] for n in k})"
