#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_border.py \
  > gpurun_out/r04x_tests.log 2>&1 || { tail -40 gpurun_out/r04x_tests.log; exit 1; }
tail -2 gpurun_out/r04x_tests.log
for ts in 1 0; do
  GG_TAIL_SMALL=$ts timeout -k 10 300 python -u bench.py --workload netlist --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/r04x_netlist_ts$ts.json 2> gpurun_out/r04x_netlist_ts$ts.err || { tail -20 gpurun_out/r04x_netlist_ts$ts.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04x_netlist_ts$ts.json').read().strip().splitlines()[-1])
k=d['kernels']; print('netlist ts=$ts', d['value'], {n:k[n]['avg_us'] for n in k})"
done
