#!/bin/bash
# bordered-grid tests + netlist bench (GG_DIV_FMA default) -- one gpurun call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_border.py tests/test_gpu_parity.py \
  > gpurun_out/r04u_tests.log 2>&1 || { tail -40 gpurun_out/r04u_tests.log; exit 1; }
tail -2 gpurun_out/r04u_tests.log
timeout -k 10 300 python -u bench.py --workload netlist --steps 3 --warmup 1 --cpu-iters 0 > gpurun_out/r04u_netlist.json 2> gpurun_out/r04u_netlist.err || { tail -20 gpurun_out/r04u_netlist.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04u_netlist.json').read().strip().splitlines()[-1])
k=d['kernels']; print('netlist', d['value'], d['config']['iters_per_solve'], d['config']['relres'], {n:k[n]['avg_us'] for n in k}); print(d['roofline']); print(d.get('latency_roofline'))"
