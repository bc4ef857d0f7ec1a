#!/bin/bash
# round 4: MGS prefetch-distance A/B, bordered grids under WD_MUL, DD projections
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_border.py tests/test_gpu_residency.py \
  tests/test_gpu_c2_history.py "tests/test_gpu_parity.py::test_gmres_left_c1_parity" tests/test_gpu_fastdiv.py \
  > gpurun_out/r04q_tests.log 2>&1 || { tail -40 gpurun_out/r04q_tests.log; exit 1; }
tail -3 gpurun_out/r04q_tests.log
for pf in 2 1; do
  GG_MGS_PREFETCH=$pf timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-iters 0 > gpurun_out/r04q_c2_pf$pf.json 2> gpurun_out/r04q_c2_pf$pf.err || { tail -20 gpurun_out/r04q_c2_pf$pf.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04q_c2_pf$pf.json').read().strip().splitlines()[-1])
k=d['kernels']; print('c2 pf=$pf', d['value'], {n:k[n]['avg_us'] for n in k})"
done
timeout -k 10 400 python -u bench.py --workload netlist --steps 3 --warmup 1 --cpu-iters 60 > gpurun_out/r04q_netlist.json 2> gpurun_out/r04q_netlist.err || { tail -20 gpurun_out/r04q_netlist.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04q_netlist.json').read().strip().splitlines()[-1])
k=d['kernels']; print('netlist', d['value'], d['config']['iters_per_solve'], {n:k[n]['avg_us'] for n in k}); print(d['roofline']); print(d.get('latency_roofline'))"
for wl in "c2 grid" "c4 slabs"; do
  set -- $wl
  for P in 2 4 8; do
    timeout -k 10 300 python -u bench.py --workload dd --dd-grid $1 --dd-part $2 --dd-parts $P --steps 1 --warmup 1 \
      > gpurun_out/r04q_dd_$1_$P.json 2> gpurun_out/r04q_dd_$1_$P.err || { tail -20 gpurun_out/r04q_dd_$1_$P.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04q_dd_$1_$P.json').read().strip().splitlines()[-1])
print('dd $1 P=$P', d['value'], d['config'].get('iters_per_solve'), json.dumps(d.get('kernels_per_rank') or d.get('kernels'))[:1500])"
  done
done
