#!/bin/bash
# A/B of the flow kernel's sliced (ELL) term copy: flow-path tests, then the
# randomly permuted PG split and the C3 stand-in solve with GG_FLOW_ELL=1 / 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r04y}
[ -n "$NO_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fastdiv.py tests/test_gpu_border.py tests/test_gpu_dd.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -2 gpurun_out/${T}_tests.log
run() {   # name ell args...
  local nm=$1 e=$2; shift 2
  GG_FLOW_ELL=$e timeout -k 10 300 python -u bench.py "$@" --cpu-iters 0 > gpurun_out/${T}_${nm}_e$e.json 2> gpurun_out/${T}_${nm}_e$e.err \
    || { tail -20 gpurun_out/${T}_${nm}_e$e.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_${nm}_e$e.json').read().strip().splitlines()[-1])
k=d.get('kernels') or {}; print('$nm ell=$e', d['value'], {n:k[n].get('avg_us') for n in k if isinstance(k[n], dict)}, d.get('latency_roofline'))"
}
for e in 1 0; do
  run pgr $e --workload pg --pg-perm random --steps 3 --warmup 1 || exit 1
done
if [ -n "$BPC" ]; then
  for bp in $BPC; do
    GG_FLOW_BPC=$bp run pgr_bpc$bp 1 --workload pg --pg-perm random --steps 3 --warmup 1 || exit 1
  done
fi
if [ -z "$NO_C3" ]; then
  for e in 1 0; do
    run c3s $e --workload c3s --steps 1 --warmup 1 || exit 1
  done
fi
