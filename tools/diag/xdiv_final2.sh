#!/bin/bash
# the gated fold: split-engine tests, the permuted PG and netlist lines, the profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fastdiv.py tests/test_gpu_border.py \
  > gpurun_out/r04q2_tests.log 2>&1 || { tail -40 gpurun_out/r04q2_tests.log; exit 1; }
tail -2 gpurun_out/r04q2_tests.log
for wl in "netlist" "pg --pg-perm random"; do
  nm=${wl%% *}
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-iters 0 \
    > gpurun_out/r04q2_${nm}.json 2> gpurun_out/r04q2_${nm}.err || { tail -20 gpurun_out/r04q2_${nm}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04q2_${nm}.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$nm', d['value'], {n:k[n].get('avg_us') for n in k if isinstance(k[n], dict)})"
done
bash tools/gpu_round.sh r04q2 prof:c2 prof:netlist prof:c4 smoke || exit 1
