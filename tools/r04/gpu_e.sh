#!/bin/bash
# round 4: dd profiling + bench line; kernel gaps at C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_dd.py tests/test_gpu_bench_ranks.py > gpurun_out/r04e_tests.log 2>&1 || { tail -30 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
timeout -k 10 300 python -u bench.py --workload dd --dd-grid c2 --dd-parts 4 --steps 2 --warmup 2 > gpurun_out/r04e_dd_c2_p4.json 2> gpurun_out/r04e_dd.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r04e_dd_c2_p4.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']); print(d['kernels_per_rank'])"
bash tools/r04/gpu_d.sh
