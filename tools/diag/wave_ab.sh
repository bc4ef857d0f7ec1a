#!/bin/bash
# A/B of wavefront kernel variants (abvar/ builds) on the C2 bench, alternating
# base / variant twice on one box, after the C2 history bit-exact test under
# each variant:  tools/diag/wave_ab.sh TAG NAME...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  GGMRES_LIB=$PWD/abvar/libggmres_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_history.py -x -q \
      --timeout 240 --timeout-method thread > $O/hist_$v.log 2>&1
  echo "$v history: $(tail -1 $O/hist_$v.log)"
done
for rep in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/abvar/libggmres_$v.so"; fi
    GGMRES_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 \
        > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    python3 -c "
import json; d=json.loads(open('$O/c2_${v}_$rep.json').read().strip().splitlines()[-1])
k=d['kernels']; print('$v', $rep, d['value'], {n: k[n]['avg_us'] for n in k})" | tee -a $O/summary.txt
  done
done
