#!/bin/bash
# Per-rank timing of the sharded solve (GG_DD_LOOPBACK: rank 0's shard alone,
# its exchanges looped back): C2 / C4 at P = 2 / 4 / 8, CGS2 and MGS.
#   tools/diag/dd_loop.sh TAG ["c2 c4"] ["2 4 8"] ["cgs2 mgs"]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
for g in ${2:-c2 c4}; do for P in ${3:-2 4 8}; do for o in ${4:-cgs2 mgs}; do
  timeout -k 10 240 python -u bench.py --workload dd --dd-comm loopback --dd-grid $g --dd-parts $P --dd-orth $o \
      --steps 2 --warmup 1 --cpu-iters 0 > $O/loop_${g}_${P}_$o.json 2> $O/loop_${g}_${P}_$o.err
  python3 -c "
import json; d=json.loads(open('$O/loop_${g}_${P}_$o.json').read().strip().splitlines()[-1])
k=d['kernels_per_rank'][0]['kernels']; print('$g P=$P $o', d['value'], {n: round(v['avg_us_per_shard'],1) for n, v in k.items()})" | tee -a $O/summary.txt
done; done; done
