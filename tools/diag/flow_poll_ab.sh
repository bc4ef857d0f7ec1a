#!/bin/bash
# A/B of the flow solve's poll modes (GG_FLOW_POLL builds, tools/build_variant.sh
# with VARDIR=abvar): split-parity GPU tests under each, then per variant the
# permuted-PG (pgr) and C3-stand-in ILU(1) benches and a FETCH_SIZE pass on pgr.
#   tools/diag/flow_poll_ab.sh TAG NAME...    (NAME "base" = the main library)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="$PWD/abvar/libggmres_$v.so"; fi
  export GGMRES_LIB=$lib
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_border.py -x -q --timeout 120 \
      --timeout-method thread -m gpu -k "split or flow or pg or border or iluk" > $OUT/tests_$v.log 2>&1
  tail -1 $OUT/tests_$v.log
  timeout -k 10 200 python -u bench.py --workload pg --pg-perm random --steps 3 --warmup 1 --cpu-iters 0 \
      > $OUT/pgr_$v.json 2> $OUT/pgr_$v.err
  timeout -k 10 300 python -u bench.py --workload c3s --ilu-level 1 --steps 1 --warmup 1 --cpu-iters 0 --max-iter 600 \
      > $OUT/c3s1_$v.json 2> $OUT/c3s1_$v.err
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch_$v -o run -f csv -- \
      python3 -u bench.py --workload pg --pg-perm random --steps 1 --warmup 0 --cpu-iters 0 --no-profile \
      > /dev/null 2> $OUT/fetch_$v.err
  python3 - "$OUT/fetch_$v" "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: [0.0, set()])
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "k_trsv_flow" not in n: continue
    n = n.split("(gg::")[0].replace("void gg::(anonymous namespace)::", "")
    agg[n][0] += float(r["Counter_Value"]); agg[n][1].add(r["Dispatch_Id"])
for n, (v, d) in agg.items():
    print(sys.argv[2], n, "FETCH MB per launch (x2 corrected):", round(2 * v * 1024 / len(d) / 1e6, 1), "launches", len(d))
PY
  rm -rf $OUT/fetch_$v
  for w in pgr c3s1; do python3 -c "
import json; d=json.loads(open('$OUT/${w}_$v.json').read().strip().splitlines()[-1])
k=d.get('kernels',{}); print('$v $w', d['value'], {n:k[n]['avg_us'] for n in k if 'flow' in n or 'spmv' in n})"; done
done
