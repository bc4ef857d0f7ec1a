#!/bin/bash
# C5 many-RHS batch: FETCH_SIZE per launch of the batched kernels at S = 1 / 8 (and zmap 1)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-c5pmc}; mkdir -p $O
for item in 1 8 8:GG_BATCH_ZMAP=1; do
  S=${item%%:*}; E=""; [ "$item" != "$S" ] && E=${item#*:}
  t=$(echo "s$S${E:+_$E}" | tr '=' '-')
  env $E timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/$t -o run -f csv -- python3 -u bench.py \
      --workload c5 --c5-mode batch --c5-scenarios $S --c5-steps 20 --steps 1 --warmup 0 --cpu-iters 0 --no-profile \
      > $O/$t.json 2> $O/$t.err
  python3 - "$O/$t" "$t" <<'PY' | tee -a $O/summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: [0.0, set()])
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(gg::")[0].replace("void gg::(anonymous namespace)::", "")
    agg[n][0] += float(r["Counter_Value"]); agg[n][1].add(r["Dispatch_Id"])
for n, (v, d) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:8]:
    print(sys.argv[2], n[:60], "MB/launch", round(2 * v * 1024 / len(d) / 1e6, 2), "launches", len(d))
PY
  rm -rf $O/$t
done
