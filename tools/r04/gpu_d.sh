#!/bin/bash
# round 4: kernel gaps at C2 (kernel trace, no events)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04d/tr -o run -f csv -- \
    python3 -u bench.py --steps 1 --warmup 1 --cpu-iters 0 --max-iter 600 --no-profile > gpurun_out/r04d/b.json 2> gpurun_out/r04d/b.err || exit 1
f=$(find gpurun_out/r04d/tr -name "*kernel_trace.csv" | head -1)
python3 tools/gap_report.py $f > gpurun_out/r04d/gaps.txt
python3 - "$f" > gpurun_out/r04d/seq.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-200:]
prev = None
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0][-40:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{n:40s} dur {(e-s)/1e3:8.2f} gap {((s-prev)/1e3 if prev else 0):7.2f}")
    prev = e
PY
rm -rf gpurun_out/r04d/tr
cat gpurun_out/r04d/gaps.txt
