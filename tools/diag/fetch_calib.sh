#!/bin/bash
# FETCH_SIZE calibration (tools/fetch_calib.hip; build it on the CPU side first)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fcal}; mkdir -p $OUT
timeout -k 10 60 ./tools/fetch_calib > $OUT/plain.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -f csv -- ./tools/fetch_calib > $OUT/run.txt 2> $OUT/fetch.err
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $OUT/req -o run -f csv -- ./tools/fetch_calib > /dev/null 2> $OUT/req.err
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
python3 - $OUT <<'PY'
import csv, glob, sys
out = sys.argv[1]
for sub in ("fetch", "req"):
    for f in glob.glob(out + "/" + sub + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(sub, r["Dispatch_Id"], r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"], r["Counter_Value"])
PY
rm -rf $OUT/fetch $OUT/req
