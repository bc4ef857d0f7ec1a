#!/bin/bash
# C3 stand-in SpMV: row-tile launch (GG_SPMV_RTILE row blocks) vs panel-major
# launches (GG_SPMV_RTILE=0) at several panel widths; panel + batch GPU tests first
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-rt}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 240 \
    --timeout-method thread -k "panel or edges or bad_arguments" > $O/tests.log 2>&1
tail -1 $O/tests.log
for cfg in "0:786432" "1024:786432" "1024:524288" "1024:262144" "2048:524288" "512:524288"; do
  rt=${cfg%%:*}; w=${cfg#*:}
  GG_SPMV_RTILE=$rt GG_SPMV_PANEL=$w timeout -k 10 200 python3 -u bench.py --workload c3 > $O/c3_${rt}_$w.json 2>> $O/c3.err
  python3 -c "import json;d=json.loads(open('$O/c3_${rt}_$w.json').read().strip().splitlines()[-1]);r=d['roofline'];print('rtile $rt panel $w', d['value'], r['avg_us'], r['frac'])" | tee -a $O/summary.txt
done
