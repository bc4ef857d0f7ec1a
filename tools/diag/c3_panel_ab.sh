# C3 stand-in SpMV: column-panel widths A/B (one gpurun call)
set -o pipefail
O=gpurun_out/${TAG:-r06l}; mkdir -p $O
for w in ${WIDTHS:-0 393216 262144 131072 65536}; do
  GG_SPMV_PANEL=$w timeout -k 10 200 python3 -u bench.py --workload c3 > $O/c3_$w.json 2>> $O/c3.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_$w.json').read().strip().splitlines()[-1]);r=d['roofline'];print('panel $w', d['value'], r['avg_us'], r['frac'])" | tee -a $O/summary.txt
done
