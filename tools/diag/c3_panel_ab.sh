# C3 stand-in SpMV: column-panel widths x library variants A/B (one gpurun call)
#   TAG=.. WIDTHS="w1 w2" LIBS="base name .." bash tools/diag/c3_panel_ab.sh
# (a library NAME is abvar/libggmres_NAME.so, tools/build_variant.sh with VARDIR=abvar)
set -o pipefail
O=gpurun_out/${TAG:-r06l}; mkdir -p $O
for lib in ${LIBS:-base}; do
  if [ "$lib" = base ]; then export GGMRES_LIB=; else export GGMRES_LIB=$PWD/abvar/libggmres_$lib.so; fi
  for w in ${WIDTHS:-0 393216 262144 131072 65536}; do
    GG_SPMV_PANEL=$w timeout -k 10 200 python3 -u bench.py --workload c3 > $O/c3_${lib}_$w.json 2>> $O/c3.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/c3_${lib}_$w.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$lib panel $w', d['value'], r['avg_us'], r['frac'])" | tee -a $O/summary.txt
  done
done
