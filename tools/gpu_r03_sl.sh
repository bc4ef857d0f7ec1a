set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
D="python -u bench.py --workload dd --dd-grid c2 --steps 1 --warmup 1 --dd-parts 4"
timeout -k 10 300 $D > $O/r03_sl_4.json 2> $O/r03_sl.err &&
GGMRES_LIB=variants/libggmres_sl16.so timeout -k 10 300 $D > $O/r03_sl_16.json 2>> $O/r03_sl.err &&
GGMRES_LIB=variants/libggmres_sl1.so timeout -k 10 300 $D > $O/r03_sl_1.json 2>> $O/r03_sl.err &&
timeout -k 10 300 $D > $O/r03_sl_4b.json 2>> $O/r03_sl.err
