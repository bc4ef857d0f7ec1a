# round-3 GPU batch: C2 A/B, the 2D wavefront's early barrier (boundary wave) under GG_DIV_FMA
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python -u bench.py --cpu-iters 0"
timeout -k 10 200 $B > $O/r03_ab2_base.json 2> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_earlybar.so timeout -k 10 200 $B > $O/r03_ab2_earlybar.json 2>> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_lxcd8.so timeout -k 10 200 $B > $O/r03_ab2_lxcd8.json 2>> $O/r03_ab2.err &&
timeout -k 10 200 $B > $O/r03_ab2_base2.json 2>> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_earlybar.so timeout -k 10 200 $B > $O/r03_ab2_earlybar2.json 2>> $O/r03_ab2.err &&
GGMRES_LIB=variants/libggmres_lxcd8.so timeout -k 10 200 $B > $O/r03_ab2_lxcd8_2.json 2>> $O/r03_ab2.err
