# round-3 GPU batch: C2 A/B of 2D wavefront knobs under GG_DIV_FMA
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python -u bench.py --cpu-iters 0"
timeout -k 10 200 $B > $O/r03_ab_base.json 2> $O/r03_ab.err &&
GGMRES_LIB=variants/libggmres_lxcd8.so timeout -k 10 200 $B > $O/r03_ab_lxcd8.json 2>> $O/r03_ab.err &&
GGMRES_LIB=variants/libggmres_look2.so timeout -k 10 200 $B > $O/r03_ab_look2.json 2>> $O/r03_ab.err &&
GGMRES_LIB=variants/libggmres_look4.so timeout -k 10 200 $B > $O/r03_ab_look4.json 2>> $O/r03_ab.err &&
timeout -k 10 200 $B > $O/r03_ab_base2.json 2>> $O/r03_ab.err &&
GGMRES_LIB=variants/libggmres_lxcd8.so timeout -k 10 200 $B > $O/r03_ab_lxcd8_2.json 2>> $O/r03_ab.err
