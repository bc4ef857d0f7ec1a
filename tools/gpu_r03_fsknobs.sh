# fused SpMV knobs A/B at C2: slice-group size and SpMV block count (variants/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
B="python -u bench.py --steps 3 --warmup 1 --cpu-iters 0"
timeout -k 10 120 $B > $O/fs_base.json 2> $O/fs_base.err &&
GGMRES_LIB=variants/libggmres_fsg2.so timeout -k 10 120 $B > $O/fs_g2.json 2> $O/fs_g2.err &&
GGMRES_LIB=variants/libggmres_fsg8.so timeout -k 10 120 $B > $O/fs_g8.json 2> $O/fs_g8.err &&
GGMRES_LIB=variants/libggmres_fsb128.so timeout -k 10 120 $B > $O/fs_b128.json 2> $O/fs_b128.err &&
GGMRES_LIB=variants/libggmres_fsb480.so timeout -k 10 120 $B > $O/fs_b480.json 2> $O/fs_b480.err &&
timeout -k 10 120 $B > $O/fs_base2.json 2> $O/fs_base2.err
