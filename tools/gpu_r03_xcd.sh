set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python -u bench.py --workload c4 --steps 2"
GG_TILE_XCD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "tile or c4 or 3d" --timeout 300 --timeout-method thread > $O/r03_xcd_tests.log 2>&1 &&
timeout -k 10 300 $B > $O/r03_xcd_r5x0.json 2> $O/r03_xcd.err &&
GG_TILE_XCD=1 timeout -k 10 300 $B > $O/r03_xcd_r5x1.json 2>> $O/r03_xcd.err &&
GGMRES_LIB=variants/libggmres_tring3.so timeout -k 10 300 $B > $O/r03_xcd_r3x0.json 2>> $O/r03_xcd.err &&
GGMRES_LIB=variants/libggmres_tring3.so GG_TILE_XCD=1 timeout -k 10 300 $B > $O/r03_xcd_r3x1.json 2>> $O/r03_xcd.err
