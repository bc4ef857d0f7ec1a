# round-3: plane-skew-1 tile wavefront -- bit-exactness on the 3D cases, C4 bench, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastdiv.py -x -q -k "tile or 3d or 7pt or c4 or wave3" --timeout 250 --timeout-method thread > $O/r03_tile_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k "c4_single" --timeout 250 --timeout-method thread >> $O/r03_tile_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_c4_skew1.json 2> $O/r03_c4.err &&
timeout -k 10 200 python -u tools/tile_trace.py > $O/r03_tile_trace_c4.txt 2>&1
