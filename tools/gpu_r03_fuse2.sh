# fused SpMV, per-group flags: bit-identity test, then the C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastdiv.py -x -v -k "fused or fma_gmres" --timeout 200 --timeout-method thread > $O/fused_tests2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-iters 0 > $O/bench_fused2.json 2> $O/bench_fused2.err
