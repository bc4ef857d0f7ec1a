# fused SpMV -> forward solve: bit-identity tests, then C2 bench A/B (fused / separate launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fastdiv.py -x -v --timeout 200 --timeout-method thread > $O/fused_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_fused.json 2> $O/bench_fused.err &&
GG_FUSE_SPMV=0 timeout -k 10 300 python -u bench.py > $O/bench_unfused.json 2> $O/bench_unfused.err
