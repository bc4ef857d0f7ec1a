# round-3 closing batch, part 1 (fused SpMV kernels): the GPU suite, then the
# C2 profile with PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03_gpu_tests_fused.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03fs c2 > $O/prof_c2.log 2>&1
