# round-3 re-entry batch: the GPU suite on the block-sum kernels, then the C2
# profile (bench line, rocprof stats, PMC traffic on the current sources)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03_gpu_tests_bs.log 2>&1 &&
timeout -k 10 600 bash tools/profile_round.sh r03bs c2 > $O/prof_c2.log 2>&1
