set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -k "gmres or arnoldi or wide or c4" --timeout 300 --timeout-method thread > $O/r03_leader_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 2 --cpu-iters 0 > $O/r03_ld_c2.json 2> $O/r03_ld.err &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 > $O/r03_ld_c4.json 2>> $O/r03_ld.err
