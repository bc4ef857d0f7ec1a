#!/bin/bash
# Round 5 end: compute-wave loop specialised per wave (compile-time staging
# share) against the run-time wave test (libggmres_pre) and round 4's tree, one
# box; then the C2 history / wavefront parity tests on the new library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
A="--steps 3 --warmup 1 --cpu-iters 0 --tol 1e-30 --max-iter 1200"
for rep in 1 2; do
    (cd variants/r04tree && timeout -k 10 300 python -u bench.py $A) \
        > gpurun_out/r05am_r04_$rep.json 2> gpurun_out/r05am_r04_$rep.err || { tail -20 gpurun_out/r05am_r04_$rep.err; exit 1; }
    GGMRES_LIB=variants/libggmres_pre.so timeout -k 10 300 python -u bench.py $A \
        > gpurun_out/r05am_pre_$rep.json 2> gpurun_out/r05am_pre_$rep.err || { tail -20 gpurun_out/r05am_pre_$rep.err; exit 1; }
    timeout -k 10 300 python -u bench.py $A \
        > gpurun_out/r05am_new_$rep.json 2> gpurun_out/r05am_new_$rep.err || { tail -20 gpurun_out/r05am_new_$rep.err; exit 1; }
    for t in r04 pre new; do
        python3 - gpurun_out/r05am_${t}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], {n: v.get("avg_us") for n, v in k.items() if n in ("trsv_L", "trsv_U", "mgs_givens")})
PY
    done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_c2_history.py tests/test_gpu_parity.py > gpurun_out/r05am_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05am_tests.log
exit $rc
