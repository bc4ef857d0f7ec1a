#!/bin/bash
# Round 5: the persistent MGS's per-step time stamps (GG_MGS_TRACE: the 540th launch,
# C2 inner index 28) on the final tree -- raw lines for tools/diag/mgs_trace_fmt.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
GG_MGS_TRACE=540 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --cpu-iters 0 --no-profile \
    > gpurun_out/r05_mgs_trace.json 2> gpurun_out/r05_mgs_trace.err || { tail -20 gpurun_out/r05_mgs_trace.err; exit 1; }
grep -c mgs_trace gpurun_out/r05_mgs_trace.err
