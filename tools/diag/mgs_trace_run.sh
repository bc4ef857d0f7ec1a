#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GG_MGS_TRACE=540 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --cpu-iters 0 --no-profile > gpurun_out/r04t_trace.json 2> gpurun_out/r04t_trace.err || { tail -20 gpurun_out/r04t_trace.err; exit 1; }
grep mgs_trace gpurun_out/r04t_trace.err | head -80
