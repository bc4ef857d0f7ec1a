#!/bin/bash
# end-of-round: the bench lines, smoke, the default bench line, the GPU suite
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
TAG=${1:-r06F}
bash tools/final_lines.sh $TAG c2 c4 pgr pg netlist c3 c2_ilu1 c5 c5b8 c3s_ilu1 > gpurun_out/${TAG}_lines.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err
