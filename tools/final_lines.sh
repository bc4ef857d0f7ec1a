#!/bin/bash
# End-of-round bench lines (PMC traffic from the committed profiles/pmc_traffic*.json):
#   tools/final_lines.sh TAG WL...   -> gpurun_out/TAG/bench_WL.json
# WL: c2 c4 pgr pg netlist c3 c3s_ilu1 c2_ilu1 c5 c5b8 (c5b8: 8 scenarios as one batch)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for wl in "$@"; do
  case $wl in
    c2) ARGS="" ;;
    pgr) ARGS="--workload pg --pg-perm random" ;;
    c2_ilu1) ARGS="--ilu-level 1" ;;
    c3s_ilu1) ARGS="--workload c3s --ilu-level 1" ;;
    c5b8) ARGS="--workload c5 --c5-scenarios 8 --c5-mode batch" ;;
    *) ARGS="--workload $wl" ;;
  esac
  timeout -k 10 400 python -u bench.py $ARGS > $O/bench_$wl.json 2> $O/bench_$wl.err
  python3 -c "
import json; d=json.loads(open('$O/bench_$wl.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$wl', d['value'], d['unit'], r.get('kernel'), r.get('avg_us'), r.get('frac'), r.get('traffic'))"
done
