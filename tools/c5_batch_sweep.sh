#!/bin/bash
# C5 many-RHS batch: rocprof kernel summary + knob sweep (one gpurun call).
#   bash tools/c5_batch_sweep.sh TAG [STEPS]
set -o pipefail
TAG=${1:-c5sweep}; ST=${2:-300}
O=gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 -u bench.py --workload c5 --c5-steps $ST --steps 1 --warmup 1 --cpu-iters 0 --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- $B --c5-scenarios 8 > $O/prof_line.json 2> $O/prof.err || exit 1
for v in "S=8" "S=8 GG_BATCH_ZMAP=1" "S=8 GG_BATCH_CHUNK=2" "S=8 GG_BATCH_CHUNK=5" "S=4" "S=16" "S=1"; do
  S=${v%% *}; S=${S#S=}; E=${v#S=$S}; t=$(echo "s$S$E" | tr ' =' '_-')
  env $E timeout -k 10 300 $B --c5-scenarios $S > $O/$t.json 2> $O/$t.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/$t.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])" | tee -a $O/summary.txt
done
