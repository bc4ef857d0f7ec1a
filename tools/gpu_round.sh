#!/bin/bash
# One gpurun call for a round's GPU work, by stage (run from the repo root):
#   tools/gpu_round.sh TAG STAGE...
# stages:
#   tests           the whole GPU suite (pytest -m gpu), log -> gpurun_out/TAG_tests.log
#   c2 | c4 | netlist | pg
#                   bench.py on that workload -> gpurun_out/TAG_bench_WL.json
#   dd              the sharded solve with local shards: C2 on px x py rectangles, C4 on
#                   px x py x pz boxes, P = 2 / 4 / 8 -> gpurun_out/TAG_dd_{c2,c4}_P.json
#   prof:WL         tools/profile_round.sh TAG WL (rocprofv3 stats + PMC traffic)
#   smoke           __graft_entry__.smoke()
# Every step has its own time limit and the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1
shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
summary() {
    python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(sys.argv[1], d["value"], d["unit"], {n: k[n].get("avg_us") for n in k if isinstance(k[n], dict)})
print("  roofline", d.get("roofline"))
if d.get("latency_roofline"):
    print("  latency", d["latency_roofline"])
EOF
}
for st in "$@"; do
    case $st in
    tests)
        timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
        tail -3 gpurun_out/${TAG}_tests.log ;;
    c2 | c4 | netlist | pg)
        args=""
        [ "$st" = c2 ] || args="--workload $st"
        timeout -k 10 600 python -u bench.py $args > gpurun_out/${TAG}_bench_$st.json 2> gpurun_out/${TAG}_bench_$st.err \
            || { tail -20 gpurun_out/${TAG}_bench_$st.err; exit 1; }
        summary gpurun_out/${TAG}_bench_$st.json ;;
    dd)
        for wl in "c2 grid" "c4 grid"; do
            set -- $wl
            for P in 2 4 8; do
                f=gpurun_out/${TAG}_dd_$1_$P
                timeout -k 10 300 python -u bench.py --workload dd --dd-grid $1 --dd-part $2 --dd-parts $P \
                    --steps 1 --warmup 1 > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
                summary $f.json
            done
        done ;;
    prof:*)
        timeout -k 10 900 bash tools/profile_round.sh $TAG ${st#prof:} || exit 1 ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    *)
        echo "unknown stage $st"; exit 2 ;;
    esac
done
