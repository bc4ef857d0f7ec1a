# A/B of tile-kernel build variants at C4 (each line: bench json)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 --cpu-iters 0 > $O/r03_c4_base.json 2> $O/r03_c4ab.err &&
GGMRES_LIB=variants/libggmres_tb4.so timeout -k 10 300 python -u bench.py --workload c4 --steps 2 --cpu-iters 0 > $O/r03_c4_tb4.json 2>> $O/r03_c4ab.err &&
timeout -k 10 300 python -u bench.py --workload c4 --steps 2 --cpu-iters 0 > $O/r03_c4_base2.json 2>> $O/r03_c4ab.err
