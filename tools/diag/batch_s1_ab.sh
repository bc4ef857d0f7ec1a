set -o pipefail
O=gpurun_out/r06e; mkdir -p $O; export TMPDIR=/tmp
B="python3 -u bench.py --workload c5 --c5-mode batch --c5-scenarios 1 --c5-steps 60 --steps 1 --warmup 0 --cpu-iters 0 --no-profile"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/a -o run -- $B > $O/a.json 2> $O/a.err || exit 1
GG_BATCH_S1_SINGLE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/b -o run -- $B > $O/b.json 2> $O/b.err || exit 1
