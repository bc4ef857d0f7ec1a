set -e
mkdir -p gpurun_out/r06p
for nx in 300 600 1000; do
  for v in 1 0; do
    GG_BATCH_MGS2=$v timeout -k 10 120 python -u tools/diag/batch_mgs2_ab.py $nx 8 300 >> gpurun_out/r06p/ab.jsonl
  done
done
