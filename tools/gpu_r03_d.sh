# round-3 GPU batch: GG_DIV_FMA on the 3D tiles, per triangle (diagnostics)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
GG_FMA_TILE=1 timeout -k 10 120 python -u tools/fma_tile_probe.py > $O/r03_fma_tile_probe.txt 2>&1 &&
GG_FMA_TILE=2 timeout -k 10 120 python -u tools/fma_tile_probe.py >> $O/r03_fma_tile_probe.txt 2>&1
