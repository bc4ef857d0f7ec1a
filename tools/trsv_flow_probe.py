"""Level-path triangular solves on 7-pt grids: dataflow kernel vs one launch per
level (GG_TRSV_LEVELS=1).  python tools/trsv_flow_probe.py grid [grid ...]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-gmres_amd"))
import numpy as np                      # noqa: E402
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

mode = os.environ.get("GG_TRSV_LEVELS", "0")
s = G.Solver()
for grid in [int(a) for a in sys.argv[1:]]:
    A = M.grid_7pt(grid)
    s.set_matrix(A)
    s.set_precond_ilu0()
    t = time.perf_counter()
    ms = s.time_precond(reps=3)
    print(f"levels={mode} grid {grid}: n={A.shape[0]} apply {ms:.3f} ms (wall {time.perf_counter() - t:.2f} s)",
          flush=True)
s.close()
