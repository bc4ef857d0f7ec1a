"""Diagnostics: GG_DIV_FMA on the 3D tile wavefront, per triangle (GG_FMA_TILE
bit 0 = L, bit 1 = U), one apply per grid, checked against the oracle's fused rows.
Run one process per mask: GG_FMA_TILE=<mask> python tools/fma_tile_probe.py"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "gpu-gmres_amd")]
import ggmres as G                      # noqa: E402
import oracle as O                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

mask = int(os.environ.get("GG_FMA_TILE", "0"))
for name, A in (("7pt_12", M.grid_7pt(12)), ("7pt_20x30x7_upwind", M.grid_7pt(20, 30, 7, upwind=0.1)),
                ("7pt_40", M.grid_7pt(40))):
    s = G.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.set_division(G.DIV_FMA)
    md = (s.division_active(0), s.division_active(1))
    L, U = O.ilu0(A)
    y = np.random.default_rng(3).standard_normal(A.shape[0])
    try:
        z = s.precond_apply(G.APPLY_MINV, y)
        O.set_div_mode(*md)
        try:
            zm = O.lusolve(L, U, y)
        finally:
            O.set_div_mode()
        print(f"mask {mask} {name}: modes {md} kernels {s.trsv_kernel(0)} / {s.trsv_kernel(1)}: "
              f"bit-exact {np.array_equal(z, zm)}", flush=True)
    except G.GGError as e:
        print(f"mask {mask} {name}: modes {md}: {e}", flush=True)
    s.close()
