"""Diagnostics: the split engine on grid-shaped factors (wavefront) vs the
order-matched oracle -- first diverging history entry."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gpu-gmres_amd"), os.path.join(REPO, "tests")]
import numpy as np
import ggmres
import oracle as O
from ggmres import matrices as M
from helpers import make_split, device_layout

A = M.laplacian_5pt(48, 40)
n = A.shape[0]
P = make_split(A, seed=9, identity_perm=True)
b = M.rhs_uniform(n)
x0 = np.random.default_rng(3).random(n) * 0.1
wave = os.environ.get("GG_NO_WAVEFRONT") != "1"
lay, G = device_layout(n, 48 if wave else None)
for mi in (3, 31, 32, 33, 40, 64, 80):
    O.set_dot_order(lay, G)
    ot = O.gmres_split(A, P, b, x0=x0, m=32, max_iter=mi, tol=1e-11)
    O.set_dot_order(None)
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    g = s.solve(b, x0=x0, restart=32, max_iter=mi, tol=1e-11)
    s.close()
    h, ho = np.asarray(g["hist"]), np.asarray(ot["hist"])
    k = min(len(h), len(ho))
    d = np.nonzero(h[:k] != ho[:k])[0]
    print(f"max_iter {mi}: wave {wave} len {len(h)}/{len(ho)} first diff {d[:3]} "
          f"x equal {np.array_equal(g['x'], ot['x'])} nan_x {np.isnan(g['x']).sum()} "
          f"h {h[d[0]] if len(d) else None} ho {ho[d[0]] if len(d) else None}", flush=True)
