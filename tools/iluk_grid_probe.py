"""ILU(0) vs ILU(1) vs ILU(2) on a 5-point grid (GPU): the skewed wavefront
(lane skew k+1) against the unskewed ILU(0) one.  Per level: set-up time,
GMRES(30) iterations/s over a fixed run, per-launch kernel times, and the
iterations and milliseconds to a relative residual of 1e-8.
python tools/iluk_grid_probe.py [grid] [fixed_iters]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-gmres_amd"))
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
fixed = int(sys.argv[2]) if len(sys.argv) > 2 else 600
A = M.laplacian_5pt(grid)
b = M.rhs_ones(A)
s = G.Solver(0)
s.set_matrix(A)
for k in (0, 1, 2):
    t = time.perf_counter()
    if k == 0:
        s.set_precond_ilu0_device()
    else:
        s.set_precond_iluk_device(k)
    setup = (time.perf_counter() - t) * 1e3
    s.solve(b, restart=30, max_iter=30, tol=1e-300)           # warm-up
    g = s.solve(b, restart=30, max_iter=fixed, tol=1e-300)
    rate = g["inner"] / g["solve_ms"] * 1e3
    s.profile(True)
    s.solve(b, restart=30, max_iter=30, tol=1e-300)
    parts = []
    for kind, name in ((G.PROF_SPMV, "spmv"), (G.PROF_TRSV_L, "L"), (G.PROF_TRSV_U, "U"),
                       (G.PROF_MGS, "mgs")):
        cnt, ms = s.profile_get(kind)
        if cnt:
            parts.append(f"{name} {ms * 1e3 / cnt:.1f}us")
    s.profile(False)
    c = s.solve(b, restart=30, max_iter=20000, tol=1e-8)
    print(f"ILU({k}) grid {grid}: wavefront={s.uses_wavefront} setup {setup:.0f} ms; "
          f"{rate:.0f} it/s ({', '.join(parts)}); to 1e-8: ret {c['ret']} {c['inner']} it "
          f"in {c['solve_ms']:.0f} ms", flush=True)
s.close()
