"""C3 stand-in end to end (GPU): GMRES(30) with ILU(0) or ILU(k) on the seeded
power-law matrix (circuit5M's n and nnz; matrices.power_law), general-sparsity
triangular solves (the sync-free flow kernel).  Prints setup and per-iteration
times.  python tools/c3_solve_probe.py [k] [iters] [scale]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-gmres_amd"))
import numpy as np                      # noqa: E402
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 0
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 60
scale = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
t = time.perf_counter()
A = M.power_law(int(5_558_326 * scale), int(59_524_291 * scale))
print(f"matrix n={A.shape[0]} nnz={A.nnz} built in {time.perf_counter() - t:.1f} s", flush=True)
s = G.Solver(0)
s.set_matrix(A)
t = time.perf_counter()
if k == 0:
    s.set_precond_ilu0_device()
else:
    s.set_precond_iluk_device(k)
print(f"ILU({k}) set up (device numeric) in {time.perf_counter() - t:.1f} s, wavefront={s.uses_wavefront}",
      flush=True)
b = M.rhs_ones(A)
g = s.solve(b, restart=30, max_iter=30, tol=1e-300)       # warm-up cycle
g = s.solve(b, restart=30, max_iter=iters, tol=1e-300)
print(f"GMRES(30) {g['inner']} iterations in {g['solve_ms']:.1f} ms = "
      f"{g['inner'] / g['solve_ms'] * 1e3:.1f} it/s; relres {g['relres']:.3e}", flush=True)
s.profile(True)
g = s.solve(b, restart=30, max_iter=30, tol=1e-300)
for kind, name in ((G.PROF_SPMV, "spmv"), (G.PROF_TRSV_L, "trsv_L"), (G.PROF_TRSV_U, "trsv_U"),
                   (G.PROF_MGS, "mgs")):
    cnt, ms = s.profile_get(kind)
    if cnt:
        print(f"  {name}: {ms * 1e3 / cnt:.1f} us per launch ({cnt})", flush=True)
s.close()
