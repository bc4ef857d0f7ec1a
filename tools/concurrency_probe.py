"""Aggregate GMRES throughput of S independent systems solved concurrently on
one GPU (one solver object, HIP stream and host thread each): the wavefront
triangular solves occupy 16 CUs per system, so S systems can overlap them.
python tools/concurrency_probe.py [grid] [iters] [S ...]
Prints per S: aggregate inner iterations / wall second."""
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-gmres_amd"))
import numpy as np                      # noqa: E402
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

grid = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 600
Ss = [int(a) for a in sys.argv[3:]] or [1, 2, 4, 8]
A = M.laplacian_5pt(grid)
solvers = []
for k in range(max(Ss)):
    s = G.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    solvers.append(s)
bs = [M.rhs_uniform(A.shape[0], seed=100 + k) for k in range(max(Ss))]
for s, b in zip(solvers, bs):
    s.solve(b, restart=30, max_iter=60, tol=1e-300)      # warm-up
for S in Ss:
    out = [None] * S

    def run(k):
        out[k] = solvers[k].solve(bs[k], restart=30, max_iter=iters, tol=1e-300)

    th = [threading.Thread(target=run, args=(k,)) for k in range(S)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    tot = sum(o["inner"] for o in out)
    print(f"S={S} persist={os.environ.get('GG_NO_PERSIST') != '1'}: {tot} iterations in {el:.3f} s "
          f"= {tot / el:.1f} it/s aggregate ({tot / el / S:.1f} per system)", flush=True)
for s in solvers:
    s.close()
