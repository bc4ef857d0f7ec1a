"""A/B of the batch's persistent orthogonalization: one launch per scenario
(GG_BATCH_MGS2=0) vs one per pair of scenarios (k_arnoldi_persist2, default).

usage: python tools/diag/batch_mgs2_ab.py NX [S] [ITERS]   (run once per env setting)
Prints one JSON line: batched solve time per inner step over S scenarios of a
5-point Laplacian NX x NX with ILU(0), restart 30, a fixed iteration count.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gpu-gmres_amd"))
import ggmres  # noqa: E402
from ggmres import matrices as M  # noqa: E402


def main():
    nx = int(sys.argv[1])
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    it = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    A = M.laplacian_5pt(nx, nx)
    n = A.shape[0]
    rng = np.random.default_rng(1)
    B = rng.standard_normal((S, n))
    X0 = np.zeros((S, n))
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.solve_batch(B, X0, restart=30, max_iter=60, tol=1e-300)        # warm-up (arenas, code objects)
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        g = s.solve_batch(B, X0, restart=30, max_iter=it, tol=1e-300)
        t.append(time.perf_counter() - t0)
    steps = int(sum(g["iters"]))
    print(json.dumps({"nx": nx, "S": S, "mgs2": os.environ.get("GG_BATCH_MGS2", "1"),
                      "us_per_scenario_step": 1e6 * min(t) / steps, "steps": steps}))
    s.close()


if __name__ == "__main__":
    main()
