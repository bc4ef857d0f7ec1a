"""Generate the committed golden vectors (tests/golden/golden.npz) from the fp64
oracle restatement (oracle/, test infrastructure) on the reference's own fixture
matrices and the C1 grid.

    python tests/golden/make_golden.py

For each case: the ILU(0) factors (leftILU, src/leftILU.cu:27-336), and GMRES
left-ILU(0) (GMRES_leftILU0, src/gmres.cu:566-717) from x0 = 0 with the
reference driver's default right-hand side y = 0.5 (src_thermal/main.cu:128-133)
and with b = A*1 (src/mna_solve_gmres.cpp:302-303): return code, iteration
count, residual history and solution.  tests/test_golden.py checks that the
oracle still reproduces them bit for bit and checks them against scipy
independently; the GPU tests compare the device against the oracle directly.
Serial (reference) summation order.  Stored with numpy.savez (no pickles)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-gmres_amd"))
import oracle as O                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

FIX = os.path.join(HERE, "fixtures")
CASES = {
    "5pt_10x10": lambda: M.read_mtx(os.path.join(FIX, "5pt_10x10.mtx")),
    "7pt_10x10x10": lambda: M.read_mtx(os.path.join(FIX, "7pt_10x10x10.mtx")),
    "9pt_10x10": lambda: M.read_mtx(os.path.join(FIX, "9pt_10x10.mtx")),
    "3pt_100": lambda: M.read_mtx(os.path.join(FIX, "3pt_100.mtx")),
    "sherman1": lambda: M.read_rua(os.path.join(FIX, "sherman1.rua")),
    "c1_5pt_100x100": lambda: M.laplacian_5pt(100),
}
RHS = {"half": lambda A: np.full(A.shape[0], 0.5), "ones": lambda A: M.rhs_ones(A)}
M_RESTART, MAX_ITER, TOL = 32, 2000, 1e-10     # restart = the reference default (src/defs.h:11)


def main():
    out = {}
    for name, mk in CASES.items():
        A = mk()
        L, U = O.ilu0(A)
        out[f"{name}/L_v"] = L.v
        out[f"{name}/U_v"] = U.v
        for rn, rf in RHS.items():
            b = rf(A)
            o = O.gmres_left(A, L, U, b, m=M_RESTART, max_iter=MAX_ITER, tol=TOL)
            key = f"{name}/{rn}"
            out[f"{key}/ret_iters"] = np.array([o["ret"], o["iters"]], np.int64)
            out[f"{key}/hist"] = o["hist"]
            out[f"{key}/x"] = o["x"]
    np.savez(os.path.join(HERE, "golden.npz"), **out)
    print(f"wrote {len(out)} arrays to tests/golden/golden.npz")


if __name__ == "__main__":
    main()
