"""Committed golden vectors (tests/golden/golden.npz, made by
tests/golden/make_golden.py from the oracle on the reference's fixture matrices
and the C1 grid): the oracle must still reproduce them bit for bit, they must
satisfy independent scipy checks, and the device must match them within the
north_star's 1e-10 (GPU)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle as O
from golden.make_golden import CASES, MAX_ITER, M_RESTART, RHS, TOL

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def factors(A):
    return O.ilu0(A)


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_golden(gold, name):
    A = CASES[name]()
    L, U = factors(A)
    assert np.array_equal(L.v, gold[f"{name}/L_v"]) and np.array_equal(U.v, gold[f"{name}/U_v"])
    for rn, rf in RHS.items():
        o = O.gmres_left(A, L, U, rf(A), m=M_RESTART, max_iter=MAX_ITER, tol=TOL)
        key = f"{name}/{rn}"
        assert [o["ret"], o["iters"]] == list(gold[f"{key}/ret_iters"])
        assert np.array_equal(o["hist"], gold[f"{key}/hist"])
        assert np.array_equal(o["x"], gold[f"{key}/x"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_golden_independent_checks(gold, name):
    """scipy, independent of the oracle: L (unit, diagonal last) and U of the
    golden ILU(0) reproduce A on A's pattern; each converged solution's true
    preconditioned residual ||U^-1 L^-1 (b - A x)|| / ||U^-1 L^-1 b|| is at the
    tolerance (the last history entry is GMRES's own estimate of it)."""
    A = CASES[name]().tocsr()
    L, U = factors(A)
    n = A.shape[0]
    Ls = sp.csr_matrix((gold[f"{name}/L_v"], L.ci, L.rp), shape=(n, n))
    Us = sp.csr_matrix((gold[f"{name}/U_v"], U.ci, U.rp), shape=(n, n))
    LU = (Ls @ Us).tocsr()
    pat = A.copy()
    pat.data[:] = 1.0
    diff = (LU - A).multiply(pat)
    assert abs(diff).max() <= 1e-10 * abs(A).max()
    for rn, rf in RHS.items():
        b = rf(A)
        key = f"{name}/{rn}"
        ret, iters = gold[f"{key}/ret_iters"]
        x = gold[f"{key}/x"]
        if ret != 0:
            continue
        pre = lambda v: spla.spsolve_triangular(Us, spla.spsolve_triangular(Ls, v, lower=True),
                                                lower=False)
        rel = np.linalg.norm(pre(b - A @ x)) / np.linalg.norm(pre(b))
        assert rel <= 10 * TOL, (rel, gold[f"{key}/hist"][-1])
        assert abs(rel - gold[f"{key}/hist"][-1]) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("division", ["exact", "fma"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_device_matches_golden(gold, name, division):
    """The device solve against the committed vectors: same return code and
    iteration count, residual history within 1e-10 of its scale, solution
    within 1e-10 relative -- with the reference's division (exact) and with
    the bench's default arithmetic (fma: GG_DIV_FMA's fused rows where the
    wavefront admits them)."""
    import ggmres
    A = CASES[name]()
    s = ggmres.Solver(0)
    try:
        if division == "fma":
            s.set_division(ggmres.DIV_FMA)
        s.set_matrix(A)
        s.set_precond_ilu0()
        for rn, rf in RHS.items():
            g = s.solve(rf(A), restart=M_RESTART, max_iter=MAX_ITER, tol=TOL)
            key = f"{name}/{rn}"
            assert [g["ret"], g["iters"]] == list(gold[f"{key}/ret_iters"])
            h, hg = g["hist"], gold[f"{key}/hist"]
            assert h.shape == hg.shape
            assert np.max(np.abs(h - hg)) <= 1e-10 * np.max(np.abs(hg))
            xg = gold[f"{key}/x"]
            assert np.linalg.norm(g["x"] - xg) <= 1e-10 * np.linalg.norm(xg)
    finally:
        s.close()
