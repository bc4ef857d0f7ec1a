"""Pin the fp64 oracle (oracle/) against the reference's own data fixtures and
independent numpy/scipy computations.  CPU only.

The reference ships no GMRES golden vectors; what it does
hold are the cusp Laplacian / random matrices and sherman1 (copied verbatim
into tests/golden/fixtures/) and the SpMV VERIFY criterion (GPU vs CPU SpMV,
relative error < 1e-6 on y = 0.5, src_thermal/main.cu:128-133,263-279).
"""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as sla

import oracle as O
from conftest import FIXTURES, fixture_path
from ggmres import matrices as M
from helpers import csr_sp, make_split, rel_err

LAPLACIANS = ["3pt_100.mtx", "5pt_10x10.mtx", "7pt_10x10x10.mtx", "9pt_10x10.mtx"]
RANDOMS = sorted(glob.glob(os.path.join(FIXTURES, "random_10x10", "*.mtx")))


def load(name):
    if name.endswith(".rua"):
        return M.read_rua(fixture_path(name))
    return M.read_mtx(fixture_path(name) if not os.path.isabs(name) else name)


# ------------------------------------------------------------------ fixtures
def test_generators_match_reference_fixtures():
    assert abs(load("5pt_10x10.mtx") - M.laplacian_5pt(10)).max() == 0
    A7 = M.grid_7pt(10, kx=1, ky=1, kz=1, const_diag=7)
    assert abs(load("7pt_10x10x10.mtx") - A7).max() == 0
    A = load("5pt_10x10.mtx")
    assert A.nnz == 460 and A.shape == (100, 100)


def test_c1_c2_shapes():
    A = M.laplacian_5pt(100)
    assert A.shape[0] == 10_000 and A.nnz == 49_600
    # C2 nnz from the formula 5n - 4*sqrt(n)
    n = 1000
    assert 5 * n * n - 4 * n == 4_996_000


@pytest.mark.parametrize("name", LAPLACIANS + ["sherman1.rua", "test1.rua"] + RANDOMS)
def test_spmv_vs_scipy(name):
    A = load(name)
    n = A.shape[0]
    for x in (np.full(n, 0.5), np.random.default_rng(1).standard_normal(n)):
        y = O.spmv(A, x)
        ref = A @ x
        assert rel_err(y, ref) < 1e-15 or np.allclose(y, ref, rtol=1e-14, atol=1e-300)
    # the reference's VERIFY criterion (src_thermal/main.cu:263-279)
    if n:
        y = O.spmv(A, np.full(n, 0.5))
        assert rel_err(y, A @ np.full(n, 0.5)) < 1e-6


def test_residual_form():
    A = M.laplacian_5pt(12)
    rng = np.random.default_rng(3)
    x, b = rng.random(A.shape[0]), rng.random(A.shape[0])
    assert np.array_equal(O.residual(A, x, b), b - O.spmv(A, x))


# ------------------------------------------------------------------ ILU(0)
def dense_ilu0(A):
    """Independent IKJ ILU(0) on the dense image, restricted to the pattern."""
    A = sp.csr_matrix(A)
    a = A.toarray().astype(np.float64)
    P = np.zeros_like(a, dtype=bool)
    P[A.nonzero()] = True
    n = a.shape[0]
    for i in range(n):
        for k in range(i):
            if not P[i, k]:
                continue
            a[i, k] = a[i, k] / a[k, k]
            cols = np.nonzero(P[i, k + 1:])[0] + k + 1
            a[i, cols] = a[i, cols] - a[i, k] * a[k, cols]
    return a, P


@pytest.mark.parametrize("name", LAPLACIANS + ["sherman1.rua"])
def test_ilu0_matches_dense_ikj(name):
    A = load(name)
    L, U = O.ilu0(A)
    Ld = csr_sp(L).toarray()
    Ud = csr_sp(U).toarray()
    a, P = dense_ilu0(A)
    lower = np.tril(P, -1)
    upper = np.triu(P)
    # values bit-identical (same per-entry operation order), entries < 1e-9 dropped
    ref_l = np.where(lower & (np.abs(a) >= 1e-9), a, 0.0)
    ref_u = np.where(upper & (np.abs(a) >= 1e-9), a, 0.0)
    assert np.array_equal(np.tril(Ld, -1), ref_l)
    assert np.array_equal(Ud, ref_u)
    assert np.all(np.diag(Ld) == 1.0)
    # unit diagonal stored LAST in every L row (splitLU_csr, src/leftILU.cu:508-510)
    for r in range(L.n):
        assert L.ci[L.rp[r + 1] - 1] == r and L.v[L.rp[r + 1] - 1] == 1.0


def test_ilu0_product_on_pattern():
    A = M.laplacian_5pt(20)
    L, U = O.ilu0(A)
    LU = (csr_sp(L) @ csr_sp(U)).toarray()
    Ad = A.toarray()
    P = Ad != 0
    assert np.max(np.abs((LU - Ad)[P])) < 1e-14


def test_lusolve_vs_scipy():
    A = M.laplacian_5pt(15)
    L, U = O.ilu0(A)
    y = np.random.default_rng(0).random(A.shape[0])
    x = O.lusolve(L, U, y)
    t = sla.spsolve_triangular(csr_sp(L), y, lower=True, unit_diagonal=True)
    ref = sla.spsolve_triangular(csr_sp(U), t, lower=False)
    assert rel_err(x, ref) < 1e-14


def test_lusolve_ignores_near_zero_diag():
    # LUSolve_ignoreZero skips a U diagonal with |u| < 1e-9 (src/SpMV_compute.cpp:132-134)
    n = 3
    L = O.csr(sp.identity(n, format="csr"))
    U = O.csr(sp.csr_matrix(np.array([[2.0, 1.0, 0.0], [0.0, 1e-12, 1.0], [0.0, 0.0, 4.0]])))
    x = O.lusolve(L, U, np.array([1.0, 1.0, 8.0]))
    # row 2: 8/4 = 2; row 1: 1 - 1*2 = -1 (no division); row 0: (1 - 1*(-1))/2 = 1
    assert np.array_equal(x, [1.0, -1.0, 2.0])


# ------------------------------------------------------------------ ILU(k)
def test_iluk0_equals_ilu0_pattern_and_values():
    A = load("7pt_10x10x10.mtx")
    L0, U0 = O.ilu0(A)
    Lk, Uk = O.iluk(A, 0)
    assert np.array_equal(L0.rp, Lk.rp) and np.array_equal(L0.ci, Lk.ci)
    assert np.array_equal(U0.rp, Uk.rp) and np.array_equal(U0.ci, Uk.ci)
    # ITSOL scales by the inverted diagonal (iluk.cpp:145) vs leftILU's division
    assert np.max(np.abs(Lk.v - L0.v)) < 1e-15
    assert np.max(np.abs(Uk.v - U0.v)) < 1e-13


@pytest.mark.parametrize("k", [1, 2])
def test_iluk_exact_on_its_pattern(k):
    A = M.laplacian_5pt(12)
    L, U = O.iluk(A, k)
    LU = (csr_sp(L) @ csr_sp(U)).toarray()
    pat = (csr_sp(L) + csr_sp(U)).toarray() != 0
    Ad = A.toarray()
    assert np.max(np.abs((LU - Ad)[pat])) < 1e-13
    # more fill than ILU(0)
    L0, U0 = O.ilu0(A)
    assert L.rp[-1] + U.rp[-1] > L0.rp[-1] + U0.rp[-1]


def test_iluk_zero_pivot_raises():
    A = sp.csr_matrix(np.array([[0.0, 1.0], [1.0, 1.0]]))
    with pytest.raises(ZeroDivisionError):
        O.iluk(A, 1)


# ------------------------------------------------------------------ Givens
@pytest.mark.parametrize("dx,dy", [(3.0, 4.0), (4.0, 3.0), (1.0, 0.0), (-2.0, 5.0), (0.0, 2.0)])
def test_givens(dx, dy):
    cs, sn = O.gen_rot(dx, dy)
    assert abs(cs * cs + sn * sn - 1) < 1e-15
    assert abs(-sn * dx + cs * dy) < 1e-15
    if dy == 0:
        assert (cs, sn) == (1.0, 0.0)


# ------------------------------------------------------------------ split maps
def test_split_maps_inverse_and_dense():
    A = M.laplacian_5pt(9)
    P = make_split(A, seed=3)
    n = A.shape[0]
    v = np.random.default_rng(5).standard_normal(n)
    # Mr^-1(Mr(v)) == v
    assert rel_err(P.start(P.right(v)), v) < 1e-13
    # dense Ml / Mr
    Ld = csr_sp(P.L).toarray()
    Ud = csr_sp(P.U).toarray()
    t = (v / P.lscale)[P.perm_row]
    assert rel_err(P.left(v), np.linalg.solve(Ld, t)) < 1e-13
    w = np.linalg.solve(Ud, v * P.middle)
    assert rel_err(P.right(v), w[P.perm_col] / P.rscale) < 1e-13


# ------------------------------------------------------------------ GMRES
@pytest.mark.parametrize("m", [30, 32])
def test_gmres_left_c1_converges(m):
    A = M.laplacian_5pt(100)
    L, U = O.ilu0(A)
    b = M.rhs_ones(A)
    r = O.gmres_left(A, L, U, b, m=m, max_iter=3000, tol=1e-10)
    assert r["ret"] == 0
    assert r["relres"] < 1e-10
    assert np.max(np.abs(r["x"] - 1.0)) < 1e-6
    h = r["hist"]
    # history: beta0/normb first, then one entry per inner iteration (+1 per restart)
    restarts = (r["inner"] - 1) // m
    assert len(h) == 1 + r["inner"] + restarts
    assert h[-1] == r["relres"]


def test_gmres_left_history_is_true_residual_at_restarts():
    A = M.laplacian_5pt(40)
    L, U = O.ilu0(A)
    b = M.rhs_uniform(A.shape[0])
    m = 10
    r = O.gmres_left(A, L, U, b, m=m, max_iter=m, tol=1e-300)   # exactly one cycle
    assert r["ret"] == 1
    normb = np.linalg.norm(O.lusolve(L, U, b))
    true = np.linalg.norm(O.lusolve(L, U, b - A @ r["x"])) / normb
    h = r["hist"]
    assert len(h) == 1 + m + 1
    assert abs(h[-1] - true) <= 1e-12 * true
    # the Givens estimate of the last inner step equals the restart residual (exact arithmetic)
    assert abs(h[-2] - h[-1]) <= 1e-8 * h[-1]
    # and the reference's exhaustion semantics: *max_iter unchanged, *tol = last resid
    assert r["iters"] == m and r["relres"] == h[-1]


def test_gmres_left_initial_guess_converged():
    A = M.laplacian_5pt(10)
    L, U = O.ilu0(A)
    x0 = np.ones(A.shape[0])
    r = O.gmres_left(A, L, U, A @ x0, x0=x0, m=5, max_iter=50, tol=1e-10)
    assert r["ret"] == 0 and r["iters"] == 0 and r["inner"] == 0 and len(r["hist"]) == 1


def test_gmres_left_zero_rhs():
    A = M.laplacian_5pt(10)
    L, U = O.ilu0(A)
    r = O.gmres_left(A, L, U, np.zeros(A.shape[0]), m=5, max_iter=50, tol=1e-10)
    # normb == 0 -> 1 (src/gmres.cu:604); beta = 0 <= tol
    assert r["ret"] == 0 and r["iters"] == 0 and np.all(r["x"] == 0)


def test_gmres_left_restart_iteration_count_semantics():
    # converging exactly at a restart check reports j = total + 1 (src/gmres.cu:684-688)
    A = M.laplacian_5pt(30)
    L, U = O.ilu0(A)
    b = M.rhs_ones(A)
    full = O.gmres_left(A, L, U, b, m=8, max_iter=5000, tol=1e-10)
    assert full["ret"] == 0
    inner_conv = len(full["hist"]) == 1 + full["inner"] + (full["inner"] - 1) // 8
    if inner_conv:
        assert full["iters"] == full["inner"]


def test_gmres_split_converges_and_matches_scipy():
    A = M.laplacian_5pt(30)
    P = make_split(A, seed=11)
    b = M.rhs_uniform(A.shape[0])
    r = O.gmres_split(A, P, b, m=32, max_iter=2000, tol=1e-12)
    assert r["ret"] == 0
    xs = sla.spsolve(A.tocsc(), b)
    assert rel_err(r["x"], xs) < 1e-9


def test_gmres_split_warm_start():
    A = M.laplacian_5pt(20)
    P = make_split(A, seed=2)
    b = M.rhs_uniform(A.shape[0])
    r1 = O.gmres_split(A, P, b, m=32, max_iter=2000, tol=1e-10)
    r2 = O.gmres_split(A, P, b, x0=r1["x"], m=32, max_iter=2000, tol=1e-10)
    assert r2["ret"] == 0 and r2["iters"] <= 1


def test_pwl_and_dc_semantics():
    """gen_PWLut_kernel (src/kernels.cu:146-176): first point with t < t_i
    interpolates back from it; after the last point its value holds; before t0
    the restatement holds v0 (the reference reads v[-1]). gen_dcVt: constant."""
    h = 1e-9
    tv = [0.0, 0.0, 2e-9, 1.0, 5e-9, 1.0, 6e-9, 0.25]
    assert O.pwl(tv, 0, h) == 1.0 - (2e-9 - 0.0) * (1.0 - 0.0) / (2e-9 - 0.0)       # t = t0: next segment
    assert O.pwl(tv, 1, h) == 1.0 - (2e-9 - 1 * h) * (1.0 - 0.0) / (2e-9 - 0.0)     # rising segment
    assert O.pwl(tv, 3, h) == 1.0 - (5e-9 - 3 * h) * (1.0 - 1.0) / (5e-9 - 2e-9)    # flat
    t = 5 * h
    assert O.pwl(tv, 5, h) == 0.25 - (6e-9 - t) * (0.25 - 1.0) / (6e-9 - 5e-9)       # falling
    assert O.pwl(tv, 9, h) == 0.25                                                    # after the last
    assert O.pwl([1e-9, 0.5, 2e-9, 1.0], 0, h) == 0.5                                 # before t0: v0
    assert O.source_value(O.SRC_DC, [0.7], 123, h) == 0.7
    assert O.source_value(O.SRC_PWL, tv, 1, h) == O.pwl(tv, 1, h)


def test_pulse_semantics():
    """gen_PULSEut_kernel (src/kernels.cu:223-245): periodic trapezoid."""
    q = [0.0, 1e-3, 0.0, 0.1, 0.1, 1.0, 4.0]     # vlo vhi td tr tf tw tp
    h = 0.01
    assert O.pulse(q, 0, h) == 0.0
    assert O.pulse(q, 5, h) == 0.0 + (0.05 - 0.0) * (1e-3 - 0.0) / 0.1      # rising edge
    assert O.pulse(q, 50, h) == 1e-3                                          # high
    t = 115 * h
    assert O.pulse(q, 115, h) == 1e-3 - (t - 0.0 - 0.1 - 1.0) * (1e-3 - 0.0) / 0.1
    assert O.pulse(q, 300, h) == 0.0                                          # low
    assert O.pulse(q, 405, h) == O.pulse(q, 5, h) or abs(O.pulse(q, 405, h) - 5e-4) < 1e-15


def test_transient_rhs_order():
    """w = B u + (C/h) x: sources of a row in ascending k, then + (0 + c x)."""
    n = 6
    src = np.array([4, 1, 4], np.int32)
    u = np.array([1.0, 2.0, 1e-17])
    c = np.full(n, 0.5)
    x = np.arange(n, dtype=np.float64) - 2.0
    w = O.transient_rhs(c, src, u, x)
    ref = np.zeros(n)
    ref[4] = (0.0 + 1.0) + 1e-17
    ref[1] = 2.0
    ref = ref + (0.0 + c * x)
    assert np.array_equal(w, ref)


def test_ilu0_values_split_consistent():
    """orc_ilu0_values (the factored matrix before the split) splits into
    exactly orc_ilu0's L and U (drop |v| < 1e-9, unit diagonal last in L)."""
    for A in (M.laplacian_5pt(12, 9), M.power_law(400, 4000, seed=5), M.grid_7pt(5)):
        A = O.csr(A)
        fv = O.ilu0_values(A)
        L, U = O.ilu0(A)
        lv, uv = [], []
        for r in range(A.n):
            for k in range(A.rp[r], A.rp[r + 1]):
                if abs(fv[k]) < 1e-9:
                    continue
                (lv if A.ci[k] < r else uv).append(fv[k])
            lv.append(1.0)
        assert np.array_equal(np.array(lv), L.v) and np.array_equal(np.array(uv), U.v)


# ---------------------------------------- restated device modes (CPU checks)
@pytest.mark.parametrize("name", ["5pt_10x10.mtx", "7pt_10x10x10.mtx", "sherman1.rua"])
def test_cgs2_restatement_close_to_mgs(name):
    """oracle.set_orth(True) (the sharded solve's GG_SOLVE_CGS2) against the
    reference's MGS: the first restart cycle within 1e-10 of the history scale,
    the Hessenberg columns it builds keep V orthonormal (checked through the
    converged solution: the same iterations +- 1 and the same solution to 1e-9)."""
    A = load(name)
    L, U = O.ilu0(A)
    b = M.rhs_uniform(A.shape[0])
    mgs1 = O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300)
    O.set_orth(True)
    try:
        cgs1 = O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300)
        cgs = O.gmres_left(A, L, U, b, m=30, max_iter=2000, tol=1e-10)
    finally:
        O.set_orth()
    scale = np.max(np.abs(mgs1["hist"]))
    assert np.max(np.abs(cgs1["hist"] - mgs1["hist"])) <= 1e-10 * scale
    mgs = O.gmres_left(A, L, U, b, m=30, max_iter=2000, tol=1e-10)
    assert cgs["ret"] == mgs["ret"] == 0 and abs(cgs["iters"] - mgs["iters"]) <= 1
    assert rel_err(cgs["x"], mgs["x"]) <= 1e-9


def test_div_mode_restatement_within_ulps():
    """oracle.set_div_mode (the device's GG_DIV_RCP, x = acc * RN(1/d)) against
    the reference's division: per solve within a few ulps of the vector"""
    A = load("7pt_10x10x10.mtx")
    L, U = O.ilu0(A)
    y = np.random.default_rng(4).standard_normal(A.shape[0])
    ref = O.lusolve(L, U, y)
    O.set_div_mode(False, True)
    try:
        z = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert not np.array_equal(z, ref)          # it is a different rounding ...
    assert rel_err(z, ref) <= 1e-14            # ... within a few ulps


def test_fma_oracle_differs_from_divide():
    """the restatement is a different rounding, not the reference's bits (so the
    bit-exact checks above do test the fused rows)"""
    A = M.laplacian_5pt(64)
    L, U = O.ilu0(A)
    y = np.random.default_rng(11).standard_normal(A.shape[0])
    O.set_div_mode(2, 2)
    try:
        zf = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    ze = O.lusolve(L, U, y)
    assert not np.array_equal(zf, ze) and rel_err(zf, ze) <= 1e-13
