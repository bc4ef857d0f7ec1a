"""GPU parity of the reciprocal-multiply division (gg_set_division(GG_DIV_RCP)).

The reference divides every row of a non-unit triangle by its diagonal
(LUSolve_ignoreZero, src/SpMV_compute.cpp:118-133; HostPrecond_left/right,
src/preconditioner.cu:1094-1137).  GG_DIV_RCP has the wavefront solves compute
x = RN(acc * RN(1/d)) instead (kernels.hip WD_MUL): within about one ulp per
row, so it is a TOLERANCE mode.  Bars:
  * operators: bit-exact against the oracle restated with the same multiply
    (oracle.set_div_mode), and within 1e-13 (relative to the vector) of the
    reference's division;
  * GMRES: bit-identical to the order-matched oracle in the multiply mode, and
    within north_star's 1e-10 (history scale, solution) of the SERIAL oracle
    with the reference's division -- same return code and iteration counts --
    on C1, the other grid matrices, the split (PG) engine, C2's first restart
    cycle and C4's first 12 iterations.
"""
import numpy as np
import pytest

import ggmres
import oracle as O
from ggmres import matrices as M
from helpers import device_layout, make_split, rel_err

pytestmark = pytest.mark.gpu
HIST_RTOL = 1e-10


@pytest.fixture(scope="module")
def solver():
    s = ggmres.Solver(0)
    s.set_division(ggmres.DIV_RCP)
    yield s
    s.close()


def oracle_mul(run, n, nx=None, ny=None, mul=(False, True), layout=None):
    """(serial-order oracle with the reference's division, order-matched oracle
    with the device's division; layout: the solver's own, Solver.layout())"""
    o_serial = run()
    O.set_dot_order(*(layout if layout is not None else device_layout(n, nx, ny)))
    O.set_div_mode(*mul)
    try:
        o_tree = run()
    finally:
        O.set_dot_order(None)
        O.set_div_mode()
    return o_serial, o_tree


def check_tol(g, o):
    assert g["ret"] == o["ret"] and g["iters"] == o["iters"] and g["inner"] == o["inner"]
    h, ho = np.asarray(g["hist"]), np.asarray(o["hist"])
    assert h.shape == ho.shape
    scale = np.max(np.abs(ho))
    assert np.max(np.abs(h - ho)) <= HIST_RTOL * scale, np.max(np.abs(h - ho)) / scale
    assert rel_err(g["x"], o["x"]) <= HIST_RTOL


def check_exact(g, o):
    assert g["ret"] == o["ret"] and g["iters"] == o["iters"] and g["inner"] == o["inner"]
    assert np.array_equal(g["hist"], o["hist"])
    assert np.array_equal(g["x"], o["x"]), rel_err(g["x"], o["x"])


GRIDS = {
    "c1_5pt_100x100": (lambda: M.laplacian_5pt(100), 100, None),
    "5pt_37x64": (lambda: M.laplacian_5pt(37, 64), 37, None),
    "5pt_300x129": (lambda: M.laplacian_5pt(300, 129), 300, None),
    "thermal_7pt_12": (lambda: M.grid_7pt(12), 12, 12),
    "7pt_20x30x7_upwind": (lambda: M.grid_7pt(20, 30, 7, upwind=0.1), 20, 30),
}


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("scale", [1.0, 1e-250, 1e250])
def test_rcp_apply(solver, name, scale):
    make, nx, ny = GRIDS[name]
    A = make()
    L, U = O.ilu0(A)
    y = np.random.default_rng(3).standard_normal(A.shape[0]) * scale
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    assert solver.division_active(0) == ggmres.DIV_EXACT      # unit L: no division
    assert solver.division_active(1) == ggmres.DIV_RCP
    z = solver.precond_apply(ggmres.APPLY_MINV, y)
    O.set_div_mode(False, True)
    try:
        zm = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert np.array_equal(z, zm)
    ze = O.lusolve(L, U, y)
    assert rel_err(z / scale, ze / scale) <= 1e-13      # (scaled: 1e250^2 overflows the norm)


@pytest.mark.parametrize("k", [1, 2])
def test_rcp_skewed_apply(solver, k):
    A = M.laplacian_5pt(100, 70)
    L, U = O.iluk(A, k)
    solver.set_matrix(A)
    solver.set_precond_iluk(k)
    assert solver.uses_wavefront and solver.division_active(1) == ggmres.DIV_RCP
    y = np.random.default_rng(7).standard_normal(A.shape[0])
    O.set_div_mode(False, True)
    try:
        zm = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), zm)


def test_rcp_not_on_dataflow_kernel(solver):
    """other sparsity keeps the reference's division (k_trsv_flow)"""
    A = M.power_law(3000, 33000, seed=7)
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert not solver.uses_wavefront and solver.division_active(1) == ggmres.DIV_EXACT
    y = np.random.default_rng(2).standard_normal(A.shape[0])
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("rhs", ["ones", "uniform"])
def test_rcp_gmres_parity(solver, name, rhs):
    make, nx, ny = GRIDS[name]
    A = make()
    n = A.shape[0]
    b = M.rhs_ones(A) if rhs == "ones" else M.rhs_uniform(n)
    L, U = O.ilu0(A)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=3000, tol=1e-10), n, nx, ny)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=30, max_iter=3000, tol=1e-10)
    check_exact(g, ot)
    check_tol(g, o)


def test_rcp_split_parity(solver):
    """GMRESilu_GPU's split engine: both triangles (Ml's L, diagonal last, and
    Mr's U, diagonal first) are non-unit and take the multiply"""
    A = M.laplacian_5pt(40)
    P = make_split(A, seed=9)
    b = M.rhs_uniform(A.shape[0])
    x0 = np.random.default_rng(3).random(A.shape[0]) * 0.1
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    mul = (solver.division_active(0) == ggmres.DIV_RCP, solver.division_active(1) == ggmres.DIV_RCP)
    o, ot = oracle_mul(lambda: O.gmres_split(A, P, b, x0=x0, m=32, max_iter=2000, tol=1e-11),
                       A.shape[0], mul=mul, layout=solver.layout())
    g = solver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    check_exact(g, ot)
    check_tol(g, o)


def test_rcp_mode_switch_back(solver):
    """GG_DIV_EXACT restores the reference's division bit for bit"""
    A = M.laplacian_5pt(64)
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    y = np.random.default_rng(5).standard_normal(A.shape[0])
    solver.set_division(ggmres.DIV_EXACT)
    try:
        assert solver.division_active(1) == ggmres.DIV_EXACT
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))
    finally:
        solver.set_division(ggmres.DIV_RCP)
    with pytest.raises(ggmres.GGError):
        solver.set_division(7)


@pytest.mark.slow
def test_rcp_c2_first_cycle(solver):
    """C2 (1000 x 1000, ILU(0), GMRES(30)): the first restart cycle"""
    A = M.laplacian_5pt(1000)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300), n, 1000)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=30, max_iter=30, tol=1e-300)
    assert g["iters"] == 30 and g["ret"] == 1
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.slow
def test_rcp_c4_first_iterations(solver):
    """C4 (216^3 7-point, 3D tile wavefront): the first 12 inner iterations"""
    A = M.grid_7pt(216)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=12, tol=1e-300), n, 216, 216)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=30, max_iter=12, tol=1e-300)
    check_exact(g, ot)
    check_tol(g, o)


# ---------------------------------------------------------------- GG_DIV_FMA
# The 2D-grid (unskewed and, round 6, the skewed ILU(k) ones) and 3D-tile
# wavefront solves as fused multiply-adds per row (nearest term first; U's b
# and coefficients pre-scaled by RN(1/d), kernels.hip WD_UFMA / WD_SFMA),
# restated by oracle.set_div_mode(2, 2).  Bars as above:
# bit-exact vs the order-matched restatement, within 1e-10 of the serial oracle
# with the reference's arithmetic.
@pytest.fixture(scope="module")
def fsolver():
    s = ggmres.Solver(0)
    s.set_division(ggmres.DIV_FMA)
    yield s
    s.close()


def modes(s):
    """per-triangle oracle mode (0 divide, 1 multiply, 2 fused) of the active solve"""
    m = {ggmres.DIV_EXACT: 0, ggmres.DIV_RCP: 1, ggmres.DIV_FMA: 2}
    return m[s.division_active(0)], m[s.division_active(1)]


def fused_expected(s):
    """(2, 2) where the triangles take the 2D band or the 3D tile kernel"""
    k0, k1 = s.trsv_kernel(0), s.trsv_kernel(1)
    if k0.startswith("k_trsv_tile3d"):
        assert k0.startswith("k_trsv_tile3d<true, 4,") and k1.startswith("k_trsv_tile3d<false, 5,")
        return True
    if k0.startswith("k_trsv_wave2d_spmv<"):  # the forward solve with the SpMV fused in
        assert k0 == "k_trsv_wave2d_spmv<4>" and k1.startswith("k_trsv_wave2d<false, 5,")
        return True
    if ", false, 1, false>" in k0:          # unskewed 2D band kernel
        assert k0.startswith("k_trsv_wave2d<true, 4,") and k1.startswith("k_trsv_wave2d<false, 5,")
        return True
    return False


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("scale", [1.0, 1e-250, 1e250])
def test_fma_apply(fsolver, name, scale):
    make, nx, ny = GRIDS[name]
    A = make()
    L, U = O.ilu0(A)
    y = np.random.default_rng(3).standard_normal(A.shape[0]) * scale
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    assert fsolver.uses_wavefront
    assert fused_expected(fsolver) and modes(fsolver) == (2, 2)
    z = fsolver.precond_apply(ggmres.APPLY_MINV, y)
    O.set_div_mode(2, 2)
    try:
        zm = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert np.array_equal(z, zm)
    ze = O.lusolve(L, U, y)
    assert rel_err(z / scale, ze / scale) <= 1e-12


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("scale", [1.0, 1e-250, 1e250])
def test_fma_skewed_apply(fsolver, k, scale):
    """ILU(1) / ILU(2) grid factors on the skewed wavefront as fused rows (round
    6): nearest term first -- in-line, the fills nx-2 (k = 2) and nx-1, the line
    term -- bit-exact vs oracle.set_div_mode(2, 2), within 1e-12 of the serial
    oracle"""
    A = M.laplacian_5pt(100, 70)
    L, U = O.iluk(A, k)
    fsolver.set_matrix(A)
    fsolver.set_precond_iluk(k)
    assert fsolver.uses_wavefront and modes(fsolver) == (2, 2)
    assert fsolver.trsv_kernel(0).startswith("k_trsv_wave2d<true, 4,") and f", {k + 1}, false>" in fsolver.trsv_kernel(0)
    y = np.random.default_rng(7).standard_normal(A.shape[0]) * scale
    z = fsolver.precond_apply(ggmres.APPLY_MINV, y)
    O.set_div_mode(2, 2)
    try:
        zm = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert np.array_equal(z, zm)
    assert rel_err(z / scale, O.lusolve(L, U, y) / scale) <= 1e-12


@pytest.mark.parametrize("k", [1, 2])
def test_fma_skewed_gmres_parity(fsolver, k):
    """GMRES(30) with ILU(k) grid factors under GG_DIV_FMA: bit-exact vs the
    order-matched oracle, within the tolerance of the serial one"""
    A = M.laplacian_5pt(90, 77)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.iluk(A, k)
    fsolver.set_matrix(A)
    fsolver.set_precond_iluk(k)
    md = modes(fsolver)
    assert md == (2, 2)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=3000, tol=1e-10), n, mul=md,
                       layout=fsolver.layout())
    g = fsolver.solve(b, restart=30, max_iter=3000, tol=1e-10)
    check_exact(g, ot)
    check_tol(g, o)


def test_fma_fallbacks(fsolver, monkeypatch):
    """GG_FMA_SKEW=0 keeps skewed ILU(1) grids on GG_DIV_RCP's multiply; other
    sparsity: the division"""
    monkeypatch.setenv("GG_FMA_SKEW", "0")
    A = M.laplacian_5pt(100, 70)
    L, U = O.iluk(A, 1)
    fsolver.set_matrix(A)
    fsolver.set_precond_iluk(1)
    monkeypatch.delenv("GG_FMA_SKEW")
    assert fsolver.uses_wavefront and modes(fsolver) == (0, 1)
    y = np.random.default_rng(7).standard_normal(A.shape[0])
    O.set_div_mode(0, 1)
    try:
        zm = O.lusolve(L, U, y)
    finally:
        O.set_div_mode()
    assert np.array_equal(fsolver.precond_apply(ggmres.APPLY_MINV, y), zm)
    A = M.power_law(3000, 33000, seed=7)
    L, U = O.ilu0(A)
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    assert not fsolver.uses_wavefront and modes(fsolver) == (0, 0)
    y = np.random.default_rng(2).standard_normal(3000)
    assert np.array_equal(fsolver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("rhs", ["ones", "uniform"])
def test_fma_gmres_parity(fsolver, name, rhs):
    make, nx, ny = GRIDS[name]
    A = make()
    n = A.shape[0]
    b = M.rhs_ones(A) if rhs == "ones" else M.rhs_uniform(n)
    L, U = O.ilu0(A)
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    md = modes(fsolver)
    assert fused_expected(fsolver) and md == (2, 2)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=3000, tol=1e-10), n, nx, ny, mul=md)
    g = fsolver.solve(b, restart=30, max_iter=3000, tol=1e-10)
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.parametrize("perm", ["random", "identity"])
def test_fma_split_parity(fsolver, perm):
    """GMRESilu_GPU's split engine: with identity permutations both factors are
    grid-shaped (2D wavefront) and both non-unit: Ml's L pre-scaled as a lower
    triangle, Mr's in-line-first U as the canonical one (the fused rows take
    the in-line term first either way); random permutations keep the dataflow
    kernel and the reference's division"""
    A = M.laplacian_5pt(48, 40)
    P = make_split(A, seed=9, identity_perm=perm == "identity")
    b = M.rhs_uniform(A.shape[0])
    x0 = np.random.default_rng(3).random(A.shape[0]) * 0.1
    fsolver.set_matrix(A)
    fsolver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    md = modes(fsolver)
    assert md == ((2, 2) if perm == "identity" else (0, 0))
    if perm == "identity":
        # A' z fused into the L launch where A' has the sliced-ELL copy (not at this size)
        assert fsolver.trsv_kernel(0) in ("k_trsv_wave2d_spmv<5>", "k_trsv_wave2d<true, 5, false, false, 1, false>")
        assert fsolver.trsv_kernel(1).startswith("k_trsv_wave2d<false, 5,")
    o, ot = oracle_mul(lambda: O.gmres_split(A, P, b, x0=x0, m=32, max_iter=2000, tol=1e-11),
                       A.shape[0], nx=48 if perm == "identity" else None, mul=md,
                       layout=None if perm == "identity" else fsolver.layout())
    g = fsolver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.slow
def test_fma_c2_first_cycle(fsolver):
    """C2 (1000 x 1000, ILU(0), GMRES(30)): the first restart cycle"""
    A = M.laplacian_5pt(1000)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    assert modes(fsolver) == (2, 2)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300), n, 1000,
                       mul=(2, 2))
    g = fsolver.solve(b, restart=30, max_iter=30, tol=1e-300)
    assert g["iters"] == 30 and g["ret"] == 1
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.slow
def test_fma_skewed_c2_first_cycle(fsolver):
    """C2 with ILU(1) grid factors (the skewed wavefront's fused rows, round 6):
    the first restart cycle at full size, bit-exact vs the order-matched oracle"""
    A = M.laplacian_5pt(1000)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.iluk(A, 1)
    fsolver.set_matrix(A)
    fsolver.set_precond_iluk(1)
    assert modes(fsolver) == (2, 2) and ", 2, false>" in fsolver.trsv_kernel(1)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300), n, mul=(2, 2),
                       layout=fsolver.layout())
    g = fsolver.solve(b, restart=30, max_iter=30, tol=1e-300)
    assert g["iters"] == 30 and g["ret"] == 1
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.slow
def test_fma_c2_full_solve_tolerance(fsolver):
    """C2 solved to 1e-8 (the bench's tolerance): same return code, iteration
    counts within 1 % of the serial oracle's divide-mode solve is not asserted
    (the serial oracle takes minutes at this size); instead the device's
    GG_DIV_FMA solve is compared with its own GG_DIV_EXACT solve: same
    convergence, histories within 1e-10 over the first 300 iterations"""
    A = M.laplacian_5pt(1000)
    b = M.rhs_ones(A)
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    g = fsolver.solve(b, restart=30, max_iter=20000, tol=1e-8)
    fsolver.set_division(ggmres.DIV_EXACT)
    try:
        e = fsolver.solve(b, restart=30, max_iter=20000, tol=1e-8)
    finally:
        fsolver.set_division(ggmres.DIV_FMA)
    assert g["ret"] == e["ret"] == 0
    assert abs(g["iters"] - e["iters"]) <= 0.01 * e["iters"]
    h, he = np.asarray(g["hist"])[:300], np.asarray(e["hist"])[:300]
    assert np.max(np.abs(h - he)) <= HIST_RTOL * np.max(np.abs(he))
    assert rel_err(g["x"], e["x"]) <= 1e-6      # both stop at relres 1e-8


@pytest.mark.slow
def test_fma_c4_first_iterations(fsolver):
    """C4 (216^3 7-point, 3D tile wavefront): the first 12 inner iterations"""
    A = M.grid_7pt(216)
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    fsolver.set_matrix(A)
    fsolver.set_precond_ilu0()
    assert fused_expected(fsolver) and modes(fsolver) == (2, 2)
    o, ot = oracle_mul(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=12, tol=1e-300), n, 216, 216,
                       mul=(2, 2))
    g = fsolver.solve(b, restart=30, max_iter=12, tol=1e-300)
    check_exact(g, ot)
    check_tol(g, o)


@pytest.mark.parametrize("engine", ["left", "split"])
@pytest.mark.parametrize("shape", [(600, 128), (1000, 192)])
def test_fused_spmv_same_bits(fsolver, monkeypatch, shape, engine):
    """GG_FUSE_SPMV: the inner iteration's A v (split engine: A' z with D_l^-1)
    computed by the forward solve's own launch (extra workgroups, per-band
    counters) gives the bits of the separate k_spmv_sell launch, solve after
    solve (the counters re-arm)"""
    nx, ny = shape
    A = M.laplacian_5pt(nx, ny)
    b = M.rhs_uniform(A.shape[0])
    fsolver.set_matrix(A)
    if engine == "left":
        fsolver.set_precond_ilu0()
    else:
        P = make_split(A, seed=9, identity_perm=True)
        fsolver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    monkeypatch.delenv("GG_FUSE_SPMV", raising=False)
    assert fsolver.trsv_kernel(0) == ("k_trsv_wave2d_spmv<4>" if engine == "left" else "k_trsv_wave2d_spmv<5>")
    g = fsolver.solve(b, restart=30, max_iter=400, tol=1e-12)
    g2 = fsolver.solve(b, restart=30, max_iter=400, tol=1e-12)
    monkeypatch.setenv("GG_FUSE_SPMV", "0")
    assert fsolver.trsv_kernel(0).startswith("k_trsv_wave2d<true, ")
    e = fsolver.solve(b, restart=30, max_iter=400, tol=1e-12)
    for r in (g, g2):
        assert r["ret"] == e["ret"] and r["iters"] == e["iters"] and r["inner"] == e["inner"]
        assert np.array_equal(r["hist"], e["hist"])
        assert np.array_equal(r["x"], e["x"])
