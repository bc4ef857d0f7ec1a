"""GPU parity: the HIP kernels (through the C ABI) against the fp64 oracle.

Bars (DESIGN.md "Parity"):
  * SpMV, triangular solves, split preconditioner maps: bit-exact (same
    per-row operation order, contraction off);
  * GMRES residual history and solution: within 1e-10 relative per entry
    (north_star), identical iteration counts and return codes.
"""
import glob
import os

import numpy as np
import pytest

import ggmres
import oracle as O
from conftest import fixture_path
from ggmres import matrices as M
from helpers import device_layout, hist_close, make_split, rel_err

pytestmark = pytest.mark.gpu
HIST_RTOL = 1e-10


@pytest.fixture(scope="module")
def solver():
    s = ggmres.Solver(0)
    yield s
    s.close()


def load(name):
    return M.read_rua(fixture_path(name)) if name.endswith(".rua") else M.read_mtx(fixture_path(name))


MATS = {
    "c1_5pt_100x100": lambda: M.laplacian_5pt(100),
    "5pt_37x64": lambda: M.laplacian_5pt(37, 64),
    "5pt_10x10": lambda: load("5pt_10x10.mtx"),
    "7pt_10x10x10": lambda: load("7pt_10x10x10.mtx"),
    "9pt_10x10": lambda: load("9pt_10x10.mtx"),
    "3pt_100": lambda: load("3pt_100.mtx"),
    "sherman1": lambda: load("sherman1.rua"),
    "thermal_7pt_12": lambda: M.grid_7pt(12),
    "powerlaw_3000": lambda: M.power_law(3000, 33000, seed=7),    # C3 stand-in, small
}
# wavefront path: 2D grids (line length) and 3D grids (line length, lines per plane)
GRID = {"c1_5pt_100x100": (100, None), "5pt_37x64": (37, None), "7pt_10x10x10": (10, 10),
        "thermal_7pt_12": (12, 12), "sherman1": (10, 10)}
WAVE = set(GRID)


@pytest.mark.parametrize("name", sorted(MATS))
def test_spmv_bitexact(solver, name):
    A = MATS[name]()
    x = np.random.default_rng(1).standard_normal(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_none()
    assert np.array_equal(solver.spmv(x), O.spmv(A, x))
    solver.set_precond_ilu0()   # wavefront layout where it applies
    assert solver.uses_wavefront == (name in WAVE)
    assert np.array_equal(solver.spmv(x), O.spmv(A, x))


RANDOMS = sorted(os.path.basename(f) for f in glob.glob(fixture_path(os.path.join("random_10x10", "*.mtx"))))


@pytest.mark.parametrize("name", RANDOMS)
def test_spmv_random_fixtures(solver, name):
    """The cusp random_10x10 fixtures (0-100 nonzeros, empty rows and an empty
    matrix): SpMV bit-exact vs the oracle, with x random and the reference
    driver's default y = 0.5 input (src_thermal/main.cu:128-133)."""
    A = load(os.path.join("random_10x10", name))
    solver.set_matrix(A)
    solver.set_precond_none()
    for x in (np.random.default_rng(7).standard_normal(A.shape[0]), np.full(A.shape[0], 0.5)):
        assert np.array_equal(solver.spmv(x), O.spmv(A, x))


@pytest.mark.parametrize("name", ["5pt_10x10", "7pt_10x10x10", "9pt_10x10", "3pt_100"])
def test_gmres_driver_default_rhs(solver, name):
    """The reference driver's CPU-vs-GPU GMRES check (src_thermal/main.cu:459-527)
    on its fixtures with its default right-hand side y = 0.5: bit-identical to
    the order-matched oracle, within 1e-10 of the serial one."""
    A = MATS[name]()
    b = np.full(A.shape[0], 0.5)
    L, U = O.ilu0(A)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=32, max_iter=1000, tol=1e-10),
                        A.shape[0], *(GRID[name] if name in GRID else (None, None)))
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=32, max_iter=1000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


def test_spmv_long_rows(solver):
    """Rows above the block capacity (2048 entries) are summed by a strided
    block reduction: within 1e-13 of the serial sum (scale |A||x|); every
    other row stays bit-exact."""
    A = M.power_law(6000, 600000, seed=3)
    rl = np.diff(A.indptr)
    assert (rl > 2048).sum() > 0
    x = np.random.default_rng(4).standard_normal(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_none()
    y, ref = solver.spmv(x), O.spmv(A, x)
    short = rl <= 2048
    assert np.array_equal(y[short], ref[short])
    scale = abs(A) @ abs(x)
    assert np.all(np.abs(y - ref) <= 1e-13 * scale)


@pytest.mark.slow
def test_spmv_c3_standin_full_size(solver):
    """The C3 stand-in at circuit5M's size (5.56M rows, 59.5M nnz): its
    sliced-ELL padding would overflow int32 offsets, so it is not sliced (a
    regression: the layout check must fall back, not fail); y = A x runs on
    column panels (k_spmv_panel), every row -- long ones too -- bit-exact."""
    A = M.power_law()
    x = np.random.default_rng(12).standard_normal(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_none()
    assert not solver.spmv_sliced and solver.spmv_panels >= 2
    y, ref = solver.spmv(x), O.spmv(A, x)
    assert np.array_equal(y, ref)


@pytest.mark.parametrize("layout", ["rtile", "rtile7", "panel_major"])
@pytest.mark.parametrize("case", ["powerlaw", "long_rows", "empty_rows"])
def test_spmv_panels_bitexact(solver, case, layout, monkeypatch):
    """Column panels at test size (GG_SPMV_PANEL / GG_SPMV_PANEL_MIN lowered):
    every row bit-exact vs the serial CSR-order sum, rows above 2,048 entries
    included (the panels sum every row serially), empty rows 0 -- in the
    row-tile launch (default 1,024 row blocks; 7 blocks: long walks, segments
    cut into pieces) and the panel-major launches (GG_SPMV_RTILE=0)."""
    monkeypatch.setenv("GG_SPMV_PANEL_MIN", "1000")
    monkeypatch.setenv("GG_SPMV_RTILE", {"rtile": "1024", "rtile7": "7", "panel_major": "0"}[layout])
    if case == "powerlaw":
        A = M.power_law(200_000, 2_200_000, seed=5)
        monkeypatch.setenv("GG_SPMV_PANEL", "30000")
    elif case == "long_rows":
        A = M.power_law(6000, 600000, seed=3)
        monkeypatch.setenv("GG_SPMV_PANEL", "700")
    else:
        B = M.power_law(50_000, 400_000, seed=8).tolil()
        for r in range(0, 50_000, 97):
            B.rows[r] = []
            B.data[r] = []
        A = B.tocsr()
        monkeypatch.setenv("GG_SPMV_PANEL", "4096")
    x = np.random.default_rng(4).standard_normal(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_none()
    assert solver.spmv_panels >= 2
    assert np.array_equal(solver.spmv(x), O.spmv(A, x))


def test_gmres_panels_bitexact(monkeypatch):
    """GMRES(30) + ILU(0) on a power-law matrix whose inner SpMV runs on column
    panels: bit-identical to the order-matched oracle (the panel sums are the
    CSR order, so the solver's arithmetic is unchanged)"""
    monkeypatch.setenv("GG_SPMV_PANEL_MIN", "1000")
    monkeypatch.setenv("GG_SPMV_PANEL", "6000")
    A = M.power_law(40_000, 400_000, seed=11)
    b = M.rhs_ones(A)
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    assert s.spmv_panels >= 2
    g = s.solve(b, restart=30, max_iter=300, tol=1e-10)
    L, U = O.ilu0(A)
    lay, G = s.layout()
    O.set_dot_order(lay, G)
    try:
        ot = O.gmres_left(A, L, U, b, m=30, max_iter=300, tol=1e-10)
    finally:
        O.set_dot_order(None)
    assert g["iters"] == ot["iters"] and np.array_equal(g["hist"], ot["hist"]) and np.array_equal(g["x"], ot["x"])
    s.close()


@pytest.mark.parametrize("name", sorted(MATS))
@pytest.mark.parametrize("force_level", [False, True, "csr", "per_level"])
def test_ilu0_apply_bitexact(solver, name, force_level, monkeypatch):
    """wavefront kernel where it applies; force_level: the dataflow level kernel
    (k_trsv_flow, short rows from its sliced term copy where built; "csr": from
    the CSR arrays, GG_FLOW_ELL=0); "per_level": one k_trsv_level launch per level"""
    if force_level:
        monkeypatch.setenv("GG_NO_WAVEFRONT", "1")
    if force_level == "csr":
        monkeypatch.setenv("GG_FLOW_ELL", "0")
    if force_level == "per_level":
        monkeypatch.setenv("GG_TRSV_LEVELS", "1")
    A = MATS[name]()
    L, U = O.ilu0(A)
    y = np.random.default_rng(2).standard_normal(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront == (name in WAVE and not force_level)
    z = solver.precond_apply(ggmres.APPLY_MINV, y)
    assert np.array_equal(z, O.lusolve(L, U, y))


@pytest.mark.parametrize("name", sorted(WAVE))
@pytest.mark.parametrize("scale", [1.0, 1e-250, 1e250])
@pytest.mark.parametrize("hwdiv", [False, True])
def test_wavefront_division_modes(solver, name, scale, hwdiv, monkeypatch):
    """The U solve divides by the diagonal: IEEE division (GG_WAVE_HWDIV=1) or
    the reciprocal + two FMA corrections (kernels.hip WD_RCP).  Both must give
    RN(acc/d) bit for bit; right-hand sides at 1e-250 / 1e250 leave WD_RCP's
    safe range, are flagged by the writer wave and redone with IEEE division."""
    if hwdiv:
        monkeypatch.setenv("GG_WAVE_HWDIV", "1")
    A = MATS[name]()
    L, U = O.ilu0(A)
    y = np.random.default_rng(3).standard_normal(A.shape[0]) * scale
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    for _ in range(2):      # the second apply runs after any fallback demotion
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


@pytest.mark.parametrize("k", [1, 2, 3])
def test_lu_precond_user_factors(solver, k):
    """ILU(1)/ILU(2) factors of a 5-point grid: the skewed wavefront (skew k+1);
    ILU(3) adds offset nx-3 -> the dataflow kernel"""
    A = M.laplacian_5pt(50, 70)
    L, U = O.iluk(A, k)
    solver.set_matrix(A)
    solver.set_precond_lu(L, U)
    assert solver.uses_wavefront == (k <= 2)
    y = np.random.default_rng(4).random(A.shape[0])
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


@pytest.mark.parametrize("k", [1, 2])
@pytest.mark.parametrize("dims", [(100, 100), (37, 64), (5, 200), (300, 129)])
@pytest.mark.parametrize("scale", [1.0, 1e250])
def test_skewed_wavefront_apply(solver, k, dims, scale, monkeypatch):
    """ILU(k) on 5-point grids (ragged bands, narrow lines, several bands): the
    skewed wavefront gives the serial solve bit for bit; at 1e250 the WD_RCP
    division leaves its safe range and the apply is redone with IEEE division"""
    A = M.laplacian_5pt(*dims)
    L, U = O.iluk(A, k)
    solver.set_matrix(A)
    solver.set_precond_iluk(k)
    assert solver.uses_wavefront
    y = np.random.default_rng(7).standard_normal(A.shape[0]) * scale
    for _ in range(2):
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


def test_split_maps_bitexact(solver):
    A = M.laplacian_5pt(30)
    P = make_split(A, seed=5)
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    v = np.random.default_rng(6).standard_normal(A.shape[0])
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_LEFT, v), P.left(v))
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_RIGHT, v), P.right(v))
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_START, v), P.start(v))


def check_gmres(g, o):
    """Against the serial-order oracle (the reference CPU engine's summation):
    same return code and iteration counts; history within 1e-10 of its own
    scale (max |h|) -- entries far below the scale differ by summation order
    alone (~eps/h relative, DESIGN.md "Parity"); x within 1e-10 relative."""
    assert g["ret"] == o["ret"]
    assert g["iters"] == o["iters"]
    assert g["inner"] == o["inner"]
    h, ho = np.asarray(g["hist"]), np.asarray(o["hist"])
    assert h.shape == ho.shape
    scale = np.max(np.abs(ho)) if ho.size else 1.0
    assert np.max(np.abs(h - ho)) <= HIST_RTOL * scale, np.max(np.abs(h - ho)) / scale
    assert abs(g["relres"] - o["relres"]) <= HIST_RTOL * scale
    assert rel_err(g["x"], o["x"]) <= 1e-10


def check_exact(g, o):
    """Against the order-matched oracle (the device reduction tree restated):
    bit-identical history, iteration counts and solution."""
    assert g["ret"] == o["ret"] and g["iters"] == o["iters"] and g["inner"] == o["inner"]
    ok, msg = hist_close(g["hist"], o["hist"], 0.0)
    assert ok, msg
    assert np.array_equal(g["x"], o["x"]), rel_err(g["x"], o["x"])


def oracle_both(run, n, nx=None, ny=None, skew=1, layout=None):
    """run() under serial and under order-matched dot products (layout: the
    solver's own (lay2nat, G), Solver.layout(), e.g. an RCM flow layout)."""
    o_serial = run()
    lay, G = layout if layout is not None else device_layout(n, nx, ny, skew)
    O.set_dot_order(lay, G)
    try:
        o_tree = run()
    finally:
        O.set_dot_order(None)
    return o_serial, o_tree


@pytest.mark.parametrize("m", [30, 32])
@pytest.mark.parametrize("rhs", ["ones", "uniform"])
@pytest.mark.parametrize("persist", [True, False])
def test_gmres_left_c1_parity(solver, m, rhs, persist, monkeypatch):
    """persist: one persistent launch per inner iteration for the orthogonalization
    (default) or the per-step kernels (GG_NO_PERSIST=1): both bit-identical."""
    if not persist:
        monkeypatch.setenv("GG_NO_PERSIST", "1")
    A = M.laplacian_5pt(100)
    b = M.rhs_ones(A) if rhs == "ones" else M.rhs_uniform(A.shape[0])
    L, U = O.ilu0(A)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=m, max_iter=3000, tol=1e-10),
                        A.shape[0], nx=100)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    g = solver.solve(b, restart=m, max_iter=3000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


@pytest.mark.parametrize("case", ["c1", "grid3d"])
def test_gmres_wide_orthogonalization_parity(solver, case, monkeypatch):
    """k_arnoldi_wide (w on chip, basis streamed; the path of vectors beyond
    the persistent kernel's registers, C4 / C3) forced onto small systems
    (GG_WIDE_FORCE=1: its 512-block tree at any size, most threads with 0-1
    units): history, iterations and solution bit-identical to the oracle in
    that reduction order."""
    monkeypatch.setenv("GG_WIDE_FORCE", "1")
    if case == "c1":
        A, nx, ny = M.laplacian_5pt(100), 100, None
    else:
        A, nx, ny = M.grid_7pt(20, 30, 7, upwind=0.1), 20, 30
    n = A.shape[0]
    b = M.rhs_uniform(n)
    L, U = O.ilu0(A)
    lay, _ = device_layout(n, nx, ny)
    O.set_dot_order(lay, 512)
    try:
        ot = O.gmres_left(A, L, U, b, m=30, max_iter=200, tol=1e-10)
    finally:
        O.set_dot_order(None)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    g = solver.solve(b, restart=30, max_iter=200, tol=1e-10)
    check_exact(g, ot)


def test_gmres_left_fixed_iterations(solver):
    # fixed-length run (tol unreachable): exhaustion semantics + full history
    A = M.laplacian_5pt(100)
    b = M.rhs_uniform(A.shape[0])
    L, U = O.ilu0(A)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=100, tol=1e-300),
                        A.shape[0], nx=100)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=30, max_iter=100, tol=1e-300)
    assert o["ret"] == 1 and o["iters"] == 100
    check_gmres(g, o)
    check_exact(g, ot)


@pytest.mark.parametrize("name", ["7pt_10x10x10", "sherman1", "thermal_7pt_12", "5pt_37x64",
                                  "powerlaw_3000"])
def test_gmres_left_other_matrices(solver, name):
    A = MATS[name]()
    b = M.rhs_uniform(A.shape[0])
    L, U = O.ilu0(A)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=2000, tol=1e-10),
                        A.shape[0], *(GRID[name] if name in GRID else (None, None)))
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g = solver.solve(b, restart=30, max_iter=2000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


def test_gmres_iluk_parity(solver):
    A = M.grid_7pt(10, 10, 8)
    b = M.rhs_uniform(A.shape[0])
    L, U = O.iluk(A, 1)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=20, max_iter=1000, tol=1e-10),
                        A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_iluk(1)
    g = solver.solve(b, restart=20, max_iter=1000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


@pytest.mark.parametrize("k,dims,device", [(1, (100, 100), False), (2, (37, 64), False),
                                           (1, (130, 70), True)])
def test_gmres_iluk_grid_parity(solver, k, dims, device):
    """GMRES + ILU(k) on 5-point grids through the skewed wavefront (layout
    lane skew k+1): serial-oracle tolerance and order-matched bit-exact"""
    A = M.laplacian_5pt(*dims)
    b = M.rhs_uniform(A.shape[0])
    L, U = O.iluk(A, k)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=2000, tol=1e-10),
                        A.shape[0], nx=dims[0], skew=k + 1)
    solver.set_matrix(A)
    if device:
        solver.set_precond_iluk_device(k)
    else:
        solver.set_precond_iluk(k)
    assert solver.uses_wavefront
    g = solver.solve(b, restart=30, max_iter=2000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


@pytest.mark.parametrize("name,k,long_rows", [("5pt_10x10", 1, None), ("7pt_10x10x10", 1, None),
                                              ("9pt_10x10", 2, None), ("sherman1", 1, None),
                                              ("c1_5pt_100x100", 0, None), ("c1_5pt_100x100", 2, None),
                                              ("thermal_7pt_12", 1, None), ("powerlaw_3000", 1, None),
                                              ("powerlaw_3000", 1, 12), ("sherman1", 1, 6),
                                              ("9pt_10x10", 2, 0), ("thermal_7pt_12", 1, 9)])
def test_iluk_device_factors_bitexact(solver, name, k, long_rows, monkeypatch):
    """ILU(k) with ilukC's numeric phase on the GPU: the same factors, bit for bit,
    as the oracle's lofC + ilukC restatement (and hence as the host path).
    long_rows: rows longer than this take the kernel's long-row path (HBM values,
    dense position map) instead of the LDS path (GG_ILUK_LONG)."""
    if long_rows is not None:
        monkeypatch.setenv("GG_ILUK_LONG", str(long_rows))
    A = MATS[name]()
    solver.set_matrix(A)
    try:
        Lo, Uo = O.iluk(A, k)
    except ZeroDivisionError:
        with pytest.raises(ggmres.GGError):
            solver.iluk_device_factors(k)
        return
    (lrp, lci, lv), (urp, uci, uv), ms = solver.iluk_device_factors(k)
    assert ms > 0
    for (rp, ci, v), o in (((lrp, lci, lv), Lo), ((urp, uci, uv), Uo)):
        assert np.array_equal(rp, o.rp) and np.array_equal(ci, o.ci)
        assert np.array_equal(v, o.v)


def test_gmres_iluk_device_parity(solver):
    """GMRES with the device-factored ILU(1): identical to the host-factored run."""
    A = M.grid_7pt(10, 10, 8)
    b = M.rhs_uniform(A.shape[0])
    L, U = O.iluk(A, 1)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=20, max_iter=1000, tol=1e-10),
                        A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_iluk_device(1)
    g = solver.solve(b, restart=20, max_iter=1000, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)


def test_iluk_device_zero_pivot(solver):
    import scipy.sparse as sp
    solver.set_matrix(sp.csr_matrix(np.array([[0.0, 1.0], [1.0, 1.0]])))
    with pytest.raises(ggmres.GGError):
        solver.set_precond_iluk_device(1)


@pytest.mark.parametrize("ell", ["1", "0"])
def test_gmres_split_parity(solver, ell, monkeypatch):
    """randomly permuted split factors (the flow kernel; ell "0": its CSR form)"""
    monkeypatch.setenv("GG_FLOW_ELL", ell)
    A = M.laplacian_5pt(40)
    P = make_split(A, seed=9)
    b = M.rhs_uniform(A.shape[0])
    x0 = np.random.default_rng(3).random(A.shape[0]) * 0.1
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    assert not solver.uses_wavefront
    lay, G = solver.layout()                    # the flow path's RCM layout (gg_layout)
    assert not np.array_equal(lay[:A.shape[0]], np.arange(A.shape[0]))
    assert np.array_equal(np.sort(lay[lay >= 0]), np.arange(A.shape[0]))
    o, ot = oracle_both(lambda: O.gmres_split(A, P, b, x0=x0, m=32, max_iter=2000, tol=1e-11),
                        A.shape[0], layout=(lay, G))
    g = solver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    check_gmres(g, o)
    check_exact(g, ot)


def test_gmres_split_parity_natural_layout(solver, monkeypatch):
    """GG_FLOW_RCM=0: the flow path in the natural layout, the same arithmetic
    per row (only the dots' reduction order follows the layout)"""
    monkeypatch.setenv("GG_FLOW_RCM", "0")
    A = M.laplacian_5pt(40)
    P = make_split(A, seed=9)
    b = M.rhs_uniform(A.shape[0])
    x0 = np.random.default_rng(3).random(A.shape[0]) * 0.1
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    lay, G = solver.layout()
    assert np.array_equal(lay[:A.shape[0]], np.arange(A.shape[0]))
    o, ot = oracle_both(lambda: O.gmres_split(A, P, b, x0=x0, m=32, max_iter=2000, tol=1e-11),
                        A.shape[0])
    g = solver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    check_gmres(g, o)
    check_exact(g, ot)


@pytest.mark.parametrize("dims", [(40, 40), (70, 130)])
def test_split_wavefront_maps_bitexact(solver, dims):
    """The split engine on grid-shaped factors: 2D wavefront L (non-unit, diag
    last) and U (diag first, in-line term first), D_r^-1 folded into the U
    solve's store, the row gather and D_l^-1 into the SpMV."""
    A = M.laplacian_5pt(*dims)
    P = make_split(A, seed=5, identity_perm=True)
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    assert solver.uses_wavefront
    rng = np.random.default_rng(6)
    for scale in (1.0, 1e250, 1e-250):
        v = rng.standard_normal(A.shape[0]) * scale
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_LEFT, v), P.left(v))
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_RIGHT, v), P.right(v))
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_START, v), P.start(v))
    x = rng.standard_normal(A.shape[0])
    assert np.array_equal(solver.spmv(x), O.spmv(A, x))


def test_gmres_split_wavefront_parity(solver):
    A = M.laplacian_5pt(48, 40)
    n = A.shape[0]
    P = make_split(A, seed=9, identity_perm=True)
    b = M.rhs_uniform(n)
    x0 = np.random.default_rng(3).random(n) * 0.1
    o, ot = oracle_both(lambda: O.gmres_split(A, P, b, x0=x0, m=32, max_iter=2000, tol=1e-11), n, nx=48)
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    assert solver.uses_wavefront
    g = solver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    check_gmres(g, o)
    check_exact(g, ot)
    # reciprocal-multiply division on both wavefront solves: tolerance parity
    solver.set_division(ggmres.DIV_RCP)
    try:
        assert solver.division_active(0) == solver.division_active(1) == ggmres.DIV_RCP
        g2 = solver.solve(b, x0=x0, restart=32, max_iter=2000, tol=1e-11)
    finally:
        solver.set_division(ggmres.DIV_EXACT)        # the fixture is shared by the module
    check_gmres(g2, o)


def test_split_random_perm_spmv(solver):
    """gg_spmv on a split solver (A' = A with permuted rows and columns inside)"""
    A = M.laplacian_5pt(30, 20)
    P = make_split(A, seed=4)
    solver.set_matrix(A)
    solver.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    assert not solver.uses_wavefront
    x = np.random.default_rng(2).standard_normal(A.shape[0])
    assert np.array_equal(solver.spmv(x), O.spmv(A, x))


def test_edge_cases(solver):
    A = M.laplacian_5pt(100)
    n = A.shape[0]
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    run = lambda f: oracle_both(f, n, nx=100)
    # converged at the initial check ("<=", iters = 0)
    x0 = np.ones(n)
    g = solver.solve(A @ x0, x0=x0, restart=10, max_iter=50, tol=1e-10)
    o, ot = run(lambda: O.gmres_left(A, L, U, A @ x0, x0=x0, m=10, max_iter=50, tol=1e-10))
    check_gmres(g, o)
    check_exact(g, ot)
    # zero right-hand side (normb -> 1)
    g = solver.solve(np.zeros(n), restart=10, max_iter=50, tol=1e-10)
    assert g["ret"] == 0 and g["iters"] == 0 and np.all(g["x"] == 0)
    # max_iter = 0: not converged, history = [beta0/normb]
    b = M.rhs_uniform(n)
    g = solver.solve(b, restart=10, max_iter=0, tol=1e-10)
    o, ot = run(lambda: O.gmres_left(A, L, U, b, m=10, max_iter=0, tol=1e-10))
    check_gmres(g, o)
    check_exact(g, ot)
    # restart m = 1, a cycle cut short by max_iter (Update of the last filled
    # column), and m = 80 (above the one-wave Update kernel: the serial one)
    for m, mi in ((1, 17), (7, 25), (64, 100), (80, 170)):
        g = solver.solve(b, restart=m, max_iter=mi, tol=1e-300)
        o, ot = run(lambda: O.gmres_left(A, L, U, b, m=m, max_iter=mi, tol=1e-300))
        check_gmres(g, o)
        check_exact(g, ot)


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 127, 513])
def test_small_and_ragged_sizes(solver, n):
    """Sizes around the 64-lane, 256-thread and 512-slot paddings: a seeded
    diagonally dominant random matrix (natural layout, flow triangular solves)
    and, where it is a grid, a 5-point n x 3 grid (wavefront layout)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(n)
    R = sp.random(n, n, density=min(1.0, 4.0 / n), random_state=np.random.RandomState(n), format="csr")
    R.data = -R.data
    A = (R + sp.diags(np.asarray(abs(R).sum(axis=1)).ravel() + 1.0)).tocsr()
    A.sort_indices()
    cases = [(A, None)]
    if n >= 2:
        cases.append((M.laplacian_5pt(n, 3), n))
    for A_, nx in cases:
        b = rng.random(A_.shape[0])
        L, U = O.ilu0(A_)
        solver.set_matrix(A_)
        solver.set_precond_ilu0()
        wave = solver.uses_wavefront            # grids with nx >= 4 (tiny grids: level path)
        assert wave == (nx is not None and nx >= 4) or not wave
        o, ot = oracle_both(lambda: O.gmres_left(A_, L, U, b, m=10, max_iter=60, tol=1e-12),
                            A_.shape[0], nx=nx if wave else None)
        g = solver.solve(b, restart=10, max_iter=60, tol=1e-12)
        check_gmres(g, o)
        check_exact(g, ot)
        x = rng.standard_normal(A_.shape[0])
        assert np.array_equal(solver.spmv(x), O.spmv(A_, x))


@pytest.mark.parametrize("k", [0, 1])
def test_concurrent_shared_solves(solver, k):
    """GG_SOLVE_SHARED_DEVICE: four solvers (own streams) solving at the same
    time from four host threads; each result bit-identical to the
    order-matched oracle (the flag swaps the persistent orthogonalization
    launch for the per-step kernels, same arithmetic).  k = 1: ILU(1) factors
    on the skewed wavefront."""
    import threading
    A = M.laplacian_5pt(300, 256)
    L, U = O.iluk(A, k) if k else O.ilu0(A)
    bs = [M.rhs_uniform(A.shape[0], seed=50 + q) for q in range(4)]
    refs = [oracle_both(lambda b=b: O.gmres_left(A, L, U, b, m=30, max_iter=90, tol=1e-300),
                        A.shape[0], nx=300, skew=k + 1)[1] for b in bs]
    ss = [ggmres.Solver(0) for _ in range(4)]
    try:
        for s_ in ss:
            s_.set_matrix(A)
            if k:
                s_.set_precond_iluk(k)
            else:
                s_.set_precond_ilu0()
            assert s_.uses_wavefront
        out = [None] * 4

        def run(q):
            out[q] = ss[q].solve(bs[q], restart=30, max_iter=90, tol=1e-300,
                                 flags=ggmres.SOLVE_SHARED_DEVICE)

        th = [threading.Thread(target=run, args=(q,)) for q in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for g, ot in zip(out, refs):
            check_exact(g, ot)
    finally:
        for s_ in ss:
            s_.close()


def test_trace_refuses_skewed_wavefront(solver):
    """gg_trace_precond instruments only the unskewed kernel: GG_ESTATE (-5) on ILU(1)."""
    A = M.laplacian_5pt(64, 64)
    solver.set_matrix(A)
    solver.set_precond_iluk(1)
    assert solver.uses_wavefront
    with pytest.raises(ggmres.GGError) as e:
        solver.trace_precond(0)
    assert e.value.code == -5


def test_shared_flag_needs_2d_wavefront(solver):
    solver.set_matrix(MATS["sherman1"]())
    solver.set_precond_ilu0()
    with pytest.raises(ggmres.GGError):
        solver.solve(np.ones(solver.n), flags=ggmres.SOLVE_SHARED_DEVICE)
    with pytest.raises(ggmres.GGError):
        solver.solve(np.ones(solver.n), flags=0x100)


def test_repeated_solves_identical(solver):
    A = M.laplacian_5pt(100)
    b = M.rhs_uniform(A.shape[0])
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    g1 = solver.solve(b, restart=30, max_iter=500, tol=1e-10)
    g2 = solver.solve(b, restart=30, max_iter=500, tol=1e-10)
    assert np.array_equal(g1["x"], g2["x"]) and np.array_equal(g1["hist"], g2["hist"])


@pytest.mark.slow
def test_c2_full_size_properties(solver):
    """C2 (1M rows): first cycle vs the oracle, then size-independent properties."""
    A = M.laplacian_5pt(1000)
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront and solver.spmv_sliced
    # one full restart cycle against the oracle (serial order and order-matched)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=30, tol=1e-300),
                        A.shape[0], nx=1000)
    g = solver.solve(b, restart=30, max_iter=30, tol=1e-300)
    check_gmres(g, o)
    check_exact(g, ot)
    # full solve to 1e-8: convergence, true preconditioned residual
    g = solver.solve(b, restart=30, max_iter=20000, tol=1e-8)
    assert g["ret"] == 0 and g["relres"] < 1e-8
    normb = np.linalg.norm(O.lusolve(L, U, b))
    true = np.linalg.norm(O.lusolve(L, U, b - A @ g["x"])) / normb
    assert true < 1e-7
    h = g["hist"]
    assert np.all(np.isfinite(h)) and h[0] == pytest.approx(1.0, rel=1e-12)


@pytest.mark.parametrize("grid", [(40, 40), (30, 70)])
def test_transient_c5(solver, grid):
    """C5: backward-Euler loop on one ILU(0) factorization (gg_transient) against
    the reference step driver restated (oracle.transient): ports and final
    state bit-identical to the order-matched oracle, within 1e-10 of the
    serial one; identical per-step iteration totals."""
    nx, ny = grid
    h = 1e-2
    Gm = M.laplacian_5pt(nx, ny)
    A = M.transient(Gm, c=1e-3, h=h)
    n = A.shape[0]
    cdiag = np.full(n, 1e-3 / h)
    nodes, pulses = M.pulse_sources(n, frac=0.01, h=h)
    ports = np.array([0, n // 3, n // 2, n - 1], np.int32)
    x0 = np.zeros(n)
    L, U = O.ilu0(A)
    run = lambda: O.transient(A, L, U, 25, h, cdiag, nodes, pulses, ports, x0, m=32,
                              max_iter=10000, tol=1e-7)
    o, ot = oracle_both(run, n, nx=nx)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    g = solver.transient(25, h, cdiag, nodes, pulses, ports, x0, restart=32, max_iter=10000, tol=1e-7)
    assert g["iters_total"] == ot["iters_total"] == o["iters_total"]
    assert np.array_equal(g["ports"], ot["ports"]) and np.array_equal(g["x"], ot["x"])
    assert rel_err(g["x"], o["x"]) <= 1e-10
    assert np.max(np.abs(g["ports"] - o["ports"])) <= 1e-10 * np.max(np.abs(o["ports"]))
    assert np.max(np.abs(o["ports"])) > 0      # the sources did drive the grid


def test_transient_mixed_sources(solver):
    """gg_transient_src with DC, PULSE and PWL sources (gen_dcVt / gen_PULSEut /
    gen_PWLut semantics, several sources on one node) against the restated
    step driver: bit-identical to the order-matched oracle."""
    nx, ny = 40, 40
    h = 1e-2
    A = M.transient(M.laplacian_5pt(nx, ny), c=1e-3, h=h)
    n = A.shape[0]
    cdiag = np.full(n, 1e-3 / h)
    rng = np.random.default_rng(21)
    nodes = np.sort(rng.choice(n, size=24, replace=False)).astype(np.int32)
    nodes[5] = nodes[4]                                   # two sources on one node
    srcs = []
    for k in range(len(nodes)):
        if k % 3 == 0:
            srcs.append((O.SRC_DC, [1e-3 * (1 + k)]))
        elif k % 3 == 1:
            srcs.append((O.SRC_PULSE, [0.0, 2e-3, 2 * h, 3 * h, 4 * h, 5 * h, 20 * h]))
        else:
            srcs.append((O.SRC_PWL, [0.0, 0.0, 3 * h, 1e-3, 7.5 * h, 1e-3, 12 * h, -5e-4]))
    ports = np.array([nodes[0], nodes[1], nodes[2], n - 1], np.int32)
    x0 = np.zeros(n)
    L, U = O.ilu0(A)
    taps = np.concatenate([nodes[:6], [0, n // 2, n - 1]]).astype(np.int32)
    run = lambda: O.transient(A, L, U, 15, h, cdiag, nodes, None, ports, x0, m=32, max_iter=10000,
                              tol=1e-7, sources=srcs, taps=taps)
    o, ot = oracle_both(run, n, nx=nx)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    solver.set_taps(taps)
    g = solver.transient_src(15, h, cdiag, nodes, srcs, ports, x0, restart=32, max_iter=10000, tol=1e-7)
    assert g["iters_total"] == ot["iters_total"]
    assert np.array_equal(g["ports"], ot["ports"]) and np.array_equal(g["x"], ot["x"])
    assert rel_err(g["x"], o["x"]) <= 1e-10
    # tap statistics (ir_info): bit-identical max / min / avg / IR drop
    for a_, b_ in zip(solver.get_taps(), ot["taps"]):
        assert np.array_equal(a_, b_)
    assert np.max(ot["taps"][3]) > 0
    solver.set_taps([])


@pytest.mark.gpu
def test_profile_kind_mask():
    """gg_profile_enable(kinds): only the selected families are bracketed."""
    A = M.laplacian_5pt(40)
    b = M.rhs_ones(A)
    s = ggmres.Solver()
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.profile(True, kinds=[ggmres.PROF_TRSV_U])
    r = s.solve(b, np.zeros(A.shape[0]), restart=30, max_iter=200, tol=1e-8)
    n_u = s.profile_get(ggmres.PROF_TRSV_U)[0]
    assert r["inner"] <= n_u <= r["inner"] + r["restarts"] + 1
    for k in (ggmres.PROF_SPMV, ggmres.PROF_PRECOND, ggmres.PROF_MGS, ggmres.PROF_TRSV_L):
        assert s.profile_get(k)[0] == 0
    s.profile(True)
    s.solve(b, np.zeros(A.shape[0]), restart=30, max_iter=200, tol=1e-8)
    assert all(s.profile_get(k)[0] > 0 for k in range(ggmres.PROF_NKINDS))
    s.close()


def _near_zero_grid():
    """5-pt grid where some structural off-diagonals are |a| < 1e-9: generateLevel
    ignores them, so the reference's column order differs from the index order
    and some columns read sources that are not factored yet."""
    A = M.laplacian_5pt(20, 17).tolil()
    rng = np.random.default_rng(11)
    n = A.shape[0]
    for r in rng.choice(n, 40, replace=False):
        for c in (r + 1, r + 20):
            if c < n and A[r, c] != 0:
                A[r, c] = 1e-12 * (1 + rng.random())
    A = A.tocsr()
    A.sort_indices()
    return A


@pytest.mark.parametrize("name", sorted(MATS) + ["near_zero_grid"])
def test_ilu0_device_factor_bitexact(solver, name):
    """Device ILU(0) (k_ilu0_columns) == leftILU restated, value for value."""
    A = _near_zero_grid() if name == "near_zero_grid" else MATS[name]()
    solver.set_matrix(A)
    fv, ms = solver.ilu0_device_values()
    assert ms > 0
    assert np.array_equal(fv, O.ilu0_values(A))
    solver.set_precond_ilu0_device()
    L, U = O.ilu0(A)
    y = np.random.default_rng(5).standard_normal(A.shape[0])
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))


@pytest.mark.parametrize("dims", [(9, 5, 3), (17, 9, 8), (33, 16, 17), (2, 40, 40)])
def test_tile3d_edges_and_ranges(solver, dims):
    """3D tile wavefront at its edges: tiles cut by the grid in both directions
    (9 x 5 x 3: one partial tile; 17 x 9 x 8 and 33 x 16 x 17: whole and
    partial tiles), the shortest lines (nx = 2), and right-hand sides at
    1e-250 / 1e250 (WD_RCP's range guard repeating the U solve with IEEE
    division): every apply bit-exact vs the oracle."""
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz, upwind=0.2)
    n = A.shape[0]
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    rng = np.random.default_rng(11)
    for scale in (1.0, 1e-250, 1e250):
        y = rng.standard_normal(n) * scale
        assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y)), scale


@pytest.mark.parametrize("dims", [(20, 30, 7), (16, 70, 5), (8, 8, 300), (130, 3, 4)])
def test_wave3d_apply_and_gmres(solver, dims):
    """3D 7-point grids on the pipelined (plane, band) wavefront kernel: several
    bands per plane (16x70), more tasks than co-resident workgroups (8x8x300),
    several batches per line (130): apply and GMRES bit-exact vs the oracle."""
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz, upwind=0.1)
    n = A.shape[0]
    L, U = O.ilu0(A)
    solver.set_matrix(A)
    solver.set_precond_ilu0()
    assert solver.uses_wavefront
    y = np.random.default_rng(8).standard_normal(n)
    assert np.array_equal(solver.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))
    b = M.rhs_uniform(n)
    # 120 iterations: long enough for several restarts, short enough that the
    # serial-order history stays within 1e-10 on the slowest case (130x3x4)
    o, ot = oracle_both(lambda: O.gmres_left(A, L, U, b, m=30, max_iter=120, tol=1e-10), n, nx, ny)
    g = solver.solve(b, restart=30, max_iter=120, tol=1e-10)
    check_gmres(g, o)
    check_exact(g, ot)
