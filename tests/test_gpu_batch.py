"""The many-RHS solve (gg_solve_batch*, gg_transient_batch; gpu-gmres_amd/csrc/batch.hip).

SURVEY.md 8(d) C5 "many-RHS": independent source scenarios solved as a batch.
Every scenario must be exactly the single-RHS solve: the batched launches only
share the matrix, the preconditioner and the launch -- so per scenario the
residual history, iteration count, return code and solution are BIT-identical
to gg_solve / gg_transient on that scenario alone (which tests/test_gpu_parity.py
pins to the order-matched oracle), and the batched C5 scenarios are checked
against the order-matched restated step driver (oracle.transient) directly.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import ggmres
import oracle as O
from ggmres import matrices as M
from helpers import device_layout, rel_err

pytestmark = pytest.mark.gpu


def _rhs_set(A, S, seed):
    """S right-hand sides of different character: ones (b = A 1), random,
    a zero vector (converged at the start), scaled random"""
    n = A.shape[0]
    rng = np.random.default_rng(seed)
    out = []
    for q in range(S):
        k = q % 4
        if k == 0:
            out.append(M.rhs_ones(A))
        elif k == 1:
            out.append(rng.standard_normal(n))
        elif k == 2:
            out.append(np.zeros(n))
        else:
            out.append(1e3 * rng.uniform(-1, 1, n))
    return np.array(out)


def _single(s, B, X0, **kw):
    out = []
    for q in range(B.shape[0]):
        out.append(s.solve(B[q], x0=X0[q], **kw))
    return out


@pytest.mark.parametrize("division", [ggmres.DIV_EXACT, ggmres.DIV_FMA, ggmres.DIV_RCP])
@pytest.mark.parametrize("grid,m,max_iter,tol", [((100, 100), 30, 3000, 1e-10),   # C1: converges inside a cycle
                                                  ((37, 64), 8, 3000, 1e-11),      # several restart cycles
                                                  ((40, 40), 30, 12, 1e-300)])     # max_iter cuts the cycle
def test_solve_batch_bitexact_vs_single(grid, m, max_iter, tol, division):
    A = M.laplacian_5pt(*grid)
    n = A.shape[0]
    S = 5
    B = _rhs_set(A, S, seed=3)
    X0 = np.zeros((S, n))
    X0[1] = np.random.default_rng(9).standard_normal(n) * 1e-2       # a warm start
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.set_division(division)
    assert s.uses_wavefront and s.batch_engine
    g = s.solve_batch(B, X0, restart=m, max_iter=max_iter, tol=tol)
    ref = _single(s, B, X0, restart=m, max_iter=max_iter, tol=tol)
    for q in range(S):
        r = ref[q]
        assert (g["status"][q], g["iters"][q], g["inner"][q], g["restarts"][q]) == \
               (r["ret"], r["iters"], r["inner"], r["restarts"]), q
        assert g["relres"][q] == r["relres"]
        assert np.array_equal(g["hist"][q], r["hist"]), q
        assert np.array_equal(g["x"][q], r["x"]), q
    assert g["iters"][2] == 0 and g["status"][2] == 0            # b = 0: converged at the start
    s.close()


def test_solve_batch_vs_order_matched_oracle():
    """one batch, every scenario against the order-matched oracle (bit-identical)
    and the serial-order oracle (1e-10), GMRES(30) + ILU(0), exact division"""
    nx = 60
    A = M.laplacian_5pt(nx)
    n = A.shape[0]
    S = 4
    B = _rhs_set(A, S, seed=5)
    L, U = O.ilu0(A)
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    g = s.solve_batch(B, restart=30, max_iter=2000, tol=1e-10)
    O.set_dot_order(*device_layout(n, nx))
    try:
        ot = [O.gmres_left(A, L, U, B[q], m=30, max_iter=2000, tol=1e-10) for q in range(S)]
    finally:
        O.set_dot_order(None)
    o = [O.gmres_left(A, L, U, B[q], m=30, max_iter=2000, tol=1e-10) for q in range(S)]
    for q in range(S):
        assert g["iters"][q] == ot[q]["iters"] and g["status"][q] == ot[q]["ret"]
        assert np.array_equal(g["hist"][q], ot[q]["hist"]) and np.array_equal(g["x"][q], ot[q]["x"])
        assert g["iters"][q] == o[q]["iters"]
        sc = max(np.max(np.abs(o[q]["hist"])), 1e-300)
        assert np.max(np.abs(g["hist"][q] - o[q]["hist"])) <= 1e-10 * sc
        if np.any(B[q]):
            assert rel_err(g["x"][q], o[q]["x"]) <= 1e-10
    s.close()


def _hip():
    """the HIP runtime libggmres itself uses (torch's bundled runtime must not
    initialize after it in this process)"""
    import ctypes
    h = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipFree.argtypes = [ctypes.c_void_p]
    return h


def test_solve_batch_many_scenarios_and_device_entry():
    """more scenarios than one batched SpMV launch carries (8), through the
    device entry point with a leading dimension above n"""
    import ctypes
    A = M.laplacian_5pt(48)
    n = A.shape[0]
    S = 11
    B = _rhs_set(A, S, seed=11)
    ld = n + 37
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.set_division(ggmres.DIV_FMA)
    hb = np.zeros(S * ld)
    for q in range(S):
        hb[q * ld:q * ld + n] = B[q]
    hx = np.zeros(S * ld)
    hip = _hip()
    db, dx = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(db), hb.nbytes) == 0 and hip.hipMalloc(ctypes.byref(dx), hx.nbytes) == 0
    try:
        assert hip.hipMemcpy(db, hb.ctypes.data, hb.nbytes, 1) == 0
        assert hip.hipMemcpy(dx, hx.ctypes.data, hx.nbytes, 1) == 0
        g = s.solve_batch_device(db.value, dx.value, S, ld=ld, restart=30, max_iter=3000, tol=1e-10)
        assert hip.hipMemcpy(hx.ctypes.data, dx, hx.nbytes, 2) == 0
    finally:
        hip.hipFree(db)
        hip.hipFree(dx)
    for q in range(S):
        r = s.solve(B[q], restart=30, max_iter=3000, tol=1e-10)
        assert g["iters"][q] == r["iters"] and np.array_equal(hx[q * ld:q * ld + n], r["x"])
        assert not np.any(hx[q * ld + n:(q + 1) * ld])          # the gaps untouched
    s.close()


def test_solve_batch_sequential_fallback(monkeypatch):
    """a configuration the batched launches do not take (sherman1: no grid
    wavefront) and the forced scenario-by-scenario path: same results"""
    from conftest import fixture_path
    A = M.read_rua(fixture_path("sherman1.rua"))
    n = A.shape[0]
    B = np.array([np.ones(n), np.random.default_rng(2).standard_normal(n)])
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    g = s.solve_batch(B, restart=30, max_iter=500, tol=1e-8)
    for q in range(2):
        r = s.solve(B[q], restart=30, max_iter=500, tol=1e-8)
        assert g["iters"][q] == r["iters"] and np.array_equal(g["x"][q], r["x"])
    A2 = M.laplacian_5pt(50)
    B2 = _rhs_set(A2, 3, seed=1)
    s.set_matrix(A2)
    s.set_precond_ilu0()
    assert s.batch_engine
    monkeypatch.setenv("GG_BATCH_SEQ", "1")
    assert not s.batch_engine
    g2 = s.solve_batch(B2, restart=30, max_iter=1000, tol=1e-10)
    monkeypatch.delenv("GG_BATCH_SEQ")
    g3 = s.solve_batch(B2, restart=30, max_iter=1000, tol=1e-10)
    assert g2["iters"] == g3["iters"] and np.array_equal(g2["x"], g3["x"])
    s.close()


@pytest.mark.parametrize("case", ["ilu1_skewed", "grid3d", "nrhs1", "max_iter0"])
def test_solve_batch_edges_match_single(case):
    """configurations at the batch's edges, each scenario against its own
    single solve: ILU(1) grid factors (the skewed wavefront: not batched, the
    scenario-by-scenario path), a 3D grid (tile wavefront: not batched), one
    right-hand side through the batched path, max_iter = 0 (no cycle: a zero
    right-hand side converged at the start, the others not converged)"""
    if case == "grid3d":
        A = M.grid_7pt(20)
    else:
        A = M.laplacian_5pt(60, 52)
    n = A.shape[0]
    S = 1 if case == "nrhs1" else 3
    B = _rhs_set(A, S, seed=21)                 # (scenario 2 is the zero vector)
    max_iter = 0 if case == "max_iter0" else 2000
    s = ggmres.Solver(0)
    s.set_matrix(A)
    if case == "ilu1_skewed":
        s.set_precond_iluk(1)
    else:
        s.set_precond_ilu0()
    s.set_division(ggmres.DIV_FMA)
    assert s.batch_engine == (case in ("nrhs1", "max_iter0"))
    g = s.solve_batch(B, restart=30, max_iter=max_iter, tol=1e-10)
    for q in range(S):
        r = s.solve(B[q], restart=30, max_iter=max_iter, tol=1e-10)
        assert (g["status"][q], g["iters"][q]) == (r["ret"], r["iters"]), q
        assert g["relres"][q] == r["relres"] and np.array_equal(g["x"][q], r["x"]), q
    if case == "max_iter0":
        assert g["status"] == [1, 1, 0] and g["iters"] == [0, 0, 0]
    s.close()


def test_solve_batch_bad_arguments():
    """nrhs < 1, a leading dimension below n and unknown flags are refused"""
    import ctypes
    A = M.laplacian_5pt(32)
    n = A.shape[0]
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    L = ggmres.lib()
    b = np.ones(2 * n)
    x = np.zeros(2 * n)
    res = (ggmres.Result * 2)()
    for nrhs, ld, flags in ((0, n, 0), (2, n - 1, 0), (2, n, ggmres.SOLVE_SHARED_DEVICE)):
        o = ggmres.Options(30, 100, 1e-8, flags)
        rc = L.gg_solve_batch(s.h, nrhs, b, ld, x, ld, ctypes.byref(o), res)
        assert rc == -1, (nrhs, ld, flags, rc)        # GG_EINVAL
    s.close()


def _scenarios(n, S, h, seed0):
    return [M.pulse_sources(n, frac=0.01, h=h, seed=seed0 + q) for q in range(S)]


@pytest.mark.parametrize("division", [ggmres.DIV_EXACT, ggmres.DIV_FMA])
def test_transient_batch_bitexact_vs_single(division):
    """C5 on a 40 x 30 grid, 4 scenarios (own seeded PULSE sets, one with a
    warm nonzero start): every scenario's ports, final state and iteration
    total bit-identical to gg_transient run on that scenario alone"""
    h = 1e-2
    A = M.transient(M.laplacian_5pt(40, 30), c=1e-3, h=h)
    n = A.shape[0]
    cdiag = np.full(n, 1e-3 / h)
    S = 4
    sc = _scenarios(n, S, h, 100)
    ports = np.array([0, n // 3, n // 2, n - 1], np.int32)
    X0 = np.zeros((S, n))
    X0[2] = 1e-4
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.set_division(division)
    assert s.batch_engine
    g = s.transient_batch(30, h, cdiag, sc, ports, X0, restart=32, max_iter=10000, tol=1e-7)
    for q in range(S):
        nodes, pulses = sc[q]
        r = s.transient(30, h, cdiag, nodes, pulses, ports, X0[q], restart=32, max_iter=10000, tol=1e-7)
        assert g["iters_total"][q] == r["iters_total"], q
        assert np.array_equal(g["ports"][q], r["ports"]) and np.array_equal(g["x"][q], r["x"]), q
    assert g["ret"] == 0 and np.max(np.abs(g["ports"])) > 0
    s.close()


@pytest.mark.slow
def test_c5_batch_full_size_vs_order_matched_oracle():
    """BASELINE C5 at its size (1000 x 1000 grid, A = G + C/h), 8 scenarios in
    one batch: the first K = 50 steps of EVERY scenario bit-identical to the
    order-matched restated step driver (oracle.transient, GG_DIV_FMA's rows and
    the device's reduction tree), within 1e-10 of the serial-order driver over
    the first 5 steps; then 1000 batched steps of every scenario equal to
    gg_transient on each scenario alone."""
    K = 50
    h = 1e-2
    A = M.transient(M.laplacian_5pt(1000), c=1e-3, h=h)
    n = A.shape[0]
    cdiag = np.full(n, 1e-3 / h)
    S = 8
    sc = _scenarios(n, S, h, 20261015)
    ports = np.array([0, n // 2, n - 1], np.int32)
    X0 = np.zeros((S, n))
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    s.set_division(ggmres.DIV_FMA)
    assert s.batch_engine
    g = s.transient_batch(K, h, cdiag, sc, ports, X0, restart=32, max_iter=10000, tol=1e-7)
    L, U = O.ilu0(A)

    def run(q, nsteps):
        nodes, pulses = sc[q]
        return O.transient(A, L, U, nsteps, h, cdiag, nodes, pulses, ports, X0[q], m=32, max_iter=10000, tol=1e-7)
    O.set_dot_order(*device_layout(n, 1000))
    O.set_div_mode(2, 2)
    try:
        with ThreadPoolExecutor(max_workers=S) as ex:      # ctypes releases the GIL
            ot = list(ex.map(lambda q: run(q, K), range(S)))
    finally:
        O.set_div_mode()
        O.set_dot_order(None)
    for q in range(S):
        assert g["iters_total"][q] == ot[q]["iters_total"], q
        assert np.array_equal(g["ports"][q], ot[q]["ports"]) and np.array_equal(g["x"][q], ot[q]["x"]), q
    with ThreadPoolExecutor(max_workers=S) as ex:
        o5 = list(ex.map(lambda q: run(q, 5), range(S)))
    for q in range(S):
        sc_ = np.max(np.abs(o5[q]["ports"]))
        assert sc_ > 0 and np.max(np.abs(g["ports"][q][:, :6] - o5[q]["ports"])) <= 1e-10 * sc_
    g = s.transient_batch(1000, h, cdiag, sc, ports, X0, restart=32, max_iter=10000, tol=1e-7)
    for q in range(S):
        nodes, pulses = sc[q]
        r = s.transient(1000, h, cdiag, nodes, pulses, ports, X0[q], restart=32, max_iter=10000, tol=1e-7)
        assert g["iters_total"][q] == r["iters_total"], q
        assert np.array_equal(g["ports"][q], r["ports"]) and np.array_equal(g["x"][q], r["x"]), q
    s.close()
