"""BASELINE.json configs C4 and C5 at their configured sizes, on the GPU.

C4 -- 216^3 7-point thermal grid (n = 10,077,696, kz = 10, convective shift):
  * single GPU: the first K1 = 12 inner iterations of GMRES(30) (cut by
    max_iter inside the first cycle: Update of x mid-cycle) bit-identical to
    the order-matched oracle and within 1e-10 of the serial-order oracle, then
    the solve to 1e-8 with size-independent properties (convergence, the true
    preconditioned residual, history shape);
  * 8-way sharded solve (partition4 slabs, arrow ordering; all 8 shards on this
    GPU, GG_DD_LOCAL -- the kernels and exchange points of one shard per GPU):
    the same K1 iterations bit-identical to the oracle on the permuted matrix
    B = P A P^T with the sharded reduction order, then the solve to 1e-8 with
    the same properties.
C5 -- backward-Euler transient A = G + C/h on the C2 grid (1000 x 1000), 1 %
  PULSE sources, ILU(0) factored once, warm start: 1000 steps on the device;
  by causality its first K5 = 50 steps must be bit-identical to the
  order-matched restated step driver run for 50 steps; the 1000-step run is repeated
  bit for bit, and its iteration total and port waveforms are checked for
  size-independent properties.
"""
import numpy as np
import pytest

import ggmres
import oracle as O
from ggmres import host, matrices as M
from ggmres.dd import DD
from helpers import device_layout, rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

HIST_RTOL = 1e-10
# inner iterations of the parity run at 10M rows: the order-matched oracle takes
# ~2 s per iteration there (serial C), so the run is cut by max_iter inside the
# first GMRES(30) cycle -- which also exercises the mid-cycle Update of x
K1 = 12
# C5 steps re-run by the order-matched step driver (~0.6 s per step at 1M rows)
K5 = 50


def _check_cycle(g, o, ot):
    """first-cycle parity: bit-identical to the order-matched oracle `ot`,
    within 1e-10 (north_star) of the serial-order oracle `o`"""
    assert g["ret"] == ot["ret"] == o["ret"] == 1
    assert g["iters"] == ot["iters"] == o["iters"] == K1
    assert np.array_equal(g["hist"], ot["hist"])
    assert np.array_equal(g["x"], ot["x"])
    scale = np.max(np.abs(o["hist"]))
    assert np.max(np.abs(g["hist"] - o["hist"])) <= HIST_RTOL * scale
    assert rel_err(g["x"], o["x"]) <= HIST_RTOL


def _check_converged(g, A, L, U, b, x_of):
    assert g["ret"] == 0 and g["relres"] < 1e-8
    h = g["hist"]
    assert np.all(np.isfinite(h)) and h[0] == pytest.approx(1.0, rel=1e-12)
    assert h[-1] < 1e-8 and h.shape[0] >= g["inner"]
    normb = np.linalg.norm(O.lusolve(L, U, b))
    true = np.linalg.norm(O.lusolve(L, U, b - A @ x_of(g["x"]))) / normb
    assert true < 1e-7, true


@pytest.fixture(scope="module")
def c4():
    A = M.grid_7pt(216)
    assert A.shape[0] == 10_077_696 and A.nnz == 70_263_936
    return A


def test_c4_single_gpu_full_size(c4):
    A = c4
    n = A.shape[0]
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    assert s.uses_wavefront
    g = s.solve(b, restart=30, max_iter=K1, tol=1e-300)
    o = O.gmres_left(A, L, U, b, m=30, max_iter=K1, tol=1e-300)
    O.set_dot_order(*device_layout(n, 216, 216))
    try:
        ot = O.gmres_left(A, L, U, b, m=30, max_iter=K1, tol=1e-300)
    finally:
        O.set_dot_order(None)
    _check_cycle(g, o, ot)
    g = s.solve(b, restart=30, max_iter=5000, tol=1e-8)
    _check_converged(g, A, L, U, b, lambda x: x)
    s.close()


def test_c4_sharded_8_full_size(c4):
    A = c4
    b = M.rhs_ones(A)
    d = DD(8, device=0)
    d.set_system(A, host.PART_BLOCKS)
    inf = d.info()
    assert inf["nparts"] == 8 and inf["shards_here"] == 8
    assert inf["wave_interior"] == 3 and inf["wave_separator"] == 3
    assert inf["nsep"] == 7 * 2 * 216 * 216           # 7 cuts, both sides of each
    pinv, q = d.perm()
    B = host.permute(A, pinv, q)
    L, U = O.ilu0(B)
    g = d.solve(b, restart=30, max_iter=K1, tol=1e-300)
    o = O.gmres_left(B, L, U, b[q], m=30, max_iter=K1, tol=1e-300)
    segs, G = zip(*[d.dot_layout(p) for p in range(8)])
    O.set_dot_order_shards(list(segs), G[0])
    try:
        ot = O.gmres_left(B, L, U, b[q], m=30, max_iter=K1, tol=1e-300)
    finally:
        O.set_dot_order(None)
    g = dict(g, x=g["x"][q])
    _check_cycle(g, o, ot)
    g = d.solve(b, restart=30, max_iter=5000, tol=1e-8)
    _check_converged(dict(g, x=g["x"][q]), B, L, U, b[q], lambda x: x)
    d.close()


def test_c5_transient_1000_steps_c2_grid():
    h = 1e-2
    A = M.transient(M.laplacian_5pt(1000), c=1e-3, h=h)
    n = A.shape[0]
    cdiag = np.full(n, 1e-3 / h)
    nodes, pulses = M.pulse_sources(n, frac=0.01, h=h)
    ports = np.array([int(nodes[0]), int(nodes[len(nodes) // 2]), n // 2, n - 1], np.int32)
    x0 = np.zeros(n)
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_ilu0()
    assert s.uses_wavefront
    g = s.transient(1000, h, cdiag, nodes, pulses, ports, x0, restart=32, max_iter=10000, tol=1e-7)
    g2 = s.transient(1000, h, cdiag, nodes, pulses, ports, x0, restart=32, max_iter=10000, tol=1e-7)
    assert g2["iters_total"] == g["iters_total"]
    assert np.array_equal(g2["ports"], g["ports"]) and np.array_equal(g2["x"], g["x"])
    # causality: the first K5 steps of the 1000-step run == a K5-step run of
    # the restated step driver (order-matched dots), bit for bit
    L, U = O.ilu0(A)
    O.set_dot_order(*device_layout(n, 1000))
    try:
        ot = O.transient(A, L, U, K5, h, cdiag, nodes, pulses, ports, x0, m=32, max_iter=10000, tol=1e-7)
    finally:
        O.set_dot_order(None)
    assert np.array_equal(g["ports"][:, :K5 + 1], ot["ports"])
    s100 = s.transient(K5, h, cdiag, nodes, pulses, ports, x0, restart=32, max_iter=10000, tol=1e-7)
    assert s100["iters_total"] == ot["iters_total"] and np.array_equal(s100["x"], ot["x"])
    # the serial-order driver agrees within 1e-10 over the first 10 steps
    o10 = O.transient(A, L, U, 10, h, cdiag, nodes, pulses, ports, x0, m=32, max_iter=10000, tol=1e-7)
    pv = g["ports"][:, :11]
    assert np.max(np.abs(pv - o10["ports"])) <= 1e-10 * np.max(np.abs(o10["ports"]))
    # properties of the whole run: finite, driven (the PULSE sources have period
    # 400 h, so the 1000 steps cover 2.5 periods), every step converged
    P = g["ports"]
    assert np.all(np.isfinite(P)) and np.max(np.abs(P)) > 0
    assert g["ret"] == 0 and g["iters_total"] >= 1000
    # the source nodes respond within the first pulse (td 0, rise 10 h)
    assert np.all(np.abs(P[:2, 20]) > 0)
    s.close()


# --------------------------------------------------------------- C3, ILU(k=1)
C3_ILU1_PATTERN = 234_215_488


def test_c3_standin_iluk1_full_size():
    """C3 -- the circuit5M stand-in (seeded power-law CSR with circuit5M's n and
    nnz, uniform columns: 5,558,326 rows, 59.5M entries; the SuiteSparse file
    is not available offline) with the ILU(1) preconditioner C3 names, at full
    size.  The factors: the level-1 pattern (234,215,488 entries with the
    diagonal: A's pattern united with U_A(k) over k in L_A(i), counted with
    scipy outside the product), unit lower L, nonzero pivots on U's diagonal,
    L*U reproducing A on A's pattern (ILU's defining property) on a sample of
    rows.  The solve: GMRES(30) to 1e-10, history monotone inside the first
    cycle, true residual ||b - A x|| / ||b|| < 1e-8.  Bit-exactness of the device factors against the oracle is pinned
    at covered sizes (test_gpu_parity.py::test_iluk_device_factors_bitexact,
    incl. the hub-row path)."""
    import scipy.sparse as sp
    A = M.power_law()
    n = A.shape[0]
    solver = ggmres.Solver(0)
    solver.set_matrix(A)
    (lrp, lci, lv), (urp, uci, uv), ms = solver.iluk_device_factors(1)
    assert ms > 0
    L = sp.csr_matrix((lv, lci, lrp), shape=(n, n))
    U = sp.csr_matrix((uv, uci, urp), shape=(n, n))
    # the level-1 pattern (diagonal included): 234,215,488 entries, counted
    # independently with scipy (pattern of tril(A,-1) @ triu(A,1) united with A's)
    assert L.nnz + U.nnz - n == C3_ILU1_PATTERN
    assert sp.tril(L, -1).nnz + sp.triu(U, 1).nnz + n == C3_ILU1_PATTERN
    assert np.array_equal(L.diagonal(), np.ones(n))
    assert np.all(U.diagonal() != 0)
    # ILU(1): (L U)_ij = a_ij on A's pattern up to rounding (a sample of rows)
    rows = np.random.default_rng(3).choice(n, 2000, replace=False)
    LU = (L[rows] @ U).tocsr()
    Ar = A[rows].tocsr()
    d = np.asarray(abs(LU - Ar).multiply(Ar != 0).max(axis=1).todense()).ravel()
    scale = np.asarray(abs(Ar).max(axis=1).todense()).ravel()
    assert np.all(d <= 1e-11 * scale)
    # GMRES(30) + ILU(1) to 1e-10
    solver.set_precond_iluk_device(1)
    b = M.rhs_ones(A)
    g = solver.solve(b, restart=30, max_iter=300, tol=1e-10)
    assert g["ret"] == 0 and g["relres"] < 1e-10
    h = g["hist"]
    assert np.all(np.isfinite(h)) and h[0] == pytest.approx(1.0, rel=1e-12)
    assert np.all(np.diff(h[: min(30, len(h))]) <= 1e-12)        # monotone inside the first cycle
    solver.close()
    r = b - A @ g["x"]
    assert np.linalg.norm(r) / np.linalg.norm(b) < 1e-8
