"""The bordered-grid wavefront (gg_internal.h Wave2D::bnt, DevTri::tail): the
split engine on an MNA power-grid system pivoted with its pads and voltage-
source branch rows first (ggmres.matrices.mna_pivot_order -- the reference's
PG workload, src/mna_solve_gpu_gmres.cpp:190-647, with ILU(0) of the pivoted
system in place of ILU++).  The tail rows run in the flow kernel, the grid
block in the 2D wavefront, the grid rows' tail terms in k_border_sub between
them -- each row in the reference's canonical order (MyILUPP::HostPrecond_left
/ _right, src/preconditioner.cu:1094-1137), so every operator is bit-identical
to the oracle and GMRES to the order-matched oracle."""
import os

import numpy as np
import pytest

import ggmres
import oracle as O
from helpers import device_layout, make_split, netlist_system, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def systems(tmp_path_factory):
    d = tmp_path_factory.mktemp("pg")
    out = {}
    for grid, stride in ((60, 20), (150, 50)):
        A, prow, pcol, nt = netlist_system(os.path.join(d, f"pg{grid}.sp"), grid, stride)
        out[grid] = (A, make_split(A, seed=3, perm=(prow, pcol)), nt)
    return out


def split_solver(A, P):
    s = ggmres.Solver(0)
    s.set_matrix(A)
    s.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
    return s


@pytest.mark.parametrize("grid", [60, 150])
def test_border_operators_bitexact(systems, grid):
    A, P, nt = systems[grid]
    s = split_solver(A, P)
    try:
        assert s.uses_wavefront
        # the tail's levels on top of the grid's wavefront steps
        assert s.trsv_levels(0) > grid + grid - 1 and s.trsv_levels(1) > grid + grid - 1
        rng = np.random.default_rng(6)
        for scale in (1.0, 1e200, 1e-200):
            v = rng.standard_normal(A.shape[0]) * scale
            assert np.array_equal(s.precond_apply(ggmres.APPLY_LEFT, v), P.left(v))
            assert np.array_equal(s.precond_apply(ggmres.APPLY_RIGHT, v), P.right(v))
            assert np.array_equal(s.precond_apply(ggmres.APPLY_START, v), P.start(v))
        x = rng.standard_normal(A.shape[0])
        assert np.array_equal(s.spmv(x), O.spmv(A, x))
    finally:
        s.close()


@pytest.mark.parametrize("grid", [60, 150])
def test_border_gmres_parity(systems, grid):
    """serial oracle within tolerance; order-matched oracle in the bordered
    layout bit for bit"""
    A, P, nt = systems[grid]
    n = A.shape[0]
    b = np.random.default_rng(1).random(n)
    run = lambda: O.gmres_split(A, P, b, m=32, max_iter=600, tol=1e-10)
    o = run()
    lay, G = device_layout(n, grid, border=nt)
    O.set_dot_order(lay, G)
    try:
        ot = run()
    finally:
        O.set_dot_order(None)
    s = split_solver(A, P)
    try:
        g = s.solve(b, restart=32, max_iter=600, tol=1e-10)
        assert g["ret"] == o["ret"] and g["iters"] == o["iters"]
        assert rel_err(g["x"], o["x"]) <= 1e-9
        assert g["ret"] == ot["ret"] and g["iters"] == ot["iters"] and g["inner"] == ot["inner"]
        assert np.array_equal(g["hist"], ot["hist"])
        assert np.array_equal(g["x"], ot["x"])
    finally:
        s.close()


def order_matched(A, P, b, n, grid, nt, mode_l, mode_u, tail, vs=()):
    lay, G = device_layout(n, grid, border=nt)
    O.set_dot_order(lay, G)
    O.set_div_mode(mode_l, mode_u)
    O.set_fma_tail(tail)
    try:
        ot = O.gmres_split(A, P, b, m=32, max_iter=600, tol=1e-10)
        ops = [(P.left(v), P.right(v)) for v in vs]
    finally:
        O.set_dot_order(None)
        O.set_div_mode()
        O.set_fma_tail(0)
    return ot, ops


@pytest.mark.parametrize("grid", [60, 150])
def test_border_mul_division(systems, grid):
    """gg_set_division(GG_DIV_RCP) on a bordered grid: x = RN(acc * RN(1/d)) on
    every row -- the mesh's wavefront (WD_MUL) and the tail's flow kernel alike.
    Under GG_DIV_FMA the non-unit L (whose fused rows would need the tail terms
    inside RN(b * y)) takes the multiply too, the U the fused rows.  Bit-exact
    vs the order-matched oracle in those modes, within 1e-10 of the serial
    reference arithmetic."""
    A, P, nt = systems[grid]
    n = A.shape[0]
    b = np.random.default_rng(1).random(n)
    o = O.gmres_split(A, P, b, m=32, max_iter=600, tol=1e-10)
    rng = np.random.default_rng(7)
    vs = [rng.standard_normal(n) for _ in range(2)]
    s = split_solver(A, P)
    try:
        for mode, want_u, mode_u in ((ggmres.DIV_RCP, ggmres.DIV_RCP, 1), (ggmres.DIV_FMA, ggmres.DIV_FMA, 2)):
            ot, ref_ops = order_matched(A, P, b, n, grid, nt, 1, mode_u, nt, vs)
            s.set_division(mode)
            assert s.division_active(0) == ggmres.DIV_RCP and s.division_active(1) == want_u
            for v, (l, r) in zip(vs, ref_ops):
                assert np.array_equal(s.precond_apply(ggmres.APPLY_LEFT, v), l)
                assert np.array_equal(s.precond_apply(ggmres.APPLY_RIGHT, v), r)
            g = s.solve(b, restart=32, max_iter=600, tol=1e-10)
            assert g["iters"] == ot["iters"] and np.array_equal(g["hist"], ot["hist"])
            assert np.array_equal(g["x"], ot["x"])
            # (the serial engine divides: the convergence test may fire one iteration apart)
            assert abs(g["iters"] - o["iters"]) <= 1 and rel_err(g["x"], o["x"]) <= 1e-8
    finally:
        s.close()


@pytest.mark.parametrize("grid", [60, 150])
def test_border_fma_unit_l(systems, grid, tmp_path):
    """The bench's netlist split (ILU(0) of the pivoted B: unit L, unit scales)
    under GG_DIV_FMA: both triangles fused -- the mesh rows' tail terms first
    (k_border_sub, fused), then the wavefront's rows; the tail rows fused in
    the flow kernel (pre-scaled, nearest term first).  Bit-exact vs the
    order-matched oracle in FMA mode with orc_set_fma_tail, within 1e-10 of
    the serial reference arithmetic."""
    A, P0, nt = systems[grid]
    n = A.shape[0]
    import scipy.sparse as sp
    prow, pcol = P0.perm_row, P0.perm_col
    Pr = sp.csr_matrix((np.ones(n), (np.arange(n), prow)), shape=(n, n))
    Pc = sp.csr_matrix((np.ones(n), (np.arange(n), pcol)), shape=(n, n))
    B = (Pr @ A @ Pc).tocsr()
    B.sort_indices()
    Lt, Ut = O.ilu0(B)
    ones = np.ones(n)
    P = O.Split(Lt, Ut, ones, prow, pcol, ones, ones)
    b = np.random.default_rng(2).random(n)
    o = O.gmres_split(A, P, b, m=32, max_iter=600, tol=1e-10)
    rng = np.random.default_rng(9)
    vs = [rng.standard_normal(n) for _ in range(2)]
    ot, ref_ops = order_matched(A, P, b, n, grid, nt, 2, 2, nt, vs)
    s = split_solver(A, P)
    try:
        s.set_division(ggmres.DIV_FMA)
        assert s.division_active(0) == s.division_active(1) == ggmres.DIV_FMA
        for v, (l, r) in zip(vs, ref_ops):
            assert np.array_equal(s.precond_apply(ggmres.APPLY_LEFT, v), l)
            assert np.array_equal(s.precond_apply(ggmres.APPLY_RIGHT, v), r)
        g = s.solve(b, restart=32, max_iter=600, tol=1e-10)
        assert g["iters"] == ot["iters"] and np.array_equal(g["hist"], ot["hist"])
        assert np.array_equal(g["x"], ot["x"])
        assert abs(g["iters"] - o["iters"]) <= 1 and rel_err(g["x"], o["x"]) <= 1e-8
    finally:
        s.close()


def test_no_border_flow_kernel_same_bits(systems, monkeypatch):
    """GG_NO_BORDER=1: every row in the flow kernel, natural layout -- the
    order-matched oracle in natural order, bit for bit"""
    A, P, nt = systems[60]
    n = A.shape[0]
    b = np.random.default_rng(1).random(n)
    lay, G = device_layout(n)
    O.set_dot_order(lay, G)
    try:
        ot = O.gmres_split(A, P, b, m=32, max_iter=300, tol=1e-10)
    finally:
        O.set_dot_order(None)
    monkeypatch.setenv("GG_NO_BORDER", "1")
    monkeypatch.setenv("GG_FLOW_RCM", "0")          # the natural layout (the RCM one: test_gpu_parity)
    s = split_solver(A, P)
    try:
        assert not s.uses_wavefront and s.trsv_kernel(0) == "k_trsv_flow"
        g = s.solve(b, restart=32, max_iter=300, tol=1e-10)
    finally:
        s.close()
    assert g["iters"] == ot["iters"] and np.array_equal(g["hist"], ot["hist"])
    assert np.array_equal(g["x"], ot["x"])
