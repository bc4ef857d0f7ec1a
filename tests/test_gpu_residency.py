"""Persistent grids that do not fit the chip ("stop trusting the
occupancy API"; ADVICE r3 on the fused SpMV's block order).

* k_arnoldi_persist / k_arnoldi_wide: a launch whose blocks cannot all be
  resident aborts its cycle (kernels.hip gather_first: DONE_ABORT), the host
  restores the control block and reruns the cycle on the per-step kernels --
  forced here with dynamic LDS (GG_PERSIST_TEST_LDS) so that fewer blocks fit
  than the grid has.  Results bit-identical to the per-step kernels and to the
  order-matched oracle.
* k_trsv_tile3d: tiles dealt statically; a grid that is not co-resident times
  out (err bit 3) and the solve / apply repeats with tiles claimed from a queue
  (no co-residency needed) -- forced with more workgroups than can be resident
  (GG_TILE_GRID); GG_TILE_QUEUE=1 runs the queue from the start.
* k_trsv_wave2d_spmv: the SpMV blocks take the low block indices, so a grid with
  more bands than CUs still drains.
"""
import numpy as np
import pytest

import ggmres
import oracle as O
from ggmres import matrices as M
from helpers import device_layout

pytestmark = pytest.mark.gpu


def solve(A, b, env, monkeypatch, m=30, max_iter=40, tol=1e-300, division=None):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = ggmres.Solver(0)
    try:
        if division is not None:
            s.set_division(division)
        s.set_matrix(A)
        s.set_precond_ilu0()
        g = s.solve(b, restart=m, max_iter=max_iter, tol=tol)
        g["mgs_kernel"] = s.mgs_kernel()
    finally:
        s.close()
        for k in env:
            monkeypatch.delenv(k, raising=False)
    return g


def same(g, e):
    assert g["ret"] == e["ret"] and g["iters"] == e["iters"] and g["inner"] == e["inner"]
    assert np.array_equal(g["hist"], e["hist"])
    assert np.array_equal(g["x"], e["x"])


@pytest.mark.parametrize("lds", [65536, 98304])
def test_persist_grid_not_coresident_reruns_per_step(monkeypatch, lds):
    """C2 (G = 544 blocks of k_arnoldi_persist<4>): with 64 / 96 KiB of dynamic
    LDS per block only 512 / 256 fit, the first cycle aborts and reruns on the
    per-step kernels -- the same bits as a solver that never persisted"""
    A = M.laplacian_5pt(1000)
    b = M.rhs_ones(A)
    ref = solve(A, b, {"GG_NO_PERSIST": "1"}, monkeypatch)
    base = solve(A, b, {}, monkeypatch)
    assert base["mgs_kernel"].startswith("k_arnoldi_persist")
    g = solve(A, b, {"GG_PERSIST_TEST_LDS": str(lds)}, monkeypatch)
    assert g["mgs_kernel"] == ""                 # dropped for the solver's life
    same(base, ref)
    same(g, ref)


def test_wide_grid_not_coresident_reruns_per_step(monkeypatch):
    """k_arnoldi_wide (512 blocks, 2 per CU) with 40 KiB more LDS per block: one
    per CU fits, the cycle aborts and reruns -- bit-identical to the oracle in
    the 512-block reduction order, over several restart cycles"""
    A = M.laplacian_5pt(100)
    n = A.shape[0]
    b = M.rhs_uniform(n)
    L, U = O.ilu0(A)
    lay, _ = device_layout(n, 100)
    O.set_dot_order(lay, 512)
    try:
        ot = O.gmres_left(A, L, U, b, m=30, max_iter=100, tol=1e-10)
    finally:
        O.set_dot_order(None)
    g = solve(A, b, {"GG_WIDE_FORCE": "1", "GG_PERSIST_TEST_LDS": "40960"}, monkeypatch, max_iter=100,
              tol=1e-10)
    assert g["mgs_kernel"] == ""
    same(g, ot)


@pytest.mark.parametrize("queue", [False, True])
@pytest.mark.parametrize("dims, grid", [((4, 200, 200), 625), ((3, 300, 300), 1444)])
def test_tile_queue_drains_oversized_grid(monkeypatch, dims, grid, queue):
    """3D tile solve with one workgroup per tile (625 / 1,444 > the 512 that can
    be resident): dealt statically it times out and falls back to the queue
    (queue False), or runs the queue from the start (True); every apply
    bit-exact vs the oracle, the queue re-armed launch after launch"""
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz, upwind=0.1)
    n = A.shape[0]
    L, U = O.ilu0(A)
    monkeypatch.setenv("GG_TILE_GRID", str(grid))
    if queue:
        monkeypatch.setenv("GG_TILE_QUEUE", "1")
    s = ggmres.Solver(0)
    try:
        s.set_matrix(A)
        s.set_precond_ilu0()
        assert s.uses_wavefront and s.trsv_kernel(0).startswith("k_trsv_tile3d")
        rng = np.random.default_rng(4)
        for _ in range(3):
            y = rng.standard_normal(n)
            assert np.array_equal(s.precond_apply(ggmres.APPLY_MINV, y), O.lusolve(L, U, y))
        b = M.rhs_uniform(n)
        lay, G = device_layout(n, nx, ny)
        O.set_dot_order(lay, G)
        try:
            ot = O.gmres_left(A, L, U, b, m=30, max_iter=45, tol=1e-300)
        finally:
            O.set_dot_order(None)
        same(s.solve(b, restart=30, max_iter=45, tol=1e-300), ot)
    finally:
        s.close()


def test_fused_spmv_more_bands_than_cus(monkeypatch):
    """A 2D grid of 16,448 lines = 257 bands, one workgroup per CU: the fused
    forward solve (SpMV blocks first) drains and gives the separate launch's
    bits"""
    A = M.laplacian_5pt(12, 16448)
    n = A.shape[0]
    b = M.rhs_uniform(n)
    g = solve(A, b, {}, monkeypatch, max_iter=35, division=ggmres.DIV_FMA)
    e = solve(A, b, {"GG_FUSE_SPMV": "0"}, monkeypatch, max_iter=35, division=ggmres.DIV_FMA)
    same(g, e)
    L, U = O.ilu0(A)
    lay, G = device_layout(n, 12)
    O.set_dot_order(lay, G)
    O.set_div_mode(2, 2)
    try:
        ot = O.gmres_left(A, L, U, b, m=30, max_iter=35, tol=1e-300)
    finally:
        O.set_dot_order(None)
        O.set_div_mode()
    same(g, ot)
