"""The sharded solve's exchange modes (csrc/dd.hip), each against the default.

* GG_DD_HALO_INLINE / GG_DD_HALO_FUSED: the SpMV's interface exchange in the
  same launch as the rows (IPC / loopback default, k_dd_spmv_x), as its own
  launch on the solver's stream, or on the second stream beside the interior
  rows, the separator rows after an event wait -- the same bits:
  SpMV, preconditioner apply and GMRES (history, iterations, solution), for a
  2D rectangle and a 3D box partition (GG_DD_LOCAL, every shard in this
  process).
* GG_DD_LOOPBACK (one rank's shard alone, every exchange pointed at its own
  buffers -- bench.py's per-rank timing mode): at P = 1 it is the whole
  system, bit-identical to GG_DD_LOCAL; at P > 1 its values are not the
  system's, but the interior rows of its SpMV reference only the rank's own
  interior and the separator replica, so they must equal the one-process
  run's rows, and a solve must run its iterations without a time-out or a
  non-finite value, identically in both halo modes.
"""
import numpy as np
import pytest

from ggmres import host, matrices as M
from ggmres.dd import DD

pytestmark = pytest.mark.gpu

CASES = {
    "5pt_200x160_P4_grid": (lambda: M.laplacian_5pt(200, 160), 4, host.PART_GRID | host.PART_COLOR_SEP),
    "7pt_24_P8_grid": (lambda: M.grid_7pt(24), 8, host.PART_GRID | host.PART_COLOR_SEP),
}


# halo forms: "fused" (default; IPC / loopback: exchange and rows in one
# launch, k_dd_spmv_x -- GG_DD_LOCAL has no fused form and runs "inline"),
# "inline" (the exchange as its own launch, then the rows), "stream2" (the
# exchange on the second stream beside the interior rows)
FORMS = {"fused": {}, "inline": {"GG_DD_HALO_FUSED": "0"}, "stream2": {"GG_DD_HALO_INLINE": "0"}}


def _make(monkeypatch, form, P, **kw):
    for k, v in FORMS[form].items():
        monkeypatch.setenv(k, v)                                       # read at gg_dd_create
    d = DD(P, device=0, **kw)
    for k in FORMS[form]:
        monkeypatch.delenv(k)
    return d


@pytest.mark.parametrize("name", sorted(CASES))
def test_halo_modes_bitexact(name, monkeypatch):
    make, P, method = CASES[name]
    A = make()
    n = A.shape[0]
    out = []
    for form in ("inline", "stream2"):
        d = _make(monkeypatch, form, P)
        d.set_system(A, method)
        rng = np.random.default_rng(5)
        x = rng.standard_normal(n)
        v = rng.standard_normal(n)
        g = d.solve(M.rhs_ones(A), restart=30, max_iter=2000, tol=1e-10)
        out.append((d.spmv(x), d.precond_apply(v), g))
        d.close()
    (s0, a0, g0), (s1, a1, g1) = out
    assert np.array_equal(s0, s1) and np.array_equal(a0, a1)
    assert g0["ret"] == g1["ret"] == 0 and g0["iters"] == g1["iters"]
    assert np.array_equal(g0["hist"], g1["hist"]) and np.array_equal(g0["x"], g1["x"])


def test_loopback_single_part_is_the_system(monkeypatch):
    A = M.laplacian_5pt(80, 70)
    loc = DD(1, device=0)
    loc.set_system(A, host.PART_BLOCKS)
    lb = DD(1, device=0, rank=0, comm="loopback")
    lb.set_system(A, host.PART_BLOCKS)
    b = M.rhs_ones(A)
    g, h = loc.solve(b, restart=30, max_iter=1500, tol=1e-10), lb.solve(b, restart=30, max_iter=1500, tol=1e-10)
    assert g["iters"] == h["iters"] and np.array_equal(g["hist"], h["hist"]) and np.array_equal(g["x"], h["x"])
    loc.close()
    lb.close()


@pytest.mark.parametrize("rank", [0, 3])
def test_loopback_rank_interior_rows_and_run(rank, monkeypatch):
    A = M.laplacian_5pt(200, 160)
    n = A.shape[0]
    P, method = 4, host.PART_GRID | host.PART_COLOR_SEP
    loc = DD(P, device=0)
    loc.set_system(A, method)
    pinv, q = loc.perm()
    nsep = loc.info()["nsep"]
    x = np.random.default_rng(3).standard_normal(n)
    ref = loc.spmv(x)
    res = []
    for form in FORMS:
        lb = _make(monkeypatch, form, P, rank=rank, comm="loopback")
        lb.set_system(A, method)
        y = lb.spmv(x, np.full(n, np.nan))
        own = ~np.isnan(y)
        # the rank's interior rows (permuted index below n - nsep) are the system's
        interior = own & (pinv < n - nsep)
        assert interior.sum() > 0
        assert np.array_equal(y[interior], ref[interior])
        g = lb.solve(M.rhs_ones(A), restart=30, max_iter=60, tol=1e-300)
        assert g["iters"] == 60 and np.all(np.isfinite(g["hist"])) and g["hist"][0] == pytest.approx(1.0)
        res.append((y, g))
        lb.close()
    (y0, g0) = res[0]
    own = ~np.isnan(y0)
    for y1, g1 in res[1:]:
        assert np.array_equal(y0[own], y1[own]) and np.array_equal(g0["hist"], g1["hist"])
    loc.close()
