"""GPU parity of the sharded solve (include/ggmres_dd.h).

All shards of a P-way decomposition run in one process on one GPU
(GG_DD_LOCAL: the same kernels and the same exchange points as one process
per GPU over RCCL; the exchanges are done by a copy kernel), checked against
the oracle on the arrow-permuted matrix B = P A P^T:
  * SpMV and the ILU(0) apply: bit-exact vs oracle.spmv(B) / lusolve(ilu0(B));
  * GMRES: bit-identical history, iteration count and solution vs the oracle
    run with the sharded reduction order (oracle.set_dot_order_shards), and
    within 1e-10 (north_star) of the serial-order oracle.
The RCCL communicator is exercised with one rank (the GPU box has one GPU).
"""
import numpy as np
import pytest

import oracle as O
from conftest import fixture_path
from ggmres import host, matrices as M
from ggmres.dd import DD, unique_id

pytestmark = pytest.mark.gpu

CASES = {
    # name: (matrix, parts, method, expect wavefront interior / separator (0, 2 or 3))
    "5pt_200x160_P2": (lambda: M.laplacian_5pt(200, 160), 2, host.PART_BLOCKS, 2, 2),
    "5pt_200x160_P4": (lambda: M.laplacian_5pt(200, 160), 4, host.PART_BLOCKS, 2, 2),
    "7pt_24_P4": (lambda: M.grid_7pt(24), 4, host.PART_BLOCKS, 3, 3),
    "7pt_16x16x32_P8_upwind": (lambda: M.grid_7pt(16, 16, 32, upwind=0.1), 8, host.PART_BLOCKS, 3, 3),
    "7pt_16_P4_bisect": (lambda: M.grid_7pt(16), 4, host.PART_BISECT, None, None),
    "sherman1_P4": (lambda: M.read_rua(fixture_path("sherman1.rua")), 4, host.PART_BISECT, None, None),
    "5pt_60x60_P1": (lambda: M.laplacian_5pt(60, 60), 1, host.PART_BLOCKS, 2, 0),
    # the separator ordered by a greedy colouring (GG_PART_COLOR_SEP): a
    # few-level separator solve, fused with its coupling terms into one
    # dataflow launch (k_sep_flow, separator kind 1)
    "5pt_200x160_P4_color": (lambda: M.laplacian_5pt(200, 160), 4, host.PART_BLOCKS | host.PART_COLOR_SEP, 2, 1),
    "7pt_16x16x32_P8_upwind_color": (lambda: M.grid_7pt(16, 16, 32, upwind=0.1), 8,
                                     host.PART_BLOCKS | host.PART_COLOR_SEP, 3, 1),
    # px x py rectangles (GG_PART_GRID): rectangular interiors on the 2D
    # wavefront with chains of nx/px + ny/py steps, a cross-shaped separator
    "5pt_200x160_P4_grid": (lambda: M.laplacian_5pt(200, 160), 4, host.PART_GRID | host.PART_COLOR_SEP, 2, 1),
    "5pt_160x200_P8_grid": (lambda: M.laplacian_5pt(160, 200), 8, host.PART_GRID | host.PART_COLOR_SEP, 2, 1),
    # 2 x 2 x 2 boxes of a 3D grid: box interiors on the 3D tile wavefront
    "7pt_24_P8_grid": (lambda: M.grid_7pt(24), 8, host.PART_GRID | host.PART_COLOR_SEP, 3, 1),
}

_cache = {}


def setup(name):
    if name not in _cache:
        make, P, method, wi, ws = CASES[name]
        A = make()
        d = DD(P, device=0)
        d.set_system(A, method)
        pinv, q = d.perm()
        B = host.permute(A, pinv, q)
        L, U = O.ilu0(B)
        _cache[name] = (A, d, q, B, L, U)
    return _cache[name]


@pytest.mark.parametrize("name", sorted(CASES))
def test_dd_layout(name):
    A, d, q, B, L, U = setup(name)
    inf = d.info()
    _, P, _, wi, ws = CASES[name]
    assert inf["nparts"] == P and inf["shards_here"] == P
    if wi is not None:
        assert inf["wave_interior"] == wi, inf
        assert inf["wave_separator"] == ws, inf
    plan = host.DDPlan(A, P, CASES[name][2])          # the host plan agrees with the solver's
    assert np.array_equal(plan.q, q) and inf["nsep"] == plan.nsep


def test_dd_separator_four_launches_match_fused(monkeypatch):
    """GG_DD_SEPFLOW=0 keeps the four separator launches (k_sub_seq, two
    k_trsv_flow, k_sub_seq): the same bits as the fused step."""
    A, d, q, B, L, U = setup("5pt_200x160_P4_color")
    monkeypatch.setenv("GG_DD_SEPFLOW", "0")
    d0 = DD(4, device=0)
    d0.set_system(A, CASES["5pt_200x160_P4_color"][2])
    assert d0.info()["wave_separator"] == 0 and d.info()["wave_separator"] == 1
    rng = np.random.default_rng(11)
    v = rng.standard_normal(A.shape[0])
    z0, z1 = d0.precond_apply(v), d.precond_apply(v)
    assert np.array_equal(z0, z1)
    assert np.array_equal(z1[q], O.lusolve(L, U, v[q]))


@pytest.mark.parametrize("name", sorted(CASES))
def test_dd_spmv_and_apply_bitexact(name):
    A, d, q, B, L, U = setup(name)
    n = A.shape[0]
    rng = np.random.default_rng(3)
    x = rng.standard_normal(n)
    y = d.spmv(x)
    assert np.array_equal(y[q], O.spmv(B, x[q]))
    for scale in (1.0, 1e-250, 1e250):                  # WD_RCP range fallback on the U solves
        v = rng.standard_normal(n) * scale
        z = d.precond_apply(v)
        assert np.array_equal(z[q], O.lusolve(L, U, v[q])), scale


@pytest.mark.parametrize("name", sorted(CASES))
def test_dd_gmres_bitexact_order_matched(name):
    A, d, q, B, L, U = setup(name)
    P = CASES[name][1]
    b = M.rhs_ones(A)
    g = d.solve(b, restart=30, max_iter=1500, tol=1e-10)
    segs, G = zip(*[d.dot_layout(p) for p in range(P)])
    O.set_dot_order_shards(list(segs), G[0])
    try:
        ref_t = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
    finally:
        O.set_dot_order(None)
    ref = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
    assert g["ret"] == ref_t["ret"] == 0
    assert g["iters"] == ref_t["iters"]
    assert np.array_equal(g["hist"], ref_t["hist"])
    assert np.array_equal(g["x"][q], ref_t["x"])
    check_serial(g, ref, x_g=g["x"][q], tol=1e-10)


def check_serial(g, ref, x_g, tol):
    """Device vs the serial-order oracle (north_star: history within 1e-10 of
    its scale).  The reduction orders differ, so the last residuals differ by
    rounding (~1e-14 absolute after hundreds of iterations); when they straddle
    the tolerance the convergence test fires one iteration apart: then the
    common history must still agree within 1e-10 of its scale."""
    scale = np.max(np.abs(ref["hist"]))
    k = min(len(g["hist"]), len(ref["hist"]))
    assert np.max(np.abs(g["hist"][:k] - ref["hist"][:k])) <= 1e-10 * scale
    if g["iters"] == ref["iters"]:
        assert g["hist"].shape == ref["hist"].shape
        assert np.linalg.norm(x_g - ref["x"]) <= 1e-10 * np.linalg.norm(ref["x"])
    else:
        assert abs(g["iters"] - ref["iters"]) == 1, (g["iters"], ref["iters"])
        first, other = (g, ref) if g["iters"] < ref["iters"] else (ref, g)
        i = len(first["hist"]) - 1
        assert first["hist"][i] < tol * scale <= other["hist"][i] + 1e-10 * scale
        assert np.linalg.norm(x_g - ref["x"]) <= 1e-8 * np.linalg.norm(ref["x"])


def test_dd_restart_and_max_iter_semantics():
    A, d, q, B, L, U = setup("7pt_24_P4")
    b = M.rhs_uniform(A.shape[0])
    x0 = np.random.default_rng(9).standard_normal(A.shape[0])
    g = d.solve(b, x0=x0, restart=7, max_iter=40, tol=1e-14)       # cut by max_iter mid-cycle
    segs, G = zip(*[d.dot_layout(p) for p in range(4)])
    O.set_dot_order_shards(list(segs), G[0])
    try:
        ref = O.gmres_left(B, L, U, b[q], x0=x0[q], m=7, max_iter=40, tol=1e-14)
    finally:
        O.set_dot_order(None)
    assert g["ret"] == ref["ret"] == 1 and g["iters"] == ref["iters"] == 40
    assert np.array_equal(g["hist"], ref["hist"]) and np.array_equal(g["x"][q], ref["x"])


def test_dd_rccl_single_rank_matches_local():
    A = M.laplacian_5pt(64, 64)
    b = M.rhs_ones(A)
    loc = DD(1, device=0)
    loc.set_system(A, host.PART_BLOCKS)
    r0 = loc.solve(b, restart=30, max_iter=500, tol=1e-10)
    rc = DD(1, device=0, rank=0, uid=unique_id())
    rc.set_system(A, host.PART_BLOCKS)
    r1 = rc.solve(b, restart=30, max_iter=500, tol=1e-10)
    assert r0["iters"] == r1["iters"] and np.array_equal(r0["hist"], r1["hist"])
    assert np.array_equal(r0["x"], r1["x"])
    rc.close()
    loc.close()


# ---- GG_SOLVE_CGS2: three all-gathers per inner iteration ----------------------
CGS2_CASES = ["5pt_200x160_P2", "5pt_200x160_P4_color", "7pt_24_P4", "7pt_16x16x32_P8_upwind_color",
              "sherman1_P4", "5pt_60x60_P1"]


@pytest.mark.parametrize("name", CGS2_CASES)
def test_dd_cgs2_bitexact_and_tolerance(name):
    """CGS2 (h = V^T w, w -= V h, twice; H = h + h2) bit-identical to the oracle
    restating it in the sharded reduction order; its first restart cycle within
    1e-10 (north_star) of the reference's MGS in serial order; the full solve
    converges with a true preconditioned residual below the tolerance."""
    import ggmres
    A, d, q, B, L, U = setup(name)
    P = CASES[name][1]
    b = M.rhs_ones(A)
    segs, G = zip(*[d.dot_layout(p) for p in range(P)])
    # the first cycle: order-matched CGS2 bit for bit, serial MGS within 1e-10
    g1 = d.solve(b, restart=30, max_iter=30, tol=1e-300, flags=ggmres.SOLVE_CGS2)
    O.set_dot_order_shards(list(segs), G[0])
    O.set_orth(True)
    try:
        t1 = O.gmres_left(B, L, U, b[q], m=30, max_iter=30, tol=1e-300)
        tf = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
    finally:
        O.set_dot_order(None)
        O.set_orth()
    assert np.array_equal(g1["hist"], t1["hist"]) and np.array_equal(g1["x"][q], t1["x"])
    s1 = O.gmres_left(B, L, U, b[q], m=30, max_iter=30, tol=1e-300)       # serial MGS
    scale = np.max(np.abs(s1["hist"]))
    assert g1["hist"].shape == s1["hist"].shape
    assert np.max(np.abs(g1["hist"] - s1["hist"])) <= 1e-10 * scale
    assert np.linalg.norm(g1["x"][q] - s1["x"]) <= 1e-10 * np.linalg.norm(s1["x"])
    # to convergence
    g = d.solve(b, restart=30, max_iter=1500, tol=1e-10, flags=ggmres.SOLVE_CGS2)
    assert g["ret"] == tf["ret"] == 0 and g["iters"] == tf["iters"]
    assert np.array_equal(g["hist"], tf["hist"]) and np.array_equal(g["x"][q], tf["x"])
    ref = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
    assert abs(g["iters"] - ref["iters"]) <= max(2, ref["iters"] // 50), (g["iters"], ref["iters"])
    normb = np.linalg.norm(O.lusolve(L, U, b[q]))
    true = np.linalg.norm(O.lusolve(L, U, b[q] - O.spmv(B, g["x"][q]))) / normb
    assert true < 1e-9, true


@pytest.mark.parametrize("mode", ["rcp", "fma"])
@pytest.mark.parametrize("name", ["5pt_200x160_P2", "7pt_24_P4", "5pt_200x160_P4_color"])
def test_dd_division_rcp_tolerance(name, mode):
    """gg_dd_set_division(GG_DIV_RCP): the shards' wavefront solves multiply by
    RN(1/d); GG_DIV_FMA: the 2D interiors' rows are two fused multiply-adds (U
    pre-scaled by RN(1/d)); the first restart cycle within 1e-10 (north_star) of
    the serial oracle with the reference's division, the full solve converging
    in the same number of iterations (MGS and CGS2)."""
    import ggmres
    A, d, q, B, L, U = setup(name)
    b = M.rhs_ones(A)
    d.set_division(ggmres.DIV_RCP if mode == "rcp" else ggmres.DIV_FMA)
    try:
        for flags in (0, ggmres.SOLVE_CGS2):
            g1 = d.solve(b, restart=30, max_iter=30, tol=1e-300, flags=flags)
            s1 = O.gmres_left(B, L, U, b[q], m=30, max_iter=30, tol=1e-300)
            scale = np.max(np.abs(s1["hist"]))
            assert g1["hist"].shape == s1["hist"].shape
            assert np.max(np.abs(g1["hist"] - s1["hist"])) <= 1e-10 * scale
            assert np.linalg.norm(g1["x"][q] - s1["x"]) <= 1e-10 * np.linalg.norm(s1["x"])
            g = d.solve(b, restart=30, max_iter=1500, tol=1e-10, flags=flags)
            ref = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
            assert g["ret"] == ref["ret"] == 0
            assert abs(g["iters"] - ref["iters"]) <= max(2, ref["iters"] // 50), (g["iters"], ref["iters"])
    finally:
        d.set_division(ggmres.DIV_EXACT)


def test_single_solver_refuses_cgs2():
    import ggmres
    s = ggmres.Solver(0)
    A = M.laplacian_5pt(20)
    s.set_matrix(A)
    s.set_precond_ilu0()
    with pytest.raises(ggmres.GGError):
        s.solve(M.rhs_ones(A), restart=10, max_iter=20, flags=ggmres.SOLVE_CGS2)
    s.close()
