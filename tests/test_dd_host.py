"""Sharded solve, CPU: the product's host decomposition
(gg_host_dd_*, csrc/host/dd_setup.cpp) run through the CPU restatement of the
sharded algorithm (oracle/dd.py) against the global restatement on the
arrow-permuted matrix B = P A P^T -- in one process and over a 2-rank gloo
process group (the N > 1 path's exchanges: interface all-gathers, dot
partial all-gathers)."""
import os
import socket

import numpy as np
import pytest

import oracle as O
from oracle import dd as ODD
from conftest import fixture_path
from ggmres import host, matrices as M

CASES = {
    "5pt_40x30_P2_blocks": (lambda: M.laplacian_5pt(40, 30), 2, host.PART_BLOCKS),
    "5pt_40x30_P3_blocks": (lambda: M.laplacian_5pt(40, 30), 3, host.PART_BLOCKS),
    "5pt_30x30_P4_bisect": (lambda: M.laplacian_5pt(30, 30), 4, host.PART_BISECT),
    "7pt_10cube_P2_blocks": (lambda: M.grid_7pt(10), 2, host.PART_BLOCKS),
    "7pt_12cube_P4_bisect_upwind": (lambda: M.grid_7pt(12, upwind=0.1), 4, host.PART_BISECT),
    "sherman1_P4_bisect": (lambda: M.read_rua(fixture_path("sherman1.rua")), 4, host.PART_BISECT),
    "9pt_10x10_P2_bisect": (lambda: M.read_mtx(fixture_path("9pt_10x10.mtx")), 2, host.PART_BISECT),
}


def setup(name):
    make, P, method = CASES[name]
    A = make()
    plan = host.DDPlan(A, P, method)
    B = host.permute(A, plan.pinv, plan.q)
    shards = [ODD.Shard(plan.shard(p), p, P, plan.max_iface) for p in range(P)]
    g = ODD.Group(shards, P, lambda parts: parts)        # every shard in this process
    return A, B, plan, g


def gather(g, vs, n):
    out = np.full(n, np.nan)
    for s, v in zip(g.sh, vs):
        out[s.s["rows"]] = v[: s.nloc]
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_plan_structure(name):
    A, B, plan, g = setup(name)
    n, P = plan.n, plan.P
    assert plan.part_size.sum() == n and plan.nsep == plan.part_size[P]
    # every row appears exactly once as an interior row, the separator on every shard
    interior = np.concatenate([s.s["rows"][: s.nI] for s in g.sh])
    assert np.array_equal(np.sort(interior), np.arange(plan.begin[P]))
    for s in g.sh:
        assert np.array_equal(s.s["rows"][s.nI:], np.arange(plan.begin[P], n))
        assert len(s.s["iface"]) <= plan.max_iface
    # the local A reassembles B (halo columns map back to the owners' interface nodes)
    Bd = B.toarray()
    for s in g.sh:
        Al = s.s["A"].toarray()
        cols = np.concatenate([s.s["rows"], np.full(P * plan.max_iface, -1)])
        for q in g.sh:
            base = s.nloc + q.p * plan.max_iface
            cols[base: base + len(q.s["iface"])] = q.s["rows"][q.s["iface"]]
        for r, gr in enumerate(s.s["rows"]):
            nz = np.nonzero(Al[r])[0]
            assert np.all(cols[nz] >= 0)
            assert np.array_equal(np.sort(cols[nz]), np.nonzero(Bd[gr])[0])
            assert np.array_equal(Al[r, nz][np.argsort(cols[nz])], Bd[gr, np.nonzero(Bd[gr])[0]])


@pytest.mark.parametrize("name", sorted(CASES))
def test_sharded_spmv_and_ilu_apply_bitexact(name):
    A, B, plan, g = setup(name)
    n = plan.n
    rng = np.random.default_rng(5)
    xB = rng.standard_normal(n)
    ys = g.spmv([s.local(xB) for s in g.sh])
    assert np.array_equal(gather(g, ys, n), O.spmv(B, xB))
    L, U = O.ilu0(B)
    yB = rng.standard_normal(n)
    zs = g.apply([s.local(yB) for s in g.sh])
    for s, z in zip(g.sh, zs):                    # every separator replica is identical
        assert np.array_equal(z[s.nI: s.nloc], zs[0][g.sh[0].nI: g.sh[0].nloc])
    assert np.array_equal(gather(g, zs, n), O.lusolve(L, U, yB))


@pytest.mark.parametrize("name", ["5pt_40x30_P3_blocks", "7pt_10cube_P2_blocks", "sherman1_P4_bisect"])
def test_sharded_gmres_matches_global(name):
    A, B, plan, g = setup(name)
    n = plan.n
    b = M.rhs_ones(A)
    bB = b[plan.q]
    L, U = O.ilu0(B)
    ref = O.gmres_left(B, L, U, bB, m=30, max_iter=600, tol=1e-10)
    out = ODD.gmres_left(g, [s.local(bB) for s in g.sh], [s.local(np.zeros(n)) for s in g.sh],
                         m=30, max_iter=600, tol=1e-10)
    assert out["ret"] == ref["ret"] and out["iters"] == ref["iters"]
    h, hr = out["hist"], ref["hist"]
    assert h.shape == hr.shape
    assert np.max(np.abs(h - hr)) <= 1e-10 * np.max(np.abs(hr))      # north_star: 1e-10
    x = gather(g, out["x"], n)
    assert np.linalg.norm(x - ref["x"]) <= 1e-10 * np.linalg.norm(ref["x"])


# ---------------------------------------------------------------- gloo, 2 ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, name):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "gpu-gmres_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import oracle as O
    from oracle import dd as ODD
    from ggmres import host, matrices as M
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        A = M.laplacian_5pt(30, 24) if name == "5pt" else M.grid_7pt(9, upwind=0.1)
        plan = host.DDPlan(A, world, host.PART_BLOCKS if name == "5pt" else host.PART_BISECT)
        B = host.permute(A, plan.pinv, plan.q)
        me = ODD.Shard(plan.shard(rank), rank, world, plan.max_iface)

        def ag(parts):                              # one shard per process
            t = torch.from_numpy(np.ascontiguousarray(parts[0]))
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return [o.numpy() for o in out]

        g = ODD.Group([me], world, ag)
        n = plan.n
        rows = me.s["rows"]
        rng = np.random.default_rng(11)
        xB = rng.standard_normal(n)
        y = g.spmv([me.local(xB)])[0]
        assert np.array_equal(y[: me.nloc], O.spmv(B, xB)[rows])
        L, U = O.ilu0(B)
        z = g.apply([me.local(xB)])[0]
        assert np.array_equal(z[: me.nloc], O.lusolve(L, U, xB)[rows])
        bB = M.rhs_ones(A)[plan.q]
        ref = O.gmres_left(B, L, U, bB, m=20, max_iter=400, tol=1e-10)
        out = ODD.gmres_left(g, [me.local(bB)], [me.local(np.zeros(n))], m=20, max_iter=400, tol=1e-10)
        assert out["ret"] == ref["ret"] == 0 and out["iters"] == ref["iters"]
        assert out["hist"].shape == ref["hist"].shape
        assert np.max(np.abs(out["hist"] - ref["hist"])) <= 1e-10 * np.max(np.abs(ref["hist"]))
        xr = ref["x"][rows]
        assert np.linalg.norm(out["x"][0][: me.nloc] - xr) <= 1e-10 * np.linalg.norm(xr)
        # every rank holds the same Hessenberg decisions: identical histories
        h = torch.from_numpy(out["hist"])
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        assert all(torch.equal(hs[0], t) for t in hs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["5pt", "7pt"])
def test_gloo_two_ranks(name):
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(2, _free_port(), name), nprocs=2, join=True)
