"""The sharded solve across PROCESSES (include/ggmres_dd.h), on one GPU.

The GPU boxes of this pool have one GPU and RCCL refuses two ranks on one
device, so the one-shard-per-process control flow of csrc/dd.hip (rank
offsets, agree_max, the error all-gather, the halo exchange on the second
stream, one exchange per MGS dot, per-rank write-back) runs here over the
GG_DD_IPC communicator: P fresh processes (tests/dd_rank_worker.py), one
shard each, device-initiated all-gathers through hipIpc-mapped exchange
areas.  Each rank's results must be bit-identical to the same decomposition
run in one process (GG_DD_LOCAL) and to the oracle on the arrow-permuted
matrix B = P A P^T in the sharded reduction order (partition4 / dd_form
semantics: src/partition3.cpp:122-194, src/form_dd.cpp:32-110).

test_torch_nccl_then_rccl: bench.py's N > 1 library pairing -- torch's
"nccl" process group initialised and used first, then libggmres's own RCCL
communicator (GG_DD_RCCL) in the same process -- bit-identical to GG_DD_LOCAL.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from conftest import REPO
from ggmres import host, matrices as M
from ggmres.dd import DD

pytestmark = pytest.mark.gpu
WORKER = os.path.join(REPO, "tests", "dd_rank_worker.py")
sys.path.insert(0, os.path.join(REPO, "tests"))
import dd_rank_worker as W  # noqa: E402


def _port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def run_ranks(mode, P, outdir, timeout=240, xk=None, env_extra=None):
    """start P rank processes, wait for all; kill exactly those on failure
    (xk: GG_DD_XK for the ranks -- the orthogonalization's exchanges inside its
    kernels, 1, or as separate all-gather launches, 0; env_extra: more
    environment for the ranks)"""
    port = _port()
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(P), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        if xk is not None:
            env["GG_DD_XK"] = str(xk)
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, mode, str(outdir)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{o[-3000:]}"
    return [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(P)]


def merge(rs, key):
    """the ranks' owned rows into one vector; rows owned by several ranks (the
    separator replica) must agree bit for bit"""
    v = np.full(rs[0][key].shape, np.nan)
    for r in rs:
        m = ~np.isnan(r[key])
        both = m & ~np.isnan(v)
        assert np.array_equal(v[both], r[key][both]), key
        v[m] = r[key][m]
    assert not np.isnan(v).any(), f"{key}: rows nobody wrote"
    return v


@pytest.mark.parametrize("xk", [0, 1])
@pytest.mark.parametrize("case", sorted(W.CASES))
def test_dd_ipc_ranks_match_local_and_oracle(case, xk, tmp_path):
    P = int(case.split("_P")[1][0])
    rs = run_ranks(f"ipc:{case}", P, tmp_path, xk=xk)
    A, method = W.system(case)
    n = A.shape[0]
    # every rank holds the same plan and an identical control flow
    for r in rs[1:]:
        assert np.array_equal(r["q"], rs[0]["q"])
        for k in ("hist", "hist2", "hist3"):
            assert np.array_equal(r[k], rs[0][k]), k
        for k in ("iters", "inner", "ret", "iters2", "ret2", "iters3", "ret3"):
            assert int(r[k]) == int(rs[0][k]), k
    inf = rs[0]["info"]
    assert inf[1] == P and inf[8] == 1            # nparts, one shard in this process
    # the in-kernel exchanges ran (or not): ranks sharing this GPU take them only
    # when every rank's grid fits one block per CU (csrc/dd.hip use_xk)
    Gd = DD(P, device=0)
    Gd.set_system(A, method)
    fits = P * Gd.dot_layout(0)[1] <= 256
    Gd.close()
    assert int(inf[10]) == int(xk and fits), inf
    # the same decomposition in one process (GG_DD_LOCAL), the same inputs
    loc = DD(P, device=0)
    loc.set_system(A, method)
    pinv, q = loc.perm()
    assert np.array_equal(q, rs[0]["q"])
    rng = np.random.default_rng(11)
    x = rng.standard_normal(n)
    assert np.array_equal(merge(rs, "spmv"), loc.spmv(x))
    for k, scale in enumerate((1.0, 1e250)):
        v = rng.standard_normal(n) * scale
        assert np.array_equal(merge(rs, f"apply{k}"), loc.precond_apply(v)), k
    b = M.rhs_ones(A)
    g = loc.solve(b, restart=30, max_iter=1500, tol=1e-10)
    assert int(rs[0]["ret"]) == g["ret"] == 0 and int(rs[0]["iters"]) == g["iters"]
    assert np.array_equal(rs[0]["hist"], g["hist"])
    assert np.array_equal(merge(rs, "x"), g["x"])
    x0 = np.random.default_rng(9).standard_normal(n)
    g2 = loc.solve(M.rhs_uniform(n), x0=x0, restart=7, max_iter=40, tol=1e-14)
    assert int(rs[0]["ret2"]) == g2["ret"] == 1 and int(rs[0]["iters2"]) == g2["iters"] == 40
    assert np.array_equal(rs[0]["hist2"], g2["hist"])
    assert np.array_equal(merge(rs, "x2"), g2["x"])
    # CGS2 with the in-kernel exchanges: bit-identical to the launch-per-step path
    import ggmres
    g3 = loc.solve(b, restart=30, max_iter=1500, tol=1e-10, flags=ggmres.SOLVE_CGS2)
    assert int(rs[0]["ret3"]) == g3["ret"] == 0 and int(rs[0]["iters3"]) == g3["iters"]
    assert np.array_equal(rs[0]["hist3"], g3["hist"])
    assert np.array_equal(merge(rs, "x3"), g3["x"])
    # the oracle on B in the sharded reduction order
    segs, G = zip(*[loc.dot_layout(p) for p in range(P)])
    loc.close()
    B = host.permute(A, pinv, q)
    L, U = O.ilu0(B)
    O.set_dot_order_shards(list(segs), G[0])
    try:
        ref = O.gmres_left(B, L, U, b[q], m=30, max_iter=1500, tol=1e-10)
    finally:
        O.set_dot_order(None)
    assert np.array_equal(rs[0]["hist"], ref["hist"])
    assert np.array_equal(merge(rs, "x")[q], ref["x"])


@pytest.mark.parametrize("form", ["second_stream", "separate_launches"])
def test_dd_ipc_ranks_halo_forms(form, tmp_path):
    """The SpMV's interface exchange in the other two forms than the default
    (exchange and rows in one launch, k_dd_spmv_x): GG_DD_HALO_INLINE=0 on the
    second stream beside the interior rows, GG_DD_HALO_FUSED=0 as its own
    launch before the rows -- the same bits, every rank, against the
    one-process GG_DD_LOCAL run"""
    case = "5pt_200x160_P4"
    env = {"GG_DD_HALO_INLINE": "0"} if form == "second_stream" else {"GG_DD_HALO_FUSED": "0"}
    rs = run_ranks(f"ipc:{case}", 4, tmp_path, xk=0, env_extra=env)
    A, method = W.system(case)
    n = A.shape[0]
    loc = DD(4, device=0)
    loc.set_system(A, method)
    x = np.random.default_rng(11).standard_normal(n)
    assert np.array_equal(merge(rs, "spmv"), loc.spmv(x))
    g = loc.solve(M.rhs_ones(A), restart=30, max_iter=1500, tol=1e-10)
    assert int(rs[0]["iters"]) == g["iters"] and np.array_equal(rs[0]["hist"], g["hist"])
    assert np.array_equal(merge(rs, "x"), g["x"])
    loc.close()


def test_torch_nccl_then_rccl(tmp_path):
    (r,) = run_ranks("nccl_rccl", 1, tmp_path)
    A = M.laplacian_5pt(64, 64)
    loc = DD(1, device=0)
    loc.set_system(A, host.PART_BLOCKS)
    g = loc.solve(M.rhs_ones(A), restart=30, max_iter=1500, tol=1e-10)
    assert int(r["iters"]) == g["iters"] and np.array_equal(r["hist"], g["hist"])
    assert np.array_equal(r["x"], g["x"])
    loc.close()
