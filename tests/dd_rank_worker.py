"""One rank of a multi-process sharded solve (tests/test_gpu_dd_ranks.py).

    python tests/dd_rank_worker.py MODE OUTDIR       (RANK / WORLD_SIZE / MASTER_* set)

MODE
  ipc:<case>      one shard per process over GG_DD_IPC (device-initiated
                  exchanges through hipIpc-mapped areas); the handles are
                  all-gathered over torch.distributed "gloo" (CPU)
  nccl_rccl       world size 1: torch.distributed "nccl" initialised first and
                  used, then the sharded solve over its own RCCL communicator
                  (GG_DD_RCCL, one rank) -- bench.py's library pairing at N > 1
Writes OUTDIR/rank<r>.npz: natural-order results with NaN in the rows this
rank does not own (spmv, precond applies, GMRES solutions), histories,
iteration counts, info.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-gmres_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

CASES = {
    # name: (matrix factory, method); 2D grids, natural separator order: every
    # triangular solve on the 2D band wavefront, whose workgroups only wait on
    # earlier-dispatched ones -- safe with several processes on one GPU
    "5pt_200x160_P2": ("laplacian_5pt", (200, 160), "blocks"),
    "5pt_200x160_P4": ("laplacian_5pt", (200, 160), "blocks"),
    "5pt_96x150_P3_bisect": ("laplacian_5pt", (96, 150), "bisect"),
}


def system(case):
    from ggmres import host, matrices as M
    fn, args, meth = CASES[case]
    A = getattr(M, fn)(*args)
    method = host.PART_BLOCKS if meth == "blocks" else host.PART_BISECT
    return A, method


def run(d, A, n, out):
    from ggmres import matrices as M
    rng = np.random.default_rng(11)
    x = rng.standard_normal(n)
    out["spmv"] = d.spmv(x, np.full(n, np.nan))
    own = ~np.isnan(out["spmv"])              # the rows this process writes back
    for k, scale in enumerate((1.0, 1e250)):
        v = rng.standard_normal(n) * scale
        out[f"apply{k}"] = d.precond_apply(v, np.full(n, np.nan))
    b = M.rhs_ones(A)
    g = d.solve(b, restart=30, max_iter=1500, tol=1e-10)      # x0 = 0 (x is input and output)
    out.update(x=np.where(own, g["x"], np.nan), hist=g["hist"], iters=g["iters"], inner=g["inner"],
               ret=g["ret"])
    x0 = np.random.default_rng(9).standard_normal(n)
    g2 = d.solve(M.rhs_uniform(n), x0=x0, restart=7, max_iter=40, tol=1e-14)
    out.update(x2=np.where(own, g2["x"], np.nan), hist2=g2["hist"], iters2=g2["iters"], ret2=g2["ret"])
    # CGS2: the exchanges inside the orthogonalization's kernels (Xch)
    import ggmres
    g3 = d.solve(b, restart=30, max_iter=1500, tol=1e-10, flags=ggmres.SOLVE_CGS2)
    out.update(x3=np.where(own, g3["x"], np.nan), hist3=g3["hist"], iters3=g3["iters"], ret3=g3["ret"])


def main():
    mode, outdir = sys.argv[1], sys.argv[2]
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    from ggmres.dd import DD, unique_id
    out = {}
    if mode.startswith("ipc:"):
        case = mode[4:]
        dist.init_process_group("gloo", rank=rank, world_size=world)
        d = DD(world, device=0, rank=rank, comm="ipc")

        def allgather(b):
            lst = [None] * world
            dist.all_gather_object(lst, b)
            return lst

        d.connect_ipc(allgather)
        ranks, myrank = d.comm_ranks()
        assert (ranks, myrank) == (world, rank), (ranks, myrank)
        A, method = system(case)
    elif mode.startswith("xtime:"):
        # exchange latency probe (tools/ipc_exchange_probe.py): the C2 system
        # sharded over the ranks, one short solve, then timed all-gathers
        dist.init_process_group("gloo", rank=rank, world_size=world)
        d = DD(world, device=0, rank=rank, comm="ipc")

        def allgather(b):
            lst = [None] * world
            dist.all_gather_object(lst, b)
            return lst

        d.connect_ipc(allgather)
        from ggmres import host, matrices as M
        side = int(mode[6:])
        A = M.laplacian_5pt(side)
        d.set_system(A, host.PART_BLOCKS | host.PART_COLOR_SEP)
        d.solve(M.rhs_ones(A), restart=30, max_iter=30, tol=1e-300)
        G = d.dot_layout(rank)[1]
        res = {c: d.time_exchange(c, reps=500) for c in (1, G, 4 * G, 16 * G, 31 * G)}
        if rank == 0:
            print(f"IPC all-gather, {world} processes on one GPU, G = {G}: " +
                  ", ".join(f"{c} doubles {us:.2f} us" for c, us in res.items()), flush=True)
        d.close()
        dist.destroy_process_group()
        return
    elif mode == "nccl_rccl":
        assert world == 1
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)                      # torch's RCCL is loaded and initialised first
        assert float(t.sum()) == 4.0
        uid = [unique_id()]
        dist.broadcast_object_list(uid, src=0)
        d = DD(1, device=0, rank=0, uid=uid[0])
        ranks, myrank = d.comm_ranks()
        assert (ranks, myrank) == (1, 0)
        from ggmres import host, matrices as M
        A, method = M.laplacian_5pt(64, 64), host.PART_BLOCKS
    else:
        raise SystemExit(f"unknown mode {mode}")
    n = A.shape[0]
    d.set_system(A, method)
    out["info"] = np.array(list(d.info().values()))
    out["q"] = d.perm()[1]
    run(d, A, n, out)
    d.close()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **{k: np.asarray(v) for k, v in out.items()})
    dist.destroy_process_group()
    print(f"rank {rank}: ok ({mode})", flush=True)


if __name__ == "__main__":
    main()
