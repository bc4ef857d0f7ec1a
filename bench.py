#!/usr/bin/env python
"""bench.py -- fp64 GMRES iterations/s on MI355X (BASELINE.json metric).

Workload (N=1): config C2 of BASELINE.json -- 1000x1000 5-point Laplacian CSR
(n = 1,000,000, nnz = 4,996,000), ILU(0) left preconditioner, GMRES(30),
tol 1e-8, b = A*1, x0 = 0.  One step = one full solve (device-resident b, x;
the ILU factorization and H2D copies are setup, outside the timed region).

value = inner (Arnoldi) iterations of all ranks / max-over-ranks wall time.
roofline: the single kernel with the most time over the timed region: the
candidates (single-kernel families within 2x of the largest in a profiled
warmup step) are each bracketed with hipEvent pairs in a rotating share of the
timed solves, on the solver's stream (gg_profile_*), and every candidate's
entry is reported under "rooflines" (the triangular solves with their
dependency-chain fraction too); algorithmic bytes from SURVEY.md 8(d) (DESIGN.md
"Kernels"); traffic: HBM bytes per launch from the committed rocprofv3 PMC
passes (profiles/pmc_traffic.json), null when those counters were taken on
other kernel sources (src_sha).  cpu_baseline: the fp64 oracle restatement
(oracle/, serial C, one thread pinned to one core) on a bounded sample of the
same workload, rank 0 at N = 1 only.

--workload c3: SpMV on the circuit5M stand-in (seeded power-law CSR with
circuit5M's n = 5,558,326 and nnz ~ 59.5M; the SuiteSparse file
is not available offline): one step = --c3-spmvs SpMV launches, value =
algorithmic SpMV bytes / time in GB/s (no parity claim on this matrix).

--workload pg: the reference's power-grid (PG) engine, GMRESilu_GPU with an
ILU++-style SPLIT preconditioner (src/gmres.cu:2254-2446, MyILUPPfloat
src/preconditioner.cu:1162-1657), on the C2 grid: B = P_r D_l^-1 A D_r^-1 P_c,
L = Lt D1 (diagonal last), U = M D1^-1 Ut (diagonal first) from the device
ILU(0) of B, seeded scales in [0.5, 2); --pg-perm identity (default: the
factors stay grid-shaped and take the 2D wavefront) or random (P_r = P_c^-1
random: the level-scheduled flow solve).  The synthetic split stands in for
ILU++'s factors (ILU++ is not built here).

--workload c5: the transient loop (gg_transient: A = G + C/h on the C2 grid, 1 %
PULSE sources, --c5-steps backward-Euler steps per step, warm start); value =
GMRES iterations of all steps / time.

Multi-GPU: `--gpus N` (N > 1) without torchrun starts N rank processes (one
per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, before the parent makes
any GPU call) and exits with their status; under torchrun WORLD_SIZE must equal
--gpus.  At N > 1 the default workload is the SHARDED solve of the C2 system
(include/ggmres_dd.h: partition4 arrow ordering, one shard per GPU,
device-initiated all-gathers through hipIpc-mapped areas over xGMI -- --dd-comm
rccl for RCCL collectives -- and the CGS2 orthogonalization, three all-gathers
per inner iteration -- --dd-orth mgs for the reference's MGS; "scaling":
"strong", parallelism "ddN"); `--workload dd`
shards C4 (216^3 7-point) instead.  `--workload replicas` keeps the old
independent-C2-per-rank run ("scaling": "weak", no collective on the data
path); `--workload c5` gives each rank its own source scenario (many-RHS).
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gpu-gmres_amd"))

import numpy as np

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# tests only (tests/test_gpu_bench_ranks.py): every rank on GPU 0 and a gloo
# process group -- the multi-rank control flow on a one-GPU box
ONE_GPU = os.environ.get("GG_BENCH_ONE_GPU") == "1"
METRIC = "fp64 GMRES iterations/sec + SpMV HBM GB/s, 1M-row CSR @1/2/4/8 MI355X"
# --division -> ggmres.DIV_EXACT / DIV_RCP / DIV_FMA (ggmres.h gg_div_mode)
DIV_MODES = {"exact": 0, "rcp": 1, "fma": 2}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--grid", type=int, default=1000, help="grid side (1000 = C2, 100 = C1)")
    p.add_argument("--restart", type=int, default=30)
    p.add_argument("--ilu-level", type=int, default=0,
                   help="c2 only: ILU(k) factors (device numeric phase); k = 1, 2 run the skewed wavefront")
    p.add_argument("--tol", type=float, default=1e-8)
    p.add_argument("--max-iter", type=int, default=20000)
    p.add_argument("--cpu-iters", type=int, default=120,
                   help="oracle iterations timed for cpu_baseline (0 = skip)")
    p.add_argument("--no-profile", action="store_true", help="do not bracket kernels with events")
    p.add_argument("--c3-spmvs", type=int, default=20, help="SpMV launches per c3 step")
    p.add_argument("--c4-grid", type=int, default=216, help="C4: grid points per side (216^3 = 10.1M rows)")
    p.add_argument("--dd-parts", type=int, default=8,
                   help="dd workload on one process: shards held by this process (GG_DD_LOCAL)")
    p.add_argument("--dd-grid", choices=["c4", "c2"], default=None,
                   help="dd workload system: c4 (216^3 7-pt, the default of --workload dd) or c2 "
                        "(1000^2 5-pt, the default sharded system at --gpus N > 1)")
    p.add_argument("--pg-perm", choices=["identity", "random"], default="identity",
                   help="pg: the split's row / column permutations")
    p.add_argument("--pg-seed", type=int, default=20261015, help="pg: the split's seed (permutations, scales)")
    p.add_argument("--pad-stride", type=int, default=50,
                   help="netlist: a VDD pad (package R + voltage source) every this many nodes per direction")
    p.add_argument("--workload", choices=["c2", "c3", "c3s", "c4", "c5", "dd", "replicas", "pg", "netlist"],
                   default=None,
                   help="default: c2 at N = 1 (one C2 solve per step, the headline), the sharded C2 "
                        "solve at N > 1; dd: the sharded solve (C4 unless --dd-grid c2); replicas: "
                        "one independent C2 solve per rank; c5: a backward-Euler transient (A = G + C/h, "
                        "1%% PULSE sources) of --c5-steps time steps per step")
    p.add_argument("--dd-part", choices=["slabs", "grid"], default=None,
                   help="dd: base partition -- slabs = contiguous index ranges (GG_PART_BLOCKS) or grid = "
                        "px x py rectangles of the 2D grid (GG_PART_GRID: interior chains nx/px + ny/py); "
                        "default grid")
    p.add_argument("--dd-sep", choices=["color", "natural"], default="color",
                   help="dd: separator order -- a greedy colouring of its graph (GG_PART_COLOR_SEP, "
                        "default: a few-level separator solve) or partition4's ascending index")
    p.add_argument("--division", choices=["fma", "rcp", "exact"], default="fma",
                   help="triangular-solve rows: fma = two fused multiply-adds per row on the unskewed "
                        "2D-grid wavefronts, U pre-scaled by RN(1/d), rcp elsewhere (gg_set_division "
                        "GG_DIV_FMA, default); rcp = x = acc * RN(1/d) on the wavefront solves "
                        "(GG_DIV_RCP); both tolerance parity 1e-10 (tests/test_gpu_fastdiv.py); "
                        "exact = the reference's row arithmetic bit for bit")
    p.add_argument("--dd-comm", choices=["ipc", "rccl", "loopback"], default="ipc",
                   help="sharded solve at N > 1: ipc = device-initiated all-gathers through hipIpc-mapped "
                        "exchange areas over xGMI (GG_DD_IPC, default), rccl = RCCL collectives (GG_DD_RCCL); "
                        "loopback (one process, timing only): shard --dd-rank of --dd-parts alone on this GPU, "
                        "every exchange the in-process all-gather over its own buffer, --max-iter iterations")
    p.add_argument("--dd-rank", type=int, default=0, help="dd loopback: the shard this process times")
    p.add_argument("--dd-orth", choices=["cgs2", "mgs"], default="cgs2",
                   help="sharded solve: cgs2 = three all-gathers per inner iteration (GG_SOLVE_CGS2, tolerance "
                        "parity; default), mgs = the reference's modified Gram-Schmidt (i + 2 all-gathers)")
    p.add_argument("--c5-steps", type=int, default=1000)
    p.add_argument("--c5-scenarios", type=int, default=1,
                   help="c5: independent source scenarios per GPU (many-RHS), solved as one batch "
                        "(--c5-mode batch) or concurrently")
    p.add_argument("--c5-mode", choices=["auto", "batch", "streams"], default="auto",
                   help="c5: batch = gg_transient_batch, every launch serving all scenarios (batch.hip); "
                        "streams = one solver, stream and host thread per scenario (GG_SOLVE_SHARED_DEVICE); "
                        "auto = batch for several scenarios, gg_transient for one")
    a = p.parse_args()
    if a.dd_comm == "loopback" and (a.gpus > 1 or not 0 <= a.dd_rank < a.dd_parts):
        p.error("--dd-comm loopback times one rank alone: --gpus 1 and 0 <= --dd-rank < --dd-parts")
    return a


# bench family -> the kernel it times (rocprofv3 kernel names in profiles/)
KERNEL_NAMES = {
    # sliced-ELL SpMV on short even rows (grids); GG_SPMV_CSR=1 keeps the CSR-stream kernel
    "spmv": "k_spmv_stream<false>" if os.environ.get("GG_SPMV_CSR") == "1" else "k_spmv_sell<false>",
    "trsv_L": "k_trsv_wave2d<true, 0, false, false, 1, false>",  # lower, unit diagonal (ILU(0) L), 2D grid
    "trsv_U": "k_trsv_wave2d<false, 2, false, false, 1, false>", # upper, reciprocal division (ILU(0) U), 2D grid
}
PMC_FILE = os.path.join(REPO, "profiles", "pmc_traffic.json")
# bare dependent-chain latency of one wavefront step (cycles, tools/lat_probe.hip
# built like the library, -ffp-contract=off, on MI355X: profiles/r03/r03_lat_probe.txt
# "step(dpp)" = unit L, "U step (WD_RCP)" = the bit-exact reciprocal-FMA
# division, "U step (WD_MUL)" = GG_DIV_RCP's one multiply; "L step (UFMA)" /
# "U step (SFMA)" = GG_DIV_FMA's fused rows, profiles/r03/r03_lat_probe_fma.txt) and
# the shader clock
CHAIN_CYCLES = {"trsv_L": 38.89, "trsv_U": 62.66, "trsv_U_mul": 43.72,
                "trsv_L_fma": 29.19, "trsv_U_fma": 29.58}
SHADER_GHZ = 2.399
TIE_FRAC = 0.05          # roofline kernel: candidates within 5 % of the top time are tied


def chain_key(kernel, dom, fma, mul):
    """CHAIN_CYCLES entry of a wavefront solve: from the kernel's division
    template argument (kernels.hip WaveDiv: 0 unit, 1 IEEE division, 2
    reciprocal + FMA corrections, 3 multiply by RN(1/d), 4 / 5 fused rows)
    when the name carries it, else from the solver's division mode"""
    import re
    m = re.match(r"k_trsv_wave2d_spmv<(\d+)>", kernel) or re.match(r"k_trsv_(?:wave2d|tile3d)<\w+, (\d+)", kernel)
    if m:
        return {0: "trsv_L", 1: "trsv_U", 2: "trsv_U", 3: "trsv_U_mul", 4: "trsv_L_fma", 5: "trsv_U_fma"}[int(m.group(1))]
    return (dom + "_fma") if fma else "trsv_U_mul" if mul else dom


def kernel_key(name):
    """a kernel's template name with trailing default arguments dropped, so the
    bench's short names ('k_spmv_stream<false>') and rocprof's
    ('k_spmv_stream<false, false>') meet: ', false' / ', 0' suffixes removed"""
    name = name.replace(" ", "")
    while name.endswith((",false>", ",0>")):
        name = name[: name.rindex(",")] + ">"
    return name


def pmc_traffic(kernel, workload=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, or profiles/pmc_traffic_<workload>.json; written
    by profiles/pmc_traffic.py: FETCH_SIZE doubled for 16-B/lane streaming
    reads, + WRITE_SIZE; MI355X_MICROARCH.md HBM section), or None when that
    file has no entry for it (names compared by kernel_key)."""
    path = PMC_FILE if workload is None else PMC_FILE.replace(".json", f"_{workload}.json")
    try:
        with open(path) as f:
            d = json.load(f)
        sys.path.insert(0, os.path.join(REPO, "profiles"))
        from pmc_traffic import src_sha
        if d.get("src_sha") != src_sha():      # counters taken on other kernel sources: stale
            return None
        ks = d["kernels"]
        if kernel in ks:
            return ks[kernel]["hbm_bytes_per_launch"]
        want = kernel_key(kernel)
        hit = [v for k, v in ks.items() if kernel_key(k) == want]
        if not hit and "<" not in kernel:
            # a bare name ('k_trsv_flow') and ONE instantiation of it in the file
            hit = [v for k, v in ks.items() if k.startswith(kernel + "<")]
        return hit[0]["hbm_bytes_per_launch"] if len(hit) == 1 else None
    except (OSError, KeyError, ValueError):
        return None


def mgs_bytes(n, m, inner_list):
    """MGS bytes for the inner iterations actually run, as (fused, reference, iterations):
    fused = what the one-launch orthogonalization (k_arnoldi_persist) must move at
    cycle index i: v_0..v_i and w read once, v_{i+1} written = 8 n (i+3); reference =
    SURVEY.md 8(d)'s count of the unfused reference operations, 40 n (i+1) (dot + AXPY
    per k) + 24 n (norm + scale) -- a reference-equivalent figure, not HBM traffic."""
    fused = ref = 0.0
    iters = 0
    for inner in inner_list:
        full, rem = divmod(inner, m)
        for i in list(range(m)) * full + list(range(rem)):
            fused += 8.0 * n * (i + 3)
            ref += 40.0 * n * (i + 1) + 24.0 * n
            iters += 1
    return fused, ref, iters


def pg_split(A, device, seed=20261015, identity=True):
    """Synthetic ILU++-style split of A (the PG engine's preconditioner):
    B = P_r D_l^-1 A D_r^-1 P_c with pcol = prow^-1, (Lt, Ut) = the device ILU(0)
    of B (leftILU semantics), L = Lt D1 (non-unit, diagonal last), U = M D1^-1 Ut
    (diagonal first), so Ml A Mr = D1^-1 Lt^-1 B Ut^-1 D1."""
    import scipy.sparse as sp
    import ggmres
    A = sp.csr_matrix(A)
    n = A.shape[0]
    rng = np.random.default_rng(seed)
    prow = np.arange(n, dtype=np.int32) if identity else rng.permutation(n).astype(np.int32)
    pcol = np.argsort(prow).astype(np.int32)
    lscale, rscale, middle, d1 = (rng.uniform(0.5, 2.0, n) for _ in range(4))
    Pr = sp.csr_matrix((np.ones(n), (np.arange(n), prow)), shape=(n, n))
    B = (Pr @ sp.diags(1.0 / lscale) @ A @ sp.diags(1.0 / rscale) @ Pr.T).tocsr()
    B.sort_indices()
    f = ggmres.Solver(device)
    f.set_matrix(B)
    vals, _ = f.ilu0_device_values()
    f.close()
    F = sp.csr_matrix((vals, B.indices, B.indptr), shape=(n, n))
    Lt = (sp.tril(F, -1) + sp.identity(n)).tocsr()
    Ut = sp.triu(F).tocsr()
    L = (Lt @ sp.diags(d1)).tocsr()
    U = (sp.diags(middle / d1) @ Ut).tocsr()
    L.sort_indices()
    U.sort_indices()
    return L, U, middle, prow, pcol, lscale, rscale


def pulse_at(q, t):
    """PULSE(v1, v2, td, tr, tf, pw, per) at time t (gen_PULSEut_kernel semantics,
    src/kernels.cu:223-245)"""
    v1, v2, td, tr, tf, pw, per = q
    if t < td:
        return v1
    tt = (t - td) % per if per > 0 else t - td
    if tt < tr:
        return v1 + (v2 - v1) * tt / tr
    if tt < tr + pw:
        return v2
    if tt < tr + pw + tf:
        return v2 + (v1 - v2) * (tt - tr - pw) / tf
    return v1


def netlist_system(a, device):
    """The reference's PG workload (src/mna_solve_gpu_gmres.cpp:190-647): a
    synthetic IBM-PG-style netlist (ggmres.matrices.pg_netlist: R mesh, decap
    to ground at every node, PULSE load currents, VDD pads = package R +
    voltage source) read by the library's SPICE front end (gg_host_read_netlist)
    into MNA G, C, B; A = G + C/h at the netlist's .tran step; the split
    preconditioner of the PG engine with non-identity permutations: the
    pivoting ordering that puts the voltage-source branch rows' zero diagonals
    off the diagonal (mna_pivot_order: tail of pad / branch unknowns first),
    (L, U) = the device ILU(0) of B = P_r A P_c (leftILU semantics), unit
    scales; b = B u(t) + (C/h) x0 at t = 10 steps (loads switched on), x0 = 0.
    ILU++ itself is not built here: its multilevel factors are
    replaced by this ILU(0) with the same kind of row / column permutations."""
    import tempfile
    import scipy.sparse as sp
    import ggmres
    from ggmres import host as H, matrices as M
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "pg.sp")
        ng, npad = M.pg_netlist(path, a.grid, a.grid, pad_stride=a.pad_stride)
        t1 = time.perf_counter()
        nl = H.Netlist(path)
    t_parse = time.perf_counter() - t1
    h = nl.tstep
    A = (nl.G + nl.C / h).tocsr()
    A.sort_indices()
    n = A.shape[0]
    prow, pcol = M.mna_pivot_order(ng, npad, n)
    Pr = sp.csr_matrix((np.ones(n), (np.arange(n), prow)), shape=(n, n))
    Pc = sp.csr_matrix((np.ones(n), (np.arange(n), pcol)), shape=(n, n))
    B = (Pr @ A @ Pc).tocsr()
    B.sort_indices()
    f = ggmres.Solver(device)
    f.set_matrix(B)
    vals, _ = f.ilu0_device_values()
    f.close()
    F = sp.csr_matrix((vals, B.indices, B.indptr), shape=(n, n))
    L = (sp.tril(F, -1) + sp.identity(n)).tocsr()
    U = sp.triu(F).tocsr()
    L.sort_indices()
    U.sort_indices()
    ones = np.ones(n)
    t = 10 * h
    u = np.array([par[0] if kind == 0 else pulse_at(par, t) if kind == 1 else np.interp(t, par[0::2], par[1::2])
                  for kind, par in nl.sources])
    b = np.asarray(nl.B @ u).ravel()
    info = {"n_grid": ng, "pads": npad, "n": n, "nnz": int(A.nnz), "h": h, "t": t,
            "parse_s": round(t_parse, 3), "setup_s": round(time.perf_counter() - t0, 3)}
    return A, b, (L, U, ones, prow, pcol, ones, ones), info


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def bench_c3(a, torch, dist, world, rank, local):
    """SpMV roofline on the C3 stand-in (one matrix per rank, weak scaling)."""
    import ggmres
    from ggmres import matrices as M
    t_setup = time.perf_counter()
    A = M.power_law(seed=20261015 + rank)
    s = ggmres.Solver(local)
    s.set_matrix(A)
    s.set_precond_none()
    t_setup = time.perf_counter() - t_setup
    byt = s.bytes_spmv()

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        s.time_spmv(reps=a.c3_spmvs, nrot=1)
    barrier()
    t0 = time.perf_counter()
    ev_ms = [s.time_spmv(reps=a.c3_spmvs, nrot=1) for _ in range(a.steps)]
    barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    tot = torch.tensor([byt * a.c3_spmvs * a.steps], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    value = float(tot.item()) / float(t.item()) / 1e9
    avg_us = sum(ev_ms) / len(ev_ms) * 1e3                 # events around each launch
    ach = byt / (avg_us * 1e-6) / 1e9
    rl = np.diff(A.indptr)
    # column panels (k_spmv_panel): one launch per panel, an SpMV = all of them
    npan, nrt = s.spmv_panels, s.spmv_rtile
    if npan and nrt:
        c3_kernel = f"k_spmv_rtile (one launch: {nrt} row blocks over {npan} column panels)"
        c3_traffic = pmc_traffic("k_spmv_rtile", "c3")
    elif npan:
        c3_kernel = f"k_spmv_panel ({npan} panel launches per SpMV)"
        per = pmc_traffic("k_spmv_panel", "c3")
        c3_traffic = per * npan if per is not None else None
    else:
        c3_kernel = "k_spmv_stream<false>"
        c3_traffic = pmc_traffic("k_spmv_stream<false>", "c3")
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "GB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el * 1e3 / a.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"C3 stand-in: seeded power-law CSR (circuit5M n and nnz), "
                               f"y = A x, {a.c3_spmvs} SpMVs per step",
                   "n": int(A.shape[0]), "nnz": int(A.nnz), "max_row": int(rl.max()),
                   "mean_row": round(float(rl.mean()), 2),
                   "parallelism": "single" if world == 1 else f"replicas{world}",
                   "setup_s": round(t_setup, 3)},
        "roofline": {"kernel": c3_kernel, "bound": "hbm", "achieved": round(ach, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": c3_traffic,
                     "alg_bytes_per_launch": byt, "avg_us": round(avg_us, 3)},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    s.close()
    if dist:
        dist.destroy_process_group()


def lockstep(torch, dist, group, rank, steps):
    """Run `steps` ([(name, fn)]) in lockstep over the CPU `group`: after each
    local step every rank learns (MIN all-reduce) whether every rank succeeded,
    and all stop at the first step that failed anywhere.  A rank whose step
    raised still joins the agreement, so no rank is left waiting in a
    collective of a later step.  True iff every step succeeded on every rank."""
    for name, fn in steps:
        try:
            fn()
            ok = 1
        except Exception as e:          # noqa: BLE001 -- any failure: every rank falls back together
            print(f"bench.py rank {rank}: IPC {name} failed ({e})", file=sys.stderr, flush=True)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if not int(flag.item()):
            return False
    return True


def bench_dd(a, torch, dist, world, rank, local):
    """The sharded solve (include/ggmres_dd.h): ONE system split over the ranks
    (torchrun: one shard per GPU, RCCL exchanges; one process: --dd-parts
    shards on this GPU, in-process exchanges).  value = inner iterations of
    the one solve / max-over-ranks wall time ("scaling": "strong")."""
    from ggmres import host, matrices as M
    from ggmres.dd import DD, unique_id
    A = M.grid_7pt(a.c4_grid) if a.dd_grid == "c4" else M.laplacian_5pt(a.grid)
    n = A.shape[0]
    b = M.rhs_ones(A)
    t_setup = time.perf_counter()
    comm = a.dd_comm
    if world > 1 and comm == "ipc":
        # device-initiated exchanges: the ranks' exchange-area handles are
        # all-gathered once over a CPU (gloo) group, then every exchange is a
        # kernel storing into the peers' areas over xGMI
        import ggmres
        boot = dist.new_group(backend="gloo")
        d, hb, ranks = None, None, None

        def create():
            nonlocal d, hb
            if os.environ.get("GG_BENCH_IPC_FAIL") == f"create:{rank}":      # fault injection (tests)
                raise RuntimeError("injected")
            d = DD(world, device=local, rank=rank, comm="ipc")
            hb = d.ipc_handle()

        def connect():
            lst = [None] * world
            dist.all_gather_object(lst, hb, group=boot)     # every rank reaches this together
            if os.environ.get("GG_BENCH_IPC_FAIL") == f"connect:{rank}":
                raise RuntimeError("injected")
            d.ipc_connect(lst)

        def check():
            nonlocal ranks
            ranks, myrank = d.comm_ranks()                  # an exchange: bounded (30 s) on the device
            if ranks != world or myrank != rank:
                raise RuntimeError(f"{ranks} ranks mapped (rank {myrank})")

        ok = lockstep(torch, dist, boot, rank, [("exchange area", create), ("connect", connect),
                                                ("rank check", check)])
        if not ok:
            # every rank falls back together: RCCL collectives
            if d is not None:
                d.close()
            comm = "rccl"
    if world > 1 and comm == "rccl":
        uid = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        d = DD(world, device=local, rank=rank, uid=uid[0])
        ranks, myrank = d.comm_ranks()
        if ranks != world or myrank != rank:
            raise SystemExit(f"bench.py: RCCL communicator has {ranks} ranks (rank {myrank}), "
                             f"expected {world} (rank {rank})")
    elif world == 1 and comm == "loopback":
        d = DD(a.dd_parts, device=local, rank=a.dd_rank, comm="loopback")
        ranks = 1
    elif world == 1:
        d = DD(a.dd_parts, device=local)
        ranks = 1
    part = host.PART_GRID if a.dd_part == "grid" else host.PART_BLOCKS
    d.set_system(A, part | (host.PART_COLOR_SEP if a.dd_sep == "color" else 0))
    import ggmres
    dd_div = a.division
    d.set_division(DIV_MODES[dd_div])
    t_setup = time.perf_counter() - t_setup
    info = d.info()
    db = torch.from_numpy(b).cuda()
    dx = torch.zeros(n, dtype=torch.float64, device="cuda")

    flags = ggmres.SOLVE_CGS2 if a.dd_orth == "cgs2" else 0

    loop = comm == "loopback"
    # loopback: a fixed iteration count (the values are not the system's)
    tol = 1e-300 if loop else a.tol

    def step():
        dx.zero_()
        torch.cuda.synchronize()
        return d.solve_device(db.data_ptr(), dx.data_ptr(), restart=a.restart,
                              max_iter=a.max_iter, tol=tol, flags=flags)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    from ggmres import dd as DDM

    # shards whose launches one event bracket covers: every shard of a local
    # (in-process) run, one per rank otherwise
    per_bracket = a.dd_parts if (world == 1 and not loop) else 1

    def families(inner_run, el):
        """this rank's per-family event timing (every inner iteration's families
        bracketed; the shards of this process)"""
        fam = {}
        for k, name in enumerate(DDM.PROF_NAMES):
            cnt, ms = d.profile_get(k)
            if cnt == 0:
                continue
            fam[name] = {"launches": cnt, "avg_us": round(ms * 1e3 / cnt, 3),
                         "shards_per_launch": per_bracket,
                         "avg_us_per_shard": round(ms * 1e3 / cnt / per_bracket, 3),
                         "share_of_step": round(ms / (el * 1e3), 4)}
            if k in (DDM.PROF_SPMV, DDM.PROF_TRSV_L, DDM.PROF_TRSV_U):
                byt = d.bytes(k)
                fam[name]["alg_bytes_per_launch"] = byt
                fam[name]["achieved_gbs"] = round(byt / (ms * 1e-3 / cnt) / 1e9, 1)
        return fam

    # per-family breakdown in the last warmup step (events around every family
    # cost time, so that pass stays out of the timed region); then only the
    # dominant single-kernel family (SpMV, interior L, interior U) is bracketed
    # inside the timed region, for the roofline
    fam = {}
    for w in range(a.warmup):
        if w == a.warmup - 1 and not a.no_profile:
            d.profile(True)
            barrier()
            t1 = time.perf_counter()
            r0 = step()
            barrier()
            fam = families(r0["inner"], time.perf_counter() - t1)
            d.profile(False)
        else:
            step()
    single = {k: v for k, v in fam.items() if "alg_bytes_per_launch" in v}
    dom = max(single, key=lambda k: single[k]["share_of_step"]) if single else None
    if dom:
        d.profile(True, kinds=[DDM.PROF_NAMES.index(dom)])
    barrier()
    t0 = time.perf_counter()
    res = [step() for _ in range(a.steps)]
    barrier()
    el = time.perf_counter() - t0
    timed = families(None, el) if dom else {}
    d.profile(False)
    t = torch.tensor([el], dtype=torch.float64, device="cpu" if ONE_GPU else "cuda")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    inner = sum(r["inner"] for r in res)          # one system: every rank counts the same
    roof = None
    wi = d.info()["wave_interior"]
    fused_halo = (((world > 1 and comm == "ipc") or (world == 1 and comm == "loopback"))
                  and os.environ.get("GG_DD_HALO_FUSED", "1") != "0" and os.environ.get("GG_DD_HALO_INLINE", "1") != "0")
    kname = {"spmv": ("k_dd_spmv_x (halo exchange + interior + separator rows in one launch)" if fused_halo
                      else "k_spmv_sell<false> / k_spmv_stream<false> (interior + separator rows)"),
             "trsv_L": {2: "k_trsv_wave2d (interior L, 2D band wavefront)",
                        3: "k_trsv_tile3d (interior L, 3D tile wavefront)"}.get(wi, "k_trsv_flow (interior L)"),
             "trsv_U": {2: "k_trsv_wave2d (interior U, 2D band wavefront)",
                        3: "k_trsv_tile3d (interior U, 3D tile wavefront)"}.get(wi, "k_trsv_flow (interior U)")}
    if dom and dom in timed:
        f = timed[dom]
        roof = {"kernel": kname[dom], "bound": "hbm", "achieved": f["achieved_gbs"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(f["achieved_gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
                "alg_bytes_per_launch": f["alg_bytes_per_launch"], "avg_us": f["avg_us"],
                "avg_us_per_shard": f["avg_us_per_shard"], "shards_per_launch": per_bracket,
                "launches_timed": f["launches"], "rank": rank,
                "note": ("event-timed inside the timed region on the solver's stream; one bracket covers "
                         + ("every local shard (bytes and time of all of them: the rate is theirs together)"
                            if per_bracket > 1 else "this rank's own shard"))}
    # every rank's breakdown next to the exchange latency (rank 0 prints them)
    per_rank = [{"rank": rank, "kernels": fam}]
    if dist:
        lst = [None] * world
        dist.all_gather_object(lst, per_rank[0])
        per_rank = lst
    parts = world if world > 1 else a.dd_parts
    # the exchange every sharded operator and dot pays, timed after the timed
    # region: one dot's G partials, and CGS2's (i+1) G at i = 15
    info_g = d.dot_layout(rank if world > 1 else a.dd_rank if loop else 0)[1]
    xch = {f"{c}_doubles_us": round(d.time_exchange(c, reps=200), 2) for c in (info_g, 16 * info_g)}
    out = {
        "metric": METRIC, "value": round(inner / el_max, 3), "unit": "iterations/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(el_max * 1e3 / a.steps, 3), "higher_is_better": True,
        # one step = one solve: the time to solution next to the rate (the
        # sharded preconditioner converges in its own iteration count)
        "ms_per_solve": round(el_max * 1e3 / a.steps, 3), "iters_per_solve": res[0]["inner"],
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": (f"sharded solve: {'C4 %d^3 7-pt' % a.c4_grid if a.dd_grid == 'c4' else 'C2 %dx%d 5-pt' % (a.grid, a.grid)}"
                                f", {parts}-way partition4 ({'px x py grid rectangles' if a.dd_part == 'grid' else 'contiguous slabs'}) arrow ordering"
                                f"{', separator by colour' if a.dd_sep == 'color' else ''}, ILU(0) of "
                                f"the permuted matrix, GMRES({a.restart}), tol {a.tol:g}, b=A*1, x0=0, "
                                f"one solve per step"),
                   "n": n, "nnz": int(A.nnz), "parts": parts,
                   "exchange": ("device-initiated all-gathers into hipIpc-mapped peer areas over xGMI "
                                "(GG_DD_IPC)" if comm == "ipc" else
                                "RCCL all-gather over xGMI" + (" (IPC unavailable: fallback)"
                                                               if a.dd_comm == "ipc" else ""))
                               if world > 1 else ("loopback: the in-process all-gather kernel over this "
                                                  "shard's own buffer (timing only)") if loop
                               else f"in-process ({parts} shards on one GPU)",
                   "exchange_ranks": ranks if world > 1 else None,
                   "exchange_latency": xch,
                   "division": dd_div,
                   "orthogonalization": (("CGS2 in 4 launches, its 3 exchanges inside the kernels "
                                          "(GG_SOLVE_CGS2, Xch" if info.get("cgs2_in_kernel_exchange") else
                                          "CGS2: 3 all-gathers per inner iteration (GG_SOLVE_CGS2") +
                                         ", tolerance parity 1e-10 vs MGS over the first cycle)")
                                        if a.dd_orth == "cgs2"
                                        else "MGS (the reference's): i + 2 all-gathers per inner iteration",
                   "all_gathers_per_iteration": (2 + 3) if a.dd_orth == "cgs2" else
                                                "2 + (i + 2) at cycle index i",
                   "separator_rows": info["nsep"], "max_interface": info["max_iface"],
                   "wavefront_interior": info["wave_interior"],
                   "wavefront_separator": int(info["wave_separator"] >= 2),
                   "separator_step": {0: "level launches", 1: "fused dataflow launch (k_sep_flow)",
                                      2: "2D wavefront", 3: "3D tile wavefront"}.get(info["wave_separator"]),
                   "iters_per_solve": res[0]["inner"], "relres": res[0]["relres"],
                   "parallelism": (f"rank {a.dd_rank} of dd{parts} alone (loopback exchanges, timing only: "
                                   f"{a.max_iter} iterations, values not the system's)") if loop else f"dd{parts}",
                   "setup_s": round(t_setup, 3)},
        "roofline": roof,
        "kernels_per_rank": per_rank,
        "kernels_from": "one profiled warmup step per rank, every family bracketed by hipEvents",
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    d.close()
    if dist:
        dist.destroy_process_group()


def spawn_ranks(n, argv, visible=None):
    """--gpus N without torchrun: start n rank processes (one per GPU, running
    `argv` with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) and return their
    status.  The parent makes no GPU call (torch.cuda.device_count does not
    initialise the device on this image); a rank that fails takes the others
    down (they would wait in a collective)."""
    import signal
    import socket
    import subprocess
    if visible is None:
        import torch
        visible = n if ONE_GPU else torch.cuda.device_count()
    if visible < n:
        print(f"bench.py: --gpus {n} but only {visible} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0" if ONE_GPU else str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:                      # the exact children this process started
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(env_world or "1")
    if world != max(a.gpus, 1):
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the workload: the C2 solve on one GPU, the sharded C2 solve on N > 1
    if a.workload is None:
        a.workload = "c2" if world == 1 else "dd"
        a.dd_grid = a.dd_grid or "c2"
    a.dd_grid = a.dd_grid or "c4"
    # rectangles / boxes (GG_PART_GRID: chains nx/px + ny/py (+ nz/pz)): C2
    # converges in 3,910 iterations vs the slabs' 6,369 at 4 shards
    # (profiles/r04/r04k_dd_4_*.json); C4 at 8 shards 230 vs 175 it/s
    # (profiles/r04/r04r_dd_c4grid_8.json vs r04q_dd_c4_8.json)
    a.dd_part = a.dd_part or "grid"
    replicas = a.workload == "replicas"
    if replicas:
        a.workload = "c2"
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if ONE_GPU:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import ggmres
    from ggmres import matrices as M

    if a.workload == "c3":
        return bench_c3(a, torch, dist, world, rank, local)
    if a.workload == "dd":
        return bench_dd(a, torch, dist, world, rank, local)
    c5 = a.workload == "c5"
    c4 = a.workload == "c4"
    c3s = a.workload == "c3s"           # GMRES + ILU(0) on the C3 stand-in (general sparsity)
    pg = a.workload == "pg"             # the split (PG) engine on the C2 grid
    netlist = a.workload == "netlist"   # the split engine on an MNA system from a PG netlist
    h5 = 1e-2
    t_setup = time.perf_counter()
    if netlist:
        A, b, split, net_info = netlist_system(a, local)
    else:
        A = M.grid_7pt(a.c4_grid) if c4 else M.power_law() if c3s else M.laplacian_5pt(a.grid)
        if c5:
            A = M.transient(A, c=1e-3, h=h5)
        b = M.rhs_ones(A)
    n = A.shape[0]
    s = ggmres.Solver(local)
    s.set_matrix(A)
    kilu = a.ilu_level if a.workload in ("c2", "c3s") else 0
    if pg or netlist:
        if pg:
            split = pg_split(A, local, seed=a.pg_seed, identity=a.pg_perm == "identity")
        s.set_precond_split(*split)
    elif kilu:
        s.set_precond_iluk_device(kilu)
        if not c3s:
            for dom_ in ("trsv_L", "trsv_U"):              # the skewed instantiation (skew k+1)
                KERNEL_NAMES[dom_] = KERNEL_NAMES[dom_].replace(", 1, false>", f", {kilu + 1}, false>")
    else:
        s.set_precond_ilu0()
    s.set_division(DIV_MODES[a.division])
    if s.uses_wavefront:
        # the kernels the solver launches for L and U (2D band / 3D tile
        # wavefront, skew, division mode), as rocprofv3 names them
        KERNEL_NAMES["trsv_L"] = s.trsv_kernel(0)
        KERNEL_NAMES["trsv_U"] = s.trsv_kernel(1)
    u_mode, l_mode = s.division_active(1), s.division_active(0)
    u_mul, l_mul = u_mode != ggmres.DIV_EXACT, l_mode != ggmres.DIV_EXACT     # not the reference's division
    u_fma, l_fma = u_mode == ggmres.DIV_FMA, l_mode == ggmres.DIV_FMA
    t_setup = time.perf_counter() - t_setup
    db = torch.from_numpy(b).cuda()
    dx = torch.zeros(n, dtype=torch.float64, device="cuda")
    if c5:
        # independent many-RHS scenarios, each its own seeded source set: S per
        # rank, solved concurrently on the rank's GPU when S > 1
        S = max(1, a.c5_scenarios)
        scen = [M.pulse_sources(n, frac=0.01, h=h5, seed=20261015 + rank * S + k) for k in range(S)]
        cdiag = np.full(n, 1e-3 / h5)
        ports = np.array([0, n // 2, n - 1], np.int32)
        solvers = [s]
        c5_batch = a.c5_mode == "batch" or (S > 1 and a.c5_mode == "auto")
        if c5_batch:
            assert s.batch_engine, "c5 batch: the solver's configuration takes no batched launches"
        else:
            for _ in range(S - 1):
                s2 = ggmres.Solver(local)
                s2.set_matrix(A)
                s2.set_precond_ilu0()
                s2.set_division(DIV_MODES[a.division])
                solvers.append(s2)
        flags = ggmres.SOLVE_SHARED_DEVICE if S > 1 else 0
        X0 = np.zeros((S, n))

    def step():
        if c5 and c5_batch:
            r = s.transient_batch(a.c5_steps, h5, cdiag, scen, ports, X0, restart=a.restart,
                                  max_iter=a.max_iter, tol=a.tol)
            tot = sum(r["iters_total"])
            return dict(inner=tot, iters=tot, relres=None, ret=r["ret"])
        if c5:
            out = [None] * len(solvers)

            def run(k):
                nodes, pulses = scen[k]
                out[k] = solvers[k].transient(a.c5_steps, h5, cdiag, nodes, pulses, ports, np.zeros(n),
                                              restart=a.restart, max_iter=a.max_iter, tol=a.tol,
                                              flags=flags)

            if len(solvers) == 1:
                run(0)
            else:
                th = [threading.Thread(target=run, args=(k,)) for k in range(len(solvers))]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
            tot = sum(r["iters_total"] for r in out)
            return dict(inner=tot, iters=tot, relres=None, ret=max(r["ret"] for r in out))
        dx.zero_()
        torch.cuda.synchronize()
        return s.solve_device(db.data_ptr(), dx.data_ptr(), restart=a.restart,
                              max_iter=a.max_iter, tol=a.tol)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    FAMS = (("spmv", ggmres.PROF_SPMV, lambda: s.bytes_spmv()),
            ("ilu0_apply", ggmres.PROF_PRECOND, lambda: s.bytes_precond()),
            # with the SpMV fused into the forward solve's launch (GG_FUSE_SPMV) that
            # launch also moves the SpMV's bytes
            ("trsv_L", ggmres.PROF_TRSV_L,
             lambda: s.bytes_trsv(0) + (s.bytes_spmv() if s.trsv_kernel(0).startswith("k_trsv_wave2d_spmv")
                                        else 0)),
            ("trsv_U", ggmres.PROF_TRSV_U, lambda: s.bytes_trsv(1)),
            ("mgs_givens", ggmres.PROF_MGS, None))

    def families(res, el):
        """per-family event timing of the solves in `res` (elapsed el seconds)"""
        fam = {}
        mgs_f, mgs_r, mgs_it = mgs_bytes(n, a.restart, [r["inner"] for r in res]) if not c5 else (0.0, 0.0, 0)
        for name, kind, per in FAMS:
            cnt, ms = s.profile_get(kind)
            if cnt == 0:
                continue
            avg_us = ms * 1e3 / cnt
            # (c5: the per-step cycle lengths are not collected, so MGS has no byte count -> null)
            byt = per() if per is not None else (mgs_f / mgs_it if mgs_it else None)
            fam[name] = {"launches": cnt, "avg_us": round(avg_us, 3),
                         "alg_bytes_per_launch": byt,
                         "achieved_gbs": round(byt / (avg_us * 1e-6) / 1e9, 1) if byt is not None else None,
                         "share_of_step": round(ms / (el * 1e3), 4)}
            if per is None and mgs_it:
                # SURVEY.md 8(d)'s unfused count over the same time: what the reference's
                # separate dot / AXPY / nrm2 launches would have had to move (not a roofline)
                ref = mgs_r / mgs_it
                fam[name]["reference_equiv_bytes_per_launch"] = ref
                fam[name]["reference_equiv_gbs"] = round(ref / (avg_us * 1e-6) / 1e9, 1)
        return fam

    def profiled_pass():
        """one step with every kernel family bracketed (events cost ~10 us per
        iteration, so this pass is kept out of the timed region)"""
        s.profile(True)
        barrier()
        t1 = time.perf_counter()
        r = step()
        barrier()
        fam = families([r], time.perf_counter() - t1)
        s.profile(False)
        return fam

    # breakdown pass in the last warmup step (or after the timed region when W = 0)
    fam = {}
    for w in range(a.warmup):
        if w == a.warmup - 1 and not a.no_profile:
            fam = profiled_pass()
        else:
            step()
    # roofline candidates: the single-kernel families (the SpMV when it has its
    # own launch, each triangular solve, the orthogonalization when one launch
    # per inner iteration does it: k_arnoldi_persist / k_arnoldi_wide) that the
    # breakdown pass finds within 2x of the largest.  Inside the timed region
    # ONE candidate is bracketed with events per solve, rotating, so every
    # candidate is timed live on the solver's stream at the perturbation of a
    # single family, and the roofline kernel is the one with the most time over
    # the timed region (not chosen from one warm-up step)
    kind_of = dict((f[0], f[1]) for f in FAMS)
    cands = []
    if not a.no_profile:
        if not c5 and s.mgs_kernel():
            KERNEL_NAMES["mgs_givens"] = s.mgs_kernel()
        fused_l = s.trsv_kernel(0).startswith("k_trsv_wave2d_spmv")
        single = {k: v for k, v in fam.items()
                  if k in KERNEL_NAMES and not (k == "spmv" and fused_l) and v.get("achieved_gbs") is not None}
        if single:
            top = max(v["share_of_step"] for v in single.values())
            cands = [k for k in ("spmv", "trsv_L", "trsv_U", "mgs_givens")
                     if k in single and single[k]["share_of_step"] >= 0.5 * top]
        elif not fam:
            cands = ["trsv_U"]
        s.profile(True, kinds=[kind_of[cands[0]]] if cands else [])
    bracketed = {k: 0 for k in cands}
    barrier()
    t0 = time.perf_counter()
    res = []
    for k in range(a.steps):
        if cands:
            c = cands[k % len(cands)]
            s.profile_select([kind_of[c]])
            bracketed[c] += 1
        res.append(step())
    barrier()
    el = time.perf_counter() - t0
    timed = families(res, el) if cands else {}
    s.profile(False)

    inner = sum(r["inner"] for r in res)
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    it = torch.tensor([float(inner)], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(it, op=dist.ReduceOp.SUM)
    el_max, inner_all = float(t.item()), float(it.item())
    value = inner_all / el_max
    if not a.no_profile and not fam:
        fam = profiled_pass()

    # time of each candidate over the whole timed region: its event-timed
    # average x its launches per solve x the solves
    for k in list(timed):
        if k not in bracketed or not bracketed[k]:
            timed.pop(k)
            continue
        f = timed[k]
        f["solves_bracketed"] = bracketed[k]
        f["est_ms_timed_region"] = round(f["avg_us"] * 1e-3 * f["launches"] / bracketed[k] * a.steps, 3)
        f["share_of_step"] = round(f["est_ms_timed_region"] / (el * 1e3), 4)
    # the roofline kernel: the most time over the timed region; candidates within
    # TIE_FRAC of it count as tied (L and U 1.4 % apart made the
    # choice a coin flip) and the tie goes to the lowest HBM fraction -- the
    # conservative figure, and a stable name from run to run
    dom = None
    if timed:
        order = sorted(timed, key=lambda k: -timed[k]["est_ms_timed_region"])
        top = timed[order[0]]["est_ms_timed_region"]
        tied = [k for k in order if timed[k]["est_ms_timed_region"] >= (1 - TIE_FRAC) * top
                and timed[k].get("achieved_gbs") is not None]
        dom = min(tied, key=lambda k: timed[k]["achieved_gbs"]) if tied else order[0]

    pmc_wl = ("c4" if c4 else "c3s" if c3s else ("pgr" if a.pg_perm == "random" else "pg") if pg
              else "netlist" if netlist else "c5" if c5 else None)
    if kilu:                            # ILU(k): its own PMC pass (tools/profile_round.sh c2_ilu1 / c3s_ilu1)
        pmc_wl = f"{pmc_wl or 'c2'}_ilu{kilu}"

    def roof_of(name):
        """(roofline, latency_roofline) of one timed family"""
        f = timed[name]
        if name == "spmv":
            KERNEL_NAMES["spmv"] = ("k_spmv_rtile" if s.spmv_rtile else "k_spmv_panel" if s.spmv_panels else
                                    "k_spmv_sell<false>" if s.spmv_sliced else "k_spmv_stream<false>")
        if name in ("trsv_L", "trsv_U") and not s.uses_wavefront:
            kname = ("k_trsv_level (one launch per dependency level; one 'launch' here = one triangle)"
                     if os.environ.get("GG_TRSV_LEVELS") == "1" else "k_trsv_flow")
        else:
            kname = KERNEL_NAMES[name]
        roof = {"kernel": kname, "bound": "hbm", "achieved": f["achieved_gbs"],
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(f["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(kname, pmc_wl),
                "alg_bytes_per_launch": f["alg_bytes_per_launch"], "avg_us": f["avg_us"],
                "launches_timed": f["launches"], "solves_bracketed": f["solves_bracketed"],
                "share_of_timed_region": f["share_of_step"]}
        if name == "mgs_givens":
            roof["alg_bytes_note"] = ("v_0..v_i and w read once, v_{i+1} written: 8 n (i+3) bytes at "
                                      "cycle index i, averaged over the launches timed")
        if name in ("trsv_L", "trsv_U"):
            # algorithmic = SURVEY.md 8(d)'s CSR share of B_ilu (12 nnz_T + 4 (n+1) + 16 n,
            # + B_spmv when the SpMV rides in the forward solve's launch); the
            # wavefront kernels stream no index arrays, so they move less than that
            which = 0 if name == "trsv_L" else 1
            sb = s.bytes_trsv_stream(which)
            if which == 0 and s.trsv_kernel(0).startswith("k_trsv_wave2d_spmv"):
                sb += s.bytes_spmv()
            roof["alg_bytes_note"] = "SURVEY.md 8(d): 12 nnz_T + 4 (n+1) + 16 n per triangle (+ B_spmv if fused)"
            roof["kernel_stream_bytes_per_launch"] = sb
        # the triangular solves are latency-bound: their other roofline is the
        # dependency chain, nx + ny - 1 wavefront steps at the bare per-step chain
        # latency (tools/lat_probe.hip on MI355X, profiles/r01/r01_lat_probe.txt)
        lat = None
        if name in ("trsv_L", "trsv_U") and s.uses_wavefront and not c5:
            # a non-unit L (the split engine's) divides like U
            mul = u_mul if name == "trsv_U" else l_mul
            fm = u_fma if name == "trsv_U" else l_fma
            cyc = CHAIN_CYCLES[chain_key(roof["kernel"], name, fm, mul)]
            # the DAG's longest path (ILU(k): skew k+1; 3D: nx + ny + nz - 2, whose
            # per-step chain is the 2D one: the tile kernel's plane term is off it)
            steps = 3 * a.c4_grid - 2 if c4 else a.grid + (kilu + 1) * (a.grid - 1)
            floor_us = steps * cyc / (SHADER_GHZ * 1e3)
            lat = {"kernel": roof["kernel"], "bound": "dependency chain", "critical_steps": steps,
                   "cycles_per_step": cyc, "clock_ghz": SHADER_GHZ, "floor_us": round(floor_us, 2),
                   "achieved_us": roof["avg_us"], "frac": round(floor_us / roof["avg_us"], 4)}
        elif name in ("trsv_L", "trsv_U") and not s.uses_wavefront:
            # the dataflow solve (k_trsv_flow): its chain is the triangle's level
            # count, each level one cross-workgroup hand-off (idle sc1 store -> sc1
            # poll: 0.47 us same XCD, profiles/r04/r04_xcd_handoff.txt)
            lv = s.trsv_levels(0 if name == "trsv_L" else 1)
            floor_us = lv * 0.47
            lat = {"kernel": roof["kernel"], "bound": "dependency chain (levels x hand-off)", "critical_steps": lv,
                   "us_per_step": 0.47, "floor_us": round(floor_us, 2), "achieved_us": roof["avg_us"],
                   "frac": round(floor_us / roof["avg_us"], 4)}
        return roof, lat

    roofs = {k: roof_of(k) for k in timed}
    roof, lat = roofs[dom] if dom else (None, None)
    if roof:
        roof["chosen_by"] = (f"most time over the timed region; candidates within {TIE_FRAC:.0%} of it tied, "
                             f"the lowest HBM fraction among them")
    # the whole Arnoldi iteration against HBM: the reference's
    # operations' algorithmic bytes per inner iteration at cycle index i --
    # SpMV + ILU apply + MGS 40 n (i+1) + norm/scale 24 n -- plus each cycle's
    # update (8 n m + 16 n) and residual (B_spmv + 8n + B_ilu + 8n + 16n), summed
    # over the timed solves' iterations, times it/s, over 8 TB/s
    iter_roof = None
    if not c5 and not kilu and not netlist:
        nnz_a = int(A.nnz)
        b_spmv = 12.0 * nnz_a + 4.0 * (n + 1) + 16.0 * n
        b_ilu = 12.0 * nnz_a + 8.0 * (n + 1) + 32.0 * n            # ILU(0): pattern of A
        tot_b = tot_it = 0.0
        for r in res:
            full, rem = divmod(int(r["inner"]), a.restart)
            for i in list(range(a.restart)) * full + list(range(rem)):
                tot_b += b_spmv + b_ilu + 40.0 * n * (i + 1) + 24.0 * n
                tot_it += 1
            cycles = full + (1 if rem else 0)
            tot_b += cycles * (8.0 * n * a.restart + 16.0 * n + b_spmv + 8.0 * n + b_ilu + 8.0 * n + 16.0 * n)
        if tot_it:
            per = tot_b / tot_it
            iter_roof = {"bytes_per_iteration": round(per), "achieved_gbs": round(per * value / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(per * value / 1e9 / HBM_PEAK_GBS, 4),
                         "basis": "SURVEY.md 8(d): the reference's unfused operations, ILU(0) (nnz_LU = nnz(A)); "
                                  "fused kernels move fewer bytes than this count"}
    rooflines = {k: dict(r, **({"latency_frac": l["frac"], "latency_floor_us": l["floor_us"]} if l else {}))
                 for k, (r, l) in roofs.items()}
    spmv_bytes = s.bytes_spmv()
    # isolated SpMV (4 rotating copies of A, x, y: > 256 MiB, not Infinity-Cache served)
    spmv_iso_ms = s.time_spmv(reps=100, nrot=4)
    spmv_iso = {"avg_us": round(spmv_iso_ms * 1e3, 3),
                "achieved_gbs": round(spmv_bytes / (spmv_iso_ms * 1e-3) / 1e9, 1),
                "frac": round(spmv_bytes / (spmv_iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    # ---- CPU baseline (rank 0, N=1): the oracle restatement -----------------------
    cpu = cpu_mt = None
    if rank == 0 and world == 1 and a.cpu_iters > 0 and not c5 and not c4 and not c3s:
        import oracle as O
        if pg or netlist:
            Ls, Us, mid, pr, pc, lsc, rsc = split
            osplit = O.Split(O.csr(Ls), O.csr(Us), mid, pr, pc, lsc, rsc)
        else:
            L, U = O.ilu0(A)
        # one core, pinned in-process (taskset -c 0 equivalent, no re-exec)
        aff = os.sched_getaffinity(0)
        core = min(aff)
        os.sched_setaffinity(0, {core})
        try:
            t1 = time.perf_counter()
            if pg or netlist:
                o = O.gmres_split(A, osplit, b, m=a.restart, max_iter=a.cpu_iters, tol=a.tol)
            else:
                o = O.gmres_left(A, L, U, b, m=a.restart, max_iter=a.cpu_iters, tol=a.tol)
            ct = time.perf_counter() - t1
        finally:
            os.sched_setaffinity(0, aff)
        cpu = {"value": round(o["inner"] / ct, 3), "unit": "iterations/s", "cores": 1,
               "kind": "port", "pinned_core": core, "nproc": os.cpu_count(),
               "affinity_cores": len(aff), "cpu_model": cpu_model(),
               "sample": f"oracle/ fp64 serial C restatement of {'GMRESilu (split)' if pg or netlist else 'GMRES_leftILU0'} on the same "
                         f"system, first {o['inner']} inner iterations ({ct:.1f} s), one thread "
                         f"pinned to core {core}"}
        # the same restatement on this process's cores (OpenMP build: SpMV,
        # BLAS-1 and update loops parallel, triangular solves serial as in the
        # reference's host engine; OMP_NUM_THREADS as the box sets it)
        try:
            O.use_mt(True)
            thr = O.threads()
            t1 = time.perf_counter()
            if pg or netlist:
                o = O.gmres_split(A, osplit, b, m=a.restart, max_iter=a.cpu_iters, tol=a.tol)
            else:
                o = O.gmres_left(A, L, U, b, m=a.restart, max_iter=a.cpu_iters, tol=a.tol)
            ct = time.perf_counter() - t1
            cpu_mt = {"value": round(o["inner"] / ct, 3), "unit": "iterations/s", "cores": thr,
                      "kind": "port", "affinity_cores": len(aff),
                      "sample": f"the same restatement built with OpenMP (liboracle_mt.so: SpMV, dots, AXPYs "
                                f"and the update on {thr} threads, the ILU triangular solves serial), "
                                f"first {o['inner']} inner iterations ({ct:.1f} s)"}
        finally:
            O.use_mt(False)

    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "iterations/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el_max * 1e3 / a.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": (f"C4: {a.c4_grid}^3 7-pt 3D thermal grid (kx=ky=1, kz=10, diag = "
                                f"sum|off| + 1e-3), ILU(0) left, GMRES({a.restart}), tol {a.tol:g}, "
                                f"b=A*1, x0=0, one solve per step, one GPU") if c4 else
                               (f"C5: {a.grid}x{a.grid} 5-pt grid, A = G + C/h (c 1e-3, h 1e-2), "
                                f"1% PULSE sources (own seeded scenarios), ILU(0) left, "
                                f"GMRES({a.restart}), tol {a.tol:g}, {a.c5_steps} backward-Euler "
                                f"steps per step, warm start, {a.c5_scenarios} scenario(s) per GPU"
                                + (" solved as one batch (gg_transient_batch)" if c5_batch else
                                   " on concurrent streams" if a.c5_scenarios > 1 else "")) if c5 else
                               (f"C3 stand-in: seeded power-law CSR with circuit5M's n and nnz "
                                f"(no parity claim at this size), ILU({kilu}) left (device-factored; "
                                f"C3 names ILU(1)), GMRES({a.restart}), tol {a.tol:g}, "
                                f"b=A*1, x0=0, one solve per step") if c3s else
                               (f"PG netlist (the reference's mna_solve_gpu_gmres workload): synthetic "
                                f"IBM-PG-style {a.grid}x{a.grid} R mesh + decaps + PULSE loads + {net_info['pads']} VDD "
                                f"pads (package R + V source) -> gg_host_read_netlist -> MNA A = G + C/h "
                                f"(h {net_info['h']:g}); PG engine (GMRESilu_GPU) with the split of the device ILU(0) "
                                f"of P_r A P_c (pivoting order: pad / branch unknowns first), unit scales, "
                                f"GMRES({a.restart}), tol {a.tol:g}, b = B u(t = {net_info['t']:g}), x0=0, "
                                f"one solve per step") if netlist else
                               (f"PG engine (GMRESilu_GPU) on the C2 grid: {a.grid}x{a.grid} 5-pt Laplacian, "
                                f"synthetic ILU++-style split (device ILU(0) of P_r D_l^-1 A D_r^-1 P_c, "
                                f"{a.pg_perm} permutations, seeded scales), GMRES({a.restart}), tol {a.tol:g}, "
                                f"b=A*1, x0=0, one solve per step") if pg else
                               (f"C2: {a.grid}x{a.grid} 5-pt Laplacian CSR, ILU({kilu}) left, "
                                f"GMRES({a.restart}), tol {a.tol:g}, b=A*1, x0=0, one solve per step"),
                   **({"netlist": net_info} if netlist else {}),
                   "n": n, "nnz": int(A.nnz), "restart": a.restart, "tol": a.tol,
                   "iters_per_solve": res[0]["inner"], "relres": res[0]["relres"],
                   "wavefront_sptrsv": s.uses_wavefront,
                   "spmv_fused_into_forward_solve": s.trsv_kernel(0).startswith("k_trsv_wave2d_spmv"),
                   "division": (("rows as two fused multiply-adds, in-line term first, U's b and "
                                 "coefficients pre-scaled by RN(1/d) (GG_DIV_FMA; tolerance parity "
                                 "1e-10 vs the reference's arithmetic)") if u_fma else
                                (f"x = acc * RN(1/d) on the wavefront {'L and U solves' if l_mul else 'U solve'} "
                                 f"(GG_DIV_RCP; tolerance parity 1e-10 vs the reference's division)")
                                if u_mul else
                                "x = RN(acc / d) (the reference's division, bit-exact)"),
                   "parallelism": "single" if world == 1 else f"replicas{world}",
                   "setup_s": round(t_setup, 3)},
        "roofline": roof, "latency_roofline": lat, "iteration_roofline": iter_roof,
        "rooflines": rooflines,
        "rooflines_from": ("one candidate family bracketed with hipEvents per timed solve, rotating; "
                           "roofline = the candidate with the most time over the timed region"),
        "kernels": fam,
        "kernels_from": "one profiled warmup step, every family bracketed by hipEvents",
        "spmv_isolated": spmv_iso,
        "cpu_baseline": cpu,
        "cpu_baseline_mt": cpu_mt,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    for s_ in (solvers if c5 else [s]):
        s_.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
