"""The reference-side boundary, executed: g++-built programs that link against
libggmres.so the way the reference's callers do (tests/boundary/*.cpp).

* gmresInterfacePGfloat / gmresInterfacePG (src/gmres_interface_pg.h, caller
  sequence src/mna_solve_gpu_gmres.cpp:507-545, 608-621): setPrecondPG on
  MySpMatrix / MySpMatrixDouble filled as the reference's feeders fill them,
  rhs_h / xgmres_h written directly, a sequence of solves that warm-start from
  the previous solution.  Checked per solve: the 0/1 return code, the
  max_it / tol write-back (GMRES_dev_PG and gmresInterfacePG::GMRES_host_PG
  write the iterations and the achieved relative residual; the float class's
  GMRES_host_PG solves with local copies, max_iter 60000, and leaves the
  members alone: src/gmres_interface_pg.cu:62-139) and x against the oracle's
  GMRESilu (orc_gmres_split) on the same fp32-rounded inputs: bit-identical
  with the device's reduction order, within 1e-10 of the serial order.
* wrapperGMRESforPG (src/gpuData.h:218-223): cs_dl matrices and a gpuETBR
  block with DC voltage sources plus PWL or PULSE current sources; the port
  waveforms x_single_host / x_host against the step driver restated
  (oracle.transient_mna: the DC point on G, then backward Euler on
  left = G + C/h with right = C/h, capacitor stamps between nodes included).
"""
import os
import struct
import subprocess

import numpy as np

import ggmres
import pytest
import scipy.sparse as sp

import oracle as O
from conftest import REPO
from ggmres import matrices as M
from helpers import device_layout, make_split

pytestmark = pytest.mark.gpu

BOUNDARY = os.path.join(REPO, "tests", "boundary")


def _run(prog, payload, tmp_path, out_bytes):
    exe = os.path.join(BOUNDARY, prog)
    assert os.path.exists(exe), f"{exe} not built (make -C tests/boundary)"
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(payload)
    p = subprocess.run([exe, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    data = fout.read_bytes()
    assert len(data) == out_bytes, (len(data), out_bytes)
    return data, p.stdout


def _csr_bytes(rp, ci, v, dtype):
    return (np.asarray(rp, np.int32).tobytes() + np.asarray(ci, np.int32).tobytes() +
            np.asarray(v, dtype).tobytes())


def _split_inputs(n_side, seed, double_scales):
    """A (float values), a synthetic ILU++ split of it (double factors, float
    middle, float or double scales), all as the fp32 boundary hands them over"""
    A64 = M.laplacian_5pt(n_side)
    A64.data = A64.data + np.random.default_rng(seed).uniform(-0.05, 0.05, A64.nnz)   # nonsymmetric
    A = sp.csr_matrix((A64.data.astype(np.float32), A64.indices, A64.indptr), shape=A64.shape)
    Ad = sp.csr_matrix((A.data.astype(np.float64), A.indices, A.indptr), shape=A.shape)
    P = make_split(Ad, seed=seed)
    mid32 = P.middle.astype(np.float32)
    sdt = np.float64 if double_scales else np.float32
    ls, rs = P.lscale.astype(sdt), P.rscale.astype(sdt)
    Pd = O.Split(P.L, P.U, mid32.astype(np.float64), P.perm_row, P.perm_col, ls.astype(np.float64),
                 rs.astype(np.float64))
    return A, Ad, P, Pd, mid32, ls, rs


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_pg_classes_solve_sequence(tmp_path, mode):
    """mode 0: gmresInterfacePGfloat::GMRES_dev_PG, 1: its GMRES_host_PG, 2:
    gmresInterfacePG::GMRES_host_PG (double scales)"""
    A, Ad, P, Pd, mid32, ls, rs = _split_inputs(30, seed=13 + mode, double_scales=(mode == 2))
    n = A.shape[0]
    rng = np.random.default_rng(40 + mode)
    nsteps = 3
    x0 = rng.standard_normal(n).astype(np.float32) * 0.1
    rhs = rng.uniform(0.0, 1.0, (nsteps, n)).astype(np.float32)
    hdr = struct.pack("<6i", mode, n, A.nnz, P.L.rp[n], P.U.rp[n], nsteps)
    sdt = np.float64 if mode == 2 else np.float32
    payload = (hdr + _csr_bytes(A.indptr, A.indices, A.data, np.float32) +
               _csr_bytes(P.L.rp, P.L.ci, P.L.v, np.float64) + _csr_bytes(P.U.rp, P.U.ci, P.U.v, np.float64) +
               mid32.tobytes() + P.perm_row.astype(np.int32).tobytes() + P.perm_col.astype(np.int32).tobytes() +
               ls.astype(sdt).tobytes() + rs.astype(sdt).tobytes() + x0.tobytes() + rhs.tobytes())
    rec = 12 + 4 * n
    data, stdout = _run("pg_driver", payload, tmp_path, nsteps * rec)
    # GMRES_dev_PG / gmresInterfacePG::GMRES_host_PG: max_it 10000 (written back);
    # gmresInterfacePGfloat::GMRES_host_PG: max_iter = 60000 (src/defs.h:11), members untouched
    max_iter = 60000 if mode == 1 else 10000
    # the engine's vector space: the split's flow path takes an RCM layout, a
    # deterministic function of the factors -- read it from a solver of our own
    ref = ggmres.Solver(0)
    try:
        ref.set_matrix(Ad)
        ref.set_precond_split(P.L, P.U, P.middle, P.perm_row, P.perm_col, P.lscale, P.rscale)
        lay, G = ref.layout()
    finally:
        ref.close()
    x = x0.astype(np.float64)
    for k in range(nsteps):
        rc, max_it, tol = struct.unpack_from("<iif", data, k * rec)
        xg = np.frombuffer(data, np.float32, n, k * rec + 12)
        b = rhs[k].astype(np.float64)
        o = O.gmres_split(Ad, Pd, b, x0=x, m=32, max_iter=max_iter, tol=1e-7)
        O.set_dot_order(lay, G)
        try:
            ot = O.gmres_split(Ad, Pd, b, x0=x, m=32, max_iter=max_iter, tol=1e-7)
        finally:
            O.set_dot_order(None)
        assert rc == ot["ret"] == o["ret"] == 0
        if mode == 0:
            # the device engine: bit-identical with the device's reduction order
            assert np.array_equal(xg, ot["x"].astype(np.float32))
            assert max_it == ot["iters"] and tol == np.float32(ot["relres"])
        else:
            # GMRES_host_PG: the host engine (csrc/host/gmres_host.cpp), the
            # reference's serial order -- bit-identical to the serial oracle
            assert np.array_equal(xg, o["x"].astype(np.float32))
            if mode == 1:
                assert max_it == 10000 and tol == np.float32(1e-7)  # local copies in the reference
            else:
                assert max_it == o["iters"] and tol == np.float32(o["relres"])
        assert np.linalg.norm(xg - o["x"]) <= 1e-6 * np.linalg.norm(o["x"])     # fp32 output
        x = xg.astype(np.float64)          # the next solve warm-starts from xgmres_h (fp32)
    assert "Failed to converge" not in stdout


def _csc_bytes(S):
    S = sp.csc_matrix(S)
    S.sort_indices()
    return (struct.pack("<3q", S.shape[0], S.shape[1], S.nnz) + S.indptr.astype(np.int64).tobytes() +
            S.indices.astype(np.int64).tobytes() + S.data.astype(np.float64).tobytes())


def _mna_system(nx, h):
    """a resistive grid G (grounded diagonal), C = node caps + coupling caps
    between in-line neighbours, B = one DC source at a node plus current
    sources between node pairs"""
    n = nx * nx
    G = M.laplacian_5pt(nx).tocsc() * 1e-1
    rng = np.random.default_rng(3)
    c = sp.diags(rng.uniform(0.5e-3, 1.5e-3, n))
    ii = np.arange(0, n - 1, 7)
    ii = ii[(ii % nx) != nx - 1]
    cc = 2e-4
    coup = sp.csc_matrix((np.concatenate([np.full(len(ii), cc), np.full(len(ii), cc),
                                          np.full(len(ii), -cc), np.full(len(ii), -cc)]),
                          (np.concatenate([ii, ii + 1, ii, ii + 1]), np.concatenate([ii, ii + 1, ii + 1, ii]))),
                         shape=(n, n))
    C = (c + coup).tocsc()
    nIS = 6
    a = rng.choice(n, nIS, replace=False)
    bnode = rng.choice(n, nIS, replace=False)
    rows = [n // 2] + list(a) + list(bnode)
    cols = [0] + list(range(1, nIS + 1)) + list(range(1, nIS + 1))
    vals = [1.0] + [1.0] * nIS + [-1.0] * nIS
    B = sp.csc_matrix((vals, (rows, cols)), shape=(n, 1 + nIS))
    left = (G + C / h).tocsc()
    right = (C / h).tocsc()
    return n, G, left, right, B, nIS


@pytest.mark.parametrize("kind", ["pwl", "pulse", "mixed"])
def test_wrapper_gmres_for_pg(tmp_path, kind):
    """mixed: a netlist with both PWL and PULSE current sources -- each source
    takes its own waveform (PWL where it has points, else its PULSE row;
    include/compat/gpuData.h), PWL point counts above MAX_PWL_PTS clamped"""
    nx, h, numPts = 24, 1e-2, 40
    n, G, left, right, B, nIS = _mna_system(nx, h)
    nVS = 1
    ports = np.array([0, n // 3, n // 2, n - 1], np.int32)
    dc = np.array([2e-3])
    code = {"pwl": 1, "pulse": 2, "mixed": 3}[kind]
    hdr = struct.pack("<8i", n, nVS, nIS, numPts, len(ports), code, 1, 1) + struct.pack("<d", h)
    payload = hdr + b"".join(_csc_bytes(S) for S in (left, right, G, B)) + ports.tobytes() + dc.tobytes()
    srcs = [(O.SRC_DC, [dc[0]])]
    npts = np.array([4, 3, 5, 2, 4, 3], np.int32) if kind == "pwl" else np.array([4, 0, 5, 0, 70, 0], np.int32)
    pt = np.array([[k * h, 3 * h, 2 * h, 8 * h, 20 * h] for k in range(nIS)])   # td tr tf tw tp
    pv = np.array([[0.0, 1e-3 * (1 + k)] for k in range(nIS)])                  # vlo vhi
    if kind in ("pwl", "mixed"):
        tt = np.zeros((nIS, 64))
        vv = np.zeros((nIS, 64))
        for k in range(nIS):
            c = min(int(npts[k]), 64)
            t = np.cumsum(np.random.default_rng(k).uniform(2 * h, 9 * h, c))
            v = np.random.default_rng(50 + k).uniform(-1e-3, 1e-3, c)
            tt[k, :c], vv[k, :c] = t, v
        payload += npts.tobytes() + tt.tobytes() + vv.tobytes()
    if kind in ("pulse", "mixed"):
        payload += pt.tobytes() + pv.tobytes()
    for k in range(nIS):
        if kind != "pulse" and npts[k] > 0:
            c = min(int(npts[k]), 64)
            srcs.append((O.SRC_PWL, np.stack([tt[k, :c], vv[k, :c]], 1).reshape(-1)))
        else:
            srcs.append((O.SRC_PULSE, [pv[k, 0], pv[k, 1], *pt[k]]))
    data, stdout = _run("wrapper_driver", payload, tmp_path, numPts * len(ports) * 12)
    xs = np.frombuffer(data, np.float32, numPts * len(ports)).reshape(numPts, len(ports))
    xd = np.frombuffer(data, np.float64, numPts * len(ports), numPts * len(ports) * 4).reshape(numPts, len(ports))
    # the restated step driver, device reduction order
    LG, UG = O.ilu0(G)
    LA, UA = O.ilu0(left)
    lay, Gd = device_layout(n, nx)
    O.set_dot_order(lay, Gd)
    try:
        dcp = O.transient_mna(G, LG, UG, 0, 1, h, None, B, srcs, ports, np.zeros(n), m=32, tol=1e-7)
        x0 = dcp["x"]
        tr = O.transient_mna(left, LA, UA, 1, numPts - 1, h, right, B, srcs, ports, x0, m=32, tol=1e-7)
    finally:
        O.set_dot_order(None)
    ref = np.concatenate([dcp["ports"][:, 1:2], tr["ports"][:, 1:]], axis=1).T       # [numPts, nport]
    assert np.array_equal(xd, ref)
    assert np.array_equal(xs, ref.astype(np.float32))
    assert np.max(np.abs(ref)) > 0 and np.max(np.abs(np.diff(ref, axis=0))) > 0     # driven, time-varying
    assert "Failed to converge" not in stdout


def test_wrapper_failure_fills_nan(tmp_path):
    """a failing call (here a port outside the system) cannot be mistaken for
    results: every requested output element is NaN (include/compat/gpuData.h)"""
    nx, h, numPts = 12, 1e-2, 5
    n, G, left, right, B, nIS = _mna_system(nx, h)
    ports = np.array([0, n + 5], np.int32)
    hdr = struct.pack("<8i", n, 1, nIS, numPts, len(ports), 0, 1, 1) + struct.pack("<d", h)
    payload = hdr + b"".join(_csc_bytes(S) for S in (left, right, G, B)) + ports.tobytes() + \
        np.array([1e-3]).tobytes()
    data, _ = _run("wrapper_driver", payload, tmp_path, numPts * len(ports) * 12)
    xs = np.frombuffer(data, np.float32, numPts * len(ports))
    xd = np.frombuffer(data, np.float64, numPts * len(ports), numPts * len(ports) * 4)
    assert np.all(np.isnan(xs)) and np.all(np.isnan(xd))


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_engine_abi_preconditioner_plugin(tmp_path, mode):
    """GMRES_GPU / GMRES_GPU_tran / GMRESilu_GPU / GMRESilu (src/gmres.h:356-398)
    called by a g++ program with its own Preconditioner subclass (Jacobi:
    left M = D, split Ml = Mr = D^-1/2, start D^1/2; src/preconditioner.h:34-84).
    The plug-in works on fp32 arrays (the reference's interface) while the
    engine is fp64, so the check is against the oracle's GMRES with the same
    operators in fp64 (left: L = I, U = D; split: L = U = I, D_l = D_r = D^1/2)
    to fp32 tolerance: same convergence, iteration count within 2, x within
    1e-5, and the plug-in called once per operator application."""
    A64 = M.laplacian_5pt(16)
    A64.data = A64.data + np.random.default_rng(21).uniform(-0.3, 0.3, A64.nnz)   # nonsymmetric, D != 4
    A = sp.csr_matrix((A64.data.astype(np.float32), A64.indices, A64.indptr), shape=A64.shape)
    Ad = sp.csr_matrix((A.data.astype(np.float64), A.indices, A.indptr), shape=A.shape)
    n = A.shape[0]
    b = (Ad @ np.ones(n)).astype(np.float32)
    x0 = np.zeros(n, np.float32)
    m, max_iter, tol = 30, 2000, 1e-5
    hdr = struct.pack("<5if", mode, n, A.nnz, m, max_iter, tol)
    payload = hdr + _csr_bytes(A.indptr, A.indices, A.data, np.float32) + b.tobytes() + x0.tobytes()
    data, _ = _run("engine_driver", payload, tmp_path, 12 + 20 + 4 * n)
    rc, it, tol_out = struct.unpack_from("<iif", data, 0)
    calls = np.frombuffer(data, np.int32, 5, 12)
    xg = np.frombuffer(data, np.float32, n, 32).astype(np.float64)
    d = Ad.diagonal()
    eye = O.csr(sp.identity(n, format="csr"))
    if mode <= 1:
        o = O.gmres_left(Ad, eye, O.csr(sp.diags(d).tocsr()), b.astype(np.float64), m=m, max_iter=max_iter,
                         tol=tol)
    else:
        sq = np.sqrt(d)
        ident = np.arange(n, dtype=np.int32)
        Pj = O.Split(eye, eye, np.ones(n), ident, ident, sq, sq)
        o = O.gmres_split(Ad, Pj, b.astype(np.float64), m=m, max_iter=max_iter, tol=tol)
    assert rc == o["ret"] == 0
    assert np.linalg.norm(xg - o["x"]) <= 1e-5 * np.linalg.norm(o["x"])
    if mode == 1:        # GMRES_GPU_tran: limits by value, nothing written back
        assert it == max_iter and tol_out == np.float32(tol)
    else:
        assert abs(it - o["iters"]) <= 2 and tol_out <= tol
    iters = o["iters"]
    if mode <= 1:        # DevPrecond: b, the initial residual, one per inner iteration
        assert calls[0] >= iters + 2 and calls[1:].sum() == 0
    else:                # _rhs for b and residuals, _left / _right per iteration, _starting_value once
        assert calls[0] == 0 and calls[3] == 1 and calls[4] >= 2
        assert abs(calls[1] - iters) <= 2 and calls[2] >= calls[1]


def test_engine_abi_tran_keeps_its_solver(tmp_path):
    """a transient caller (src_thermal/main2.cu:470-506) runs
    100 GMRES_GPU_tran steps with one GMRES_GPU_Data: the engine is set up by the
    first call only (no gg_set_matrix during the 100 steps), each step costs
    within 10 % of the same solve through the C ABI alone (one gg_solver set up
    once, gg_solve_device_f32, the same plug-in), and both give the same bits"""
    A64 = (M.laplacian_5pt(64) + 2.0 * sp.identity(64 * 64)).tocsr()     # diagonally dominant: ~20 iterations
    A64.sort_indices()
    A64.data = A64.data + np.random.default_rng(5).uniform(-0.3, 0.3, A64.nnz)
    A = sp.csr_matrix((A64.data.astype(np.float32), A64.indices, A64.indptr), shape=A64.shape)
    n = A.shape[0]
    b = (sp.csr_matrix((A.data.astype(np.float64), A.indices, A.indptr), shape=A.shape) @ np.ones(n))
    b = b.astype(np.float32)
    x0 = np.zeros(n, np.float32)
    hdr = struct.pack("<5if", 4, n, A.nnz, 30, 2000, 1e-5)
    payload = hdr + _csr_bytes(A.indptr, A.indices, A.data, np.float32) + b.tobytes() + x0.tobytes()
    data, _ = _run("engine_driver", payload, tmp_path, 8 + 16 + 8 * n)
    rc, setups = struct.unpack_from("<ii", data, 0)
    tran_ms, direct_ms = struct.unpack_from("<dd", data, 8)
    xt = np.frombuffer(data, np.float32, n, 24)
    xc = np.frombuffer(data, np.float32, n, 24 + 4 * n)
    print(f"GMRES_GPU_tran {tran_ms:.3f} ms/step, C ABI alone {direct_ms:.3f} ms/step, setups {setups}")
    assert rc == 0 and setups == 0
    assert tran_ms <= 1.10 * direct_ms + 0.05, (tran_ms, direct_ms)
    assert np.array_equal(xt, xc)
