"""GMRES_host_PG's host engine (gpu-gmres_amd/csrc/host/gmres_host.cpp: the
reference's GMRESilu, src/gmres.cu:2069-2252, with MyILUPP's Host* applies,
src/preconditioner.cu:1074-1137) on the CPU, no GPU involved: the g++-built
boundary driver (tests/boundary/pg_driver.cpp) calls
gmresInterfacePG(float)::GMRES_host_PG through libggmres.so; the device
set-up fails here (no GPU) and only GMRES_dev_PG would need it.  Every solve
of the warm-started sequence is bit-identical (fp32 output) to the oracle's
GMRESilu restatement in the reference's serial order on the same fp32-rounded
inputs, with the same iteration count and relative residual written back."""
import os
import struct
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
from conftest import REPO
from ggmres import matrices as M
from helpers import make_split

BOUNDARY = os.path.join(REPO, "tests", "boundary")


def _driver():
    exe = os.path.join(BOUNDARY, "pg_driver")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", BOUNDARY, "pg_driver"], check=True, capture_output=True)
    return exe


@pytest.mark.parametrize("mode,side", [(1, 30), (2, 30), (2, 200)])
def test_host_engine_bitexact_vs_serial_oracle(tmp_path, mode, side):
    """mode 1: gmresInterfacePGfloat::GMRES_host_PG (float scales, max_iter
    60000, members untouched); 2: gmresInterfacePG::GMRES_host_PG (double
    scales, max_it / tol written back); side 200 (40,000 rows) runs the
    element-wise loops on the thread pool"""
    # (the large case: the transient system G + C/h, which GMRES(32) with an
    # ILU(0) split solves in tens of iterations at 40,000 rows)
    A64 = M.laplacian_5pt(side) if side <= 100 else M.transient(M.laplacian_5pt(side), c=1e-3, h=1e-2).tocsr()
    A64.data = A64.data + np.random.default_rng(side + mode).uniform(-0.05, 0.05, A64.nnz)
    A = sp.csr_matrix((A64.data.astype(np.float32), A64.indices, A64.indptr), shape=A64.shape)
    Ad = sp.csr_matrix((A.data.astype(np.float64), A.indices, A.indptr), shape=A.shape)
    # (the large case keeps the grid order: a randomly permuted ILU(0) of 40,000
    # rows would need far more than max_it iterations)
    P = make_split(Ad, seed=side + mode, identity_perm=side > 100)
    mid32 = P.middle.astype(np.float32)
    sdt = np.float64 if mode == 2 else np.float32
    ls, rs = P.lscale.astype(sdt), P.rscale.astype(sdt)
    Pd = O.Split(P.L, P.U, mid32.astype(np.float64), P.perm_row, P.perm_col, ls.astype(np.float64),
                 rs.astype(np.float64))
    n = A.shape[0]
    rng = np.random.default_rng(7 * side + mode)
    nsteps = 3
    x0 = rng.standard_normal(n).astype(np.float32) * 0.1
    rhs = rng.uniform(0.0, 1.0, (nsteps, n)).astype(np.float32)
    cb = lambda rp, ci, v, dt: (np.asarray(rp, np.int32).tobytes() + np.asarray(ci, np.int32).tobytes() +
                                np.asarray(v, dt).tobytes())
    payload = (struct.pack("<6i", mode, n, A.nnz, P.L.rp[n], P.U.rp[n], nsteps) +
               cb(A.indptr, A.indices, A.data, np.float32) + cb(P.L.rp, P.L.ci, P.L.v, np.float64) +
               cb(P.U.rp, P.U.ci, P.U.v, np.float64) + mid32.tobytes() + P.perm_row.astype(np.int32).tobytes() +
               P.perm_col.astype(np.int32).tobytes() + ls.tobytes() + rs.tobytes() + x0.tobytes() + rhs.tobytes())
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(payload)
    p = subprocess.run([_driver(), str(fin), str(fout)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    data = fout.read_bytes()
    rec = 12 + 4 * n
    assert len(data) == nsteps * rec
    max_iter = 60000 if mode == 1 else 10000
    x = x0.astype(np.float64)
    for k in range(nsteps):
        rc, max_it, tol = struct.unpack_from("<iif", data, k * rec)
        xg = np.frombuffer(data, np.float32, n, k * rec + 12)
        o = O.gmres_split(Ad, Pd, rhs[k].astype(np.float64), x0=x, m=32, max_iter=max_iter, tol=1e-7)
        assert rc == o["ret"] == 0
        assert np.array_equal(xg, o["x"].astype(np.float32)), k
        if mode == 1:
            assert max_it == 10000 and tol == np.float32(1e-7)
        else:
            assert max_it == o["iters"] and tol == np.float32(o["relres"])
        x = xg.astype(np.float64)
    assert "Failed to converge" not in p.stdout
