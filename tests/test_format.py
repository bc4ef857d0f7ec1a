"""The boundary feed: COO/CSC -> CSR conversions of
src/formatConvert.cpp, through the C ABI wrapper and through the reference's
C++ symbols (a small program linked against libggmres.so), against the
restatement in oracle/format.py.  Integer work and value moves: exact."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO
from oracle import format as OF

PI = ctypes.POINTER(ctypes.c_int)
PD = ctypes.POINTER(ctypes.c_double)


def random_coo(nrows, ncols, nz, seed):
    rng = np.random.default_rng(seed)
    r = rng.integers(0, nrows, nz)
    c = rng.integers(0, ncols, nz)
    dup = rng.integers(0, nz, nz // 5)        # repeated (row, col) pairs
    r[: len(dup)] = r[dup]
    c[: len(dup)] = c[dup]
    return r.astype(np.int32), c.astype(np.int32), rng.standard_normal(nz)


@pytest.mark.parametrize("shape", [(1, 1, 1), (7, 5, 30), (50, 50, 400), (300, 20, 2000)])
def test_coo2csr_in_exact(ggmres_lib, shape):
    nrows, ncols, nz = shape
    r, c, v = random_coo(nrows, ncols, nz, nz)
    ri = np.zeros(max(nz, nrows + 1), np.int32)
    ri[:nz] = r
    cj = c.copy()
    vv = v.copy()
    rc = ggmres_lib.gg_host_coo2csr_in(ctypes.c_int(nrows), ctypes.c_int(nz), vv.ctypes.data_as(PD),
                                       ri.ctypes.data_as(PI), cj.ctypes.data_as(PI))
    assert rc == 0
    rp, col, val = OF.coo2csr_in(nrows, v, r, c)
    assert np.array_equal(ri[: nrows + 1], rp)
    assert np.array_equal(cj, col) and np.array_equal(vv, val)


def test_coo2csr_in_rejects_bad_rows(ggmres_lib):
    ri = np.array([0, 5], np.int32)
    cj = np.array([0, 0], np.int32)
    v = np.zeros(2)
    assert ggmres_lib.gg_host_coo2csr_in(ctypes.c_int(3), ctypes.c_int(2), v.ctypes.data_as(PD),
                                         ri.ctypes.data_as(PI), cj.ctypes.data_as(PI)) != 0


PROG = r"""
#include <cstdio>
#include "format_convert.h"
int main() {
    long p[] = {0, 2, 3, 6, 7};            // 4 x 4 CSC, unsorted rows inside columns
    long i[] = {3, 0, 2, 1, 3, 0, 2};
    double x[] = {1.5, -2, 3.25, 4, 5, -6.5, 7};
    ucr_cs_dl M;
    M.shallowCpy(7, 4, 4, p, i, x, -1);
    MySpMatrixDouble D;
    LDcsc2csrMySpMatrixDouble(&D, &M);
    MySpMatrix F;
    LDcsc2csrMySpMatrix(&F, &M);
    for (int r = 0; r <= D.numRows; r++) std::printf("%d ", D.rowIndices[r]);
    std::printf("\n");
    for (int k = 0; k < D.numNZEntries; k++) std::printf("%d:%.17g:%.9g ", D.indices[k], D.val[k], F.val[k]);
    std::printf("\n%d %d\n", F.isCSR, F.indices[3]);
    return 0;
}
"""


def test_reference_symbols_link_and_convert(tmp_path, ggmres_lib):
    src = tmp_path / "conv.cpp"
    src.write_text(PROG)
    exe = tmp_path / "conv"
    lib = os.path.join(PKG, "lib")
    subprocess.check_call(["g++", "-std=c++11", "-I", os.path.join(REPO, "include", "compat"),
                           "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe),
                           "-L", lib, "-Wl,-rpath," + lib, "-lggmres"])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    rp = [int(t) for t in out[0].split()]
    ents = [t.split(":") for t in out[1].split()]
    ref_rp, ref_col, ref_val = OF.csc2csr(4, [0, 2, 3, 6, 7], [3, 0, 2, 1, 3, 0, 2],
                                          [1.5, -2, 3.25, 4, 5, -6.5, 7])
    assert rp == list(ref_rp)
    assert [int(e[0]) for e in ents] == list(ref_col)
    assert [float(e[1]) for e in ents] == list(ref_val)
    assert [float(e[2]) for e in ents] == [float(np.float32(v)) for v in ref_val]
    assert out[2].split()[0] == "1"
