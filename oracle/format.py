"""Test infrastructure only: restatement of the reference's boundary feed,
src/formatConvert.cpp, used by tests/test_format.py to check
gpu-gmres_amd/csrc/compat/format_convert.cpp.

coo2csr_in / coo2csrDouble_in (:112-216): in-place COO -> CSR by following
displacement cycles from the lowest unplaced entry, i_idx doubling as the
"placed" flag (-1) and then as the row pointers, then a bubble sort of every
row by column (sort / sortDouble, :66-105).
LDcsc2csrMySpMatrix(Double) (:300-398): CSC (nzmax entries) -> COO -> the above.
"""
import numpy as np


def coo2csr_in(nrows, a, i_idx, j_idx):
    """returns (row_ptr, col, val) exactly as the in-place reference leaves them"""
    a = list(a)
    ii = list(i_idx) + [0] * max(0, nrows + 1 - len(i_idx))
    jj = list(j_idx)
    nz = len(a)
    row_start = [0] * (nrows + 1)
    for k in range(nz):
        row_start[ii[k] + 1] += 1
    for r in range(nrows):
        row_start[r + 1] += row_start[r]
    init = 0
    while init < nz:
        dt, i, j = a[init], ii[init], jj[init]
        ii[init] = -1
        while True:
            pos = row_start[i]
            a_next, i_next, j_next = a[pos], ii[pos], jj[pos]
            a[pos], jj[pos], ii[pos] = dt, j, -1
            row_start[i] += 1
            if i_next < 0:
                break
            dt, i, j = a_next, i_next, j_next
        init += 1
        while init < nz and ii[init] < 0:
            init += 1
    rp = [0] + [row_start[r] for r in range(nrows)]
    for r in range(nrows):
        lb, ub = rp[r], rp[r + 1]
        for top in range(ub - 1, lb, -1):
            for k in range(lb, top):
                if jj[k] > jj[k + 1]:
                    a[k], a[k + 1] = a[k + 1], a[k]
                    jj[k], jj[k + 1] = jj[k + 1], jj[k]
    return np.array(rp, np.int64), np.array(jj, np.int64), np.array(a)


def csc2csr(m, p, i, x):
    """LDcsc2csrMySpMatrixDouble: CSC arrays -> (row_ptr, col, val)"""
    cols = []
    for j in range(len(p) - 1):
        cols += [j] * (p[j + 1] - p[j])
    return coo2csr_in(m, list(x), [int(t) for t in i], cols)
