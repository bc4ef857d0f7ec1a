// format_convert.cpp -- include/compat/format_convert.h: the reference's CSC ->
// CSR boundary feed (src/formatConvert.cpp:112-216, 300-398), same results.
#include <cstdlib>
#include <cstring>

#include "format_convert.h"
#include "ggmres.h"
#include "ggmres_host.h"

namespace {

// in-place COO -> CSR: entries move to their row's next free slot by
// following displacement cycles, started from the lowest unplaced position;
// i_idx is the placed/unplaced marker during the pass and the row pointer
// array after it; then each row is bubble-sorted by column (stable)
template <class T>
void coo_to_csr_inplace(int nrows, int nz, T *a, int *ri, int *cj)
{
    int *next = static_cast<int *>(std::malloc(sizeof(int) * (nrows + 1)));
    for (int r = 0; r <= nrows; r++) next[r] = 0;
    for (int k = 0; k < nz; k++) next[ri[k] + 1]++;
    for (int r = 0; r < nrows; r++) next[r + 1] += next[r];
    int start = 0;
    while (start < nz) {
        T carry_v = a[start];
        int carry_r = ri[start], carry_c = cj[start];
        ri[start] = -1;
        for (;;) {
            const int dst = next[carry_r]++;
            const T dv = a[dst];
            const int dr = ri[dst], dc = cj[dst];
            a[dst] = carry_v;
            cj[dst] = carry_c;
            ri[dst] = -1;
            if (dr < 0) break;              // the slot held an entry already placed (or the start)
            carry_v = dv;
            carry_r = dr;
            carry_c = dc;
        }
        start++;
        while (start < nz && ri[start] < 0) start++;
    }
    // next[r] now ends row r: row pointers into i_idx
    for (int r = 0; r < nrows; r++) ri[r + 1] = next[r];
    ri[0] = 0;
    std::free(next);
    for (int r = 0; r < nrows; r++) {
        const int lb = ri[r], ub = ri[r + 1];
        for (int top = ub - 1; top > lb; top--)
            for (int k = lb; k < top; k++)
                if (cj[k] > cj[k + 1]) {
                    const T tv = a[k];
                    a[k] = a[k + 1];
                    a[k + 1] = tv;
                    const int tc = cj[k];
                    cj[k] = cj[k + 1];
                    cj[k + 1] = tc;
                }
    }
}

template <class T, class S>
void csc_to_csr(S *out, ucr_cs_dl *M)
{
    const int nnz = (int)M->nzmax, m = (int)M->m, n = (int)M->n;
    out->numRows = m;
    out->numCols = n;
    out->numNZEntries = nnz;
    out->rowIndices = static_cast<int *>(std::malloc(sizeof(int) * (nnz > m + 1 ? nnz : m + 1)));
    out->indices = static_cast<int *>(std::malloc(sizeof(int) * (nnz > 0 ? nnz : 1)));
    out->val = static_cast<T *>(std::malloc(sizeof(T) * (nnz > 0 ? nnz : 1)));
    for (int j = 0; j < n; j++)
        for (long int k = M->p[j]; k < M->p[j + 1]; k++) out->indices[k] = j;
    for (int k = 0; k < nnz; k++) {
        out->rowIndices[k] = (int)M->i[k];
        out->val[k] = (T)M->x[k];
    }
    coo_to_csr_inplace<T>(m, nnz, out->val, out->rowIndices, out->indices);
}

}  // namespace

void coo2csr_in(int numRows, int nz, float *a, int *i_idx, int *j_idx)
{
    coo_to_csr_inplace<float>(numRows, nz, a, i_idx, j_idx);
}

void coo2csrDouble_in(int numRows, int nz, double *a, int *i_idx, int *j_idx)
{
    coo_to_csr_inplace<double>(numRows, nz, a, i_idx, j_idx);
}

void LDcsc2csrMySpMatrix(MySpMatrix *mySpM, ucr_cs_dl *M)
{
    mySpM->isCSR = 1;
    csc_to_csr<float>(mySpM, M);
}

void LDcsc2csrMySpMatrixDouble(MySpMatrixDouble *mySpM, ucr_cs_dl *M)
{
    csc_to_csr<double>(mySpM, M);
}

void LDcsc2cscMySpMatrix(MySpMatrix *mySpM, ucr_cs_dl *M)
{
    mySpM->isCSR = 0;
    const int nnz = (int)M->nzmax, m = (int)M->m, n = (int)M->n;
    mySpM->numRows = m;
    mySpM->numCols = n;
    mySpM->numNZEntries = nnz;
    mySpM->rowIndices = static_cast<int *>(std::malloc(sizeof(int) * (n + 1)));
    mySpM->indices = static_cast<int *>(std::malloc(sizeof(int) * (nnz > 0 ? nnz : 1)));
    mySpM->val = static_cast<float *>(std::malloc(sizeof(float) * (nnz > 0 ? nnz : 1)));
    for (int j = 0; j <= n; j++) mySpM->rowIndices[j] = (int)M->p[j];
    for (int k = 0; k < nnz; k++) {
        mySpM->indices[k] = (int)M->i[k];
        mySpM->val[k] = (float)M->x[k];
    }
}

extern "C" int gg_host_coo2csr_in(int nrows, int nz, double *val, int *row_idx, int *col_idx)
{
    if (nrows < 0 || nz < 0 || (nz > 0 && (!val || !row_idx || !col_idx))) return GG_EINVAL;
    for (int k = 0; k < nz; k++)
        if (row_idx[k] < 0 || row_idx[k] >= nrows) return GG_EINVAL;
    coo2csrDouble_in(nrows, nz, val, row_idx, col_idx);
    return GG_OK;
}
