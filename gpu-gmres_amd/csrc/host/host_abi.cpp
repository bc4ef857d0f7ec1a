// host_abi.cpp -- include/ggmres_host.h: setup-phase entry points (no device).
#include <cstdlib>
#include <cstring>

#include "../gg_internal.h"
#include "ggmres_host.h"

using namespace gg;

namespace {

Csr wrap(int n, const int *rp, const int *ci, const double *v)
{
    Csr C;
    C.n = n;
    C.rp.assign(rp, rp + n + 1);
    C.ci.assign(ci, ci + rp[n]);
    C.v.assign(v, v + rp[n]);
    return C;
}

void emit(const Csr &C, int *rp, int **ci, double **v)
{
    std::memcpy(rp, C.rp.data(), sizeof(int) * (C.n + 1));
    size_t nnz = C.ci.size();
    *ci = (int *)std::malloc(sizeof(int) * (nnz ? nnz : 1));
    *v = (double *)std::malloc(sizeof(double) * (nnz ? nnz : 1));
    if (nnz) {
        std::memcpy(*ci, C.ci.data(), sizeof(int) * nnz);
        std::memcpy(*v, C.v.data(), sizeof(double) * nnz);
    }
}

}  // namespace

extern "C" {

int gg_host_ilu0(int n, const int *rp, const int *ci, const double *v, int *l_rp, int **l_ci,
                 double **l_v, int *u_rp, int **u_ci, double **u_v)
{
    if (n < 0 || !rp || !l_rp || !u_rp || !l_ci || !l_v || !u_ci || !u_v) return GG_EINVAL;
    try {
        Csr L, U;
        ilu0_left(wrap(n, rp, ci, v), L, U);
        emit(L, l_rp, l_ci, l_v);
        emit(U, u_rp, u_ci, u_v);
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_iluk(int level, int n, const int *rp, const int *ci, const double *v, int *l_rp,
                 int **l_ci, double **l_v, int *u_rp, int **u_ci, double **u_v)
{
    if (n < 0 || level < 0 || !rp || !l_rp || !u_rp || !l_ci || !l_v || !u_ci || !u_v) return GG_EINVAL;
    try {
        Csr L, U;
        int rc = iluk_itsol(wrap(n, rp, ci, v), level, L, U);
        if (rc) return rc;
        emit(L, l_rp, l_ci, l_v);
        emit(U, u_rp, u_ci, u_v);
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_wave2d(int n, const int *l_rp, const int *l_ci, const double *l_v, const int *u_rp,
                   const int *u_ci, const double *u_v, int *nx, int *ny)
{
    try {
        Wave2D w = detect_wave2d(canon_lower_unit(wrap(n, l_rp, l_ci, l_v)),
                                 canon_upper_ignorezero(wrap(n, u_rp, u_ci, u_v)));
        if (nx) *nx = w.nx;
        if (ny) *ny = w.ny;
        return w.ok ? 1 : 0;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_wave3d(int n, const int *l_rp, const int *l_ci, const double *l_v, const int *u_rp,
                   const int *u_ci, const double *u_v, int *nx, int *ny, int *nz)
{
    try {
        Wave2D w = detect_wave3d(canon_lower_unit(wrap(n, l_rp, l_ci, l_v)),
                                 canon_upper_ignorezero(wrap(n, u_rp, u_ci, u_v)));
        if (nx) *nx = w.nx;
        if (ny) *ny = w.ny;
        if (nz) *nz = w.nz;
        return w.ok ? 1 : 0;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_partition(int n, const int *rp, const int *ci, int nparts, int method, int *node_part,
                      int *part_size, int *pinv, int *q)
{
    if (n < 1 || !rp || !ci || nparts < 1 || nparts > n || !node_part || !part_size || !pinv || !q ||
        (method != GG_PART_BISECT && method != GG_PART_BLOCKS))
        return GG_EINVAL;
    try {
        std::vector<double> none(rp[n], 0.0);
        Csr A = wrap(n, rp, ci, none.data());
        std::vector<int> np_, ps, pi, qq;
        partition_arrow(A, nparts, method, np_, ps, pi, qq);
        std::copy(np_.begin(), np_.end(), node_part);
        std::copy(ps.begin(), ps.end(), part_size);
        std::copy(pi.begin(), pi.end(), pinv);
        std::copy(qq.begin(), qq.end(), q);
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_permute(int n, const int *rp, const int *ci, const double *v, const int *pinv, const int *q,
                    int *b_rp, int **b_ci, double **b_v)
{
    if (n < 0 || !rp || !pinv || !q || !b_rp || !b_ci || !b_v) return GG_EINVAL;
    try {
        std::vector<int> pi(pinv, pinv + n), qq(q, q + n);
        for (int i = 0; i < n; i++)
            if (qq[i] < 0 || qq[i] >= n || pi[qq[i]] != i) return GG_EINVAL;
        emit(arrow_permute(wrap(n, rp, ci, v), pi, qq), b_rp, b_ci, b_v);
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_block(int n, const int *rp, const int *ci, const double *v, int r0, int r1, int c0, int c1,
                  int *b_rp, int **b_ci, double **b_v)
{
    if (n < 0 || !rp || r0 < 0 || r1 < r0 || r1 > n || c0 < 0 || c1 < c0 || !b_rp || !b_ci || !b_v)
        return GG_EINVAL;
    try {
        emit(csr_block(wrap(n, rp, ci, v), r0, r1, c0, c1), b_rp, b_ci, b_v);
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_read_mtx(const char *path, int expand_symmetric, int *nrows, int *ncols, int **row_ptr,
                     int **col_idx, double **val)
{
    if (!path || !nrows || !ncols || !row_ptr || !col_idx || !val) return GG_EINVAL;
    try {
        Csr A;
        int nr = 0, nc = 0;
        if (!read_mtx(path, expand_symmetric != 0, nr, nc, A)) return GG_EINVAL;
        *nrows = nr;
        *ncols = nc;
        *row_ptr = (int *)std::malloc(sizeof(int) * (nr + 1));
        std::memcpy(*row_ptr, A.rp.data(), sizeof(int) * (nr + 1));
        const size_t nnz = A.ci.size();
        *col_idx = (int *)std::malloc(sizeof(int) * (nnz ? nnz : 1));
        *val = (double *)std::malloc(sizeof(double) * (nnz ? nnz : 1));
        if (nnz) {
            std::memcpy(*col_idx, A.ci.data(), sizeof(int) * nnz);
            std::memcpy(*val, A.v.data(), sizeof(double) * nnz);
        }
        return GG_OK;
    } catch (...) {
        return GG_EINVAL;
    }
}

void gg_host_free(void *p) { std::free(p); }

}  // extern "C"
