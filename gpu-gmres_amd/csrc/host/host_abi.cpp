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

void gg_host_free(void *p) { std::free(p); }

}  // extern "C"
