// host_abi.cpp -- include/ggmres_host.h: setup-phase entry points (no device).
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>

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

int gg_host_iluk_pattern(int level, int n, const int *rp, const int *ci, int threads, int *prow, int **pcol)
{
    if (n < 0 || level < 0 || !rp || !prow || !pcol) return GG_EINVAL;
    try {
        std::vector<double> v((size_t)rp[n], 0.0);
        const Csr A = wrap(n, rp, ci, v.data());
        std::vector<long long> pr;
        std::vector<int> nl, pc;
        iluk_pattern(A, level, std::max(1, threads), pr, nl, pc);
        GG_REQUIRE(pr[n] < (1LL << 31), GG_EINVAL, "pattern above 2^31 entries");
        for (int r = 0; r <= n; r++) prow[r] = (int)pr[r];
        *pcol = static_cast<int *>(std::malloc(sizeof(int) * std::max<size_t>(pc.size(), 1)));
        if (!*pcol) return GG_ENOMEM;
        std::copy(pc.begin(), pc.end(), *pcol);
        return GG_OK;
    } catch (const Error &e) {
        return e.code;
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

int gg_host_split_layout(int n, const int *l_rp, const int *l_ci, const double *l_v, const int *u_rp,
                         const int *u_ci, const double *u_v, long long *slot, int *info)
{
    if (n < 0 || !info) return GG_EINVAL;
    try {
        const CanonTri cl = canon_lower_lastdiag(wrap(n, l_rp, l_ci, l_v));
        const CanonTri cu = canon_upper_firstdiag(wrap(n, u_rp, u_ci, u_v));
        // the solver's choice (solver.hip gg_set_precond_split), environment
        // overrides included
        CanonTri gl, gu;
        const Wave2D w = select_split_layout(cl, cu, gl, gu);
        for (int k = 0; k < 9; k++) info[k] = 0;
        if (!w.ok) {
            // the flow path: an RCM layout (GG_FLOW_RCM=0: natural, as the solver)
            const char *fr = std::getenv("GG_FLOW_RCM");
            if (fr && fr[0] == '0') return 0;
            const std::vector<int> order = rcm_order(cl, cu);
            info[0] = 6;
            if (slot)
                for (int k = 0; k < n; k++) slot[order[k]] = k;
            return 1;
        }
        info[0] = w.bnt ? 5 : 2;
        info[1] = w.nx;
        info[2] = w.ny;
        info[3] = w.nz;
        info[4] = w.nbands;
        info[5] = w.T;
        info[6] = w.bnt;
        info[7] = (int)w.bofs;
        info[8] = w.skew;
        if (slot)
            for (int r = 0; r < n; r++) slot[r] = w.slot(r);
        return 1;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_wave_layout(int n, const int *l_rp, const int *l_ci, const double *l_v, const int *u_rp,
                        const int *u_ci, const double *u_v, long long *slot, int *info)
{
    if (n < 0 || !info) return GG_EINVAL;
    try {
        const CanonTri cl = canon_lower_unit(wrap(n, l_rp, l_ci, l_v));
        const CanonTri cu = canon_upper_ignorezero(wrap(n, u_rp, u_ci, u_v));
        // the solver's choice (solver.hip setup_left): 2D band layout, else 3D
        Wave2D w = detect_wave2d(cl, cu);
        if (w.ok && w.nbands > 512) w.ok = false;
        if (!w.ok) w = detect_wave3d(cl, cu);
        for (int k = 0; k < 9; k++) info[k] = 0;
        if (!w.ok) return 0;
        info[0] = w.tile ? 3 : (w.nz > 1 ? 4 : 2);
        info[1] = w.nx;
        info[2] = w.ny;
        info[3] = w.nz;
        info[4] = w.nbands;
        info[5] = w.T;
        info[6] = w.NJ;
        info[7] = w.NK;
        info[8] = w.skew;
        if (slot)
            for (int r = 0; r < n; r++) slot[r] = w.slot(r);
        return 1;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_partition(int n, const int *rp, const int *ci, int nparts, int method, int *node_part,
                      int *part_size, int *pinv, int *q)
{
    if (n < 1 || !rp || !ci || nparts < 1 || nparts > n || !node_part || !part_size || !pinv || !q ||
        (method & ~(GG_PART_COLOR_SEP | 3)) != 0 || (method & 3) == 3)
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

struct gg_dd_plan {
    DDPlan plan;
    std::map<int, std::unique_ptr<DDShardHost>> shards;
    DDShardHost &shard(int p)
    {
        auto it = shards.find(p);
        if (it == shards.end()) it = shards.emplace(p, std::make_unique<DDShardHost>(dd_shard(plan, p))).first;
        return *it->second;
    }
};

extern "C" {

int gg_host_dd_plan(int n, const int *rp, const int *ci, const double *v, int nparts, int method,
                    gg_dd_plan **out)
{
    if (n < 1 || !rp || !ci || !v || !out) return GG_EINVAL;
    try {
        auto pl = std::make_unique<gg_dd_plan>();
        pl->plan = dd_plan(wrap(n, rp, ci, v), nparts, method);
        *out = pl.release();
        return GG_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    } catch (...) {
        return GG_EINVAL;
    }
}

int gg_host_dd_plan_sizes(const gg_dd_plan *pl, int *sizes)
{
    if (!pl || !sizes) return GG_EINVAL;
    sizes[0] = pl->plan.n;
    sizes[1] = pl->plan.P;
    sizes[2] = pl->plan.part_size[pl->plan.P];
    sizes[3] = pl->plan.maxI;
    return GG_OK;
}

int gg_host_dd_plan_perm(const gg_dd_plan *pl, int *part_size, int *pinv, int *q)
{
    if (!pl) return GG_EINVAL;
    const DDPlan &D = pl->plan;
    if (part_size) std::memcpy(part_size, D.part_size.data(), sizeof(int) * (D.P + 1));
    if (pinv) std::memcpy(pinv, D.pinv.data(), sizeof(int) * D.n);
    if (q) std::memcpy(q, D.q.data(), sizeof(int) * D.n);
    return GG_OK;
}

int gg_host_dd_shard_sizes(gg_dd_plan *pl, int part, int *sizes)
{
    if (!pl || !sizes || part < 0 || part >= pl->plan.P) return GG_EINVAL;
    try {
        DDShardHost &S = pl->shard(part);
        sizes[0] = S.nI;
        sizes[1] = S.nS;
        sizes[2] = (int)S.iface.size();
        return GG_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int gg_host_dd_shard_csr(gg_dd_plan *pl, int part, int piece, int *nrows, int **rp, int **ci,
                         double **v)
{
    if (!pl || !nrows || !rp || !ci || !v || part < 0 || part >= pl->plan.P) return GG_EINVAL;
    try {
        DDShardHost &S = pl->shard(part);
        const Csr *C = nullptr;
        switch (piece) {
        case GG_DD_A: C = &S.A; break;
        case GG_DD_LI: C = &S.LI.off; break;
        case GG_DD_LS: C = &S.LS.off; break;
        case GG_DD_LSH: C = &S.LSH; break;
        case GG_DD_UI: C = &S.UI.off; break;
        case GG_DD_US: C = &S.US.off; break;
        case GG_DD_UIS: C = &S.UIS; break;
        default: return GG_EINVAL;
        }
        *nrows = C->n;
        *rp = (int *)std::malloc(sizeof(int) * (C->n + 1));
        emit(*C, *rp, ci, v);
        return GG_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int gg_host_dd_shard_div(gg_dd_plan *pl, int part, int piece, double *d)
{
    if (!pl || !d || part < 0 || part >= pl->plan.P) return GG_EINVAL;
    DDShardHost &S = pl->shard(part);
    const CanonTri *T = piece == GG_DD_LI ? &S.LI : piece == GG_DD_LS ? &S.LS
                      : piece == GG_DD_UI ? &S.UI : piece == GG_DD_US ? &S.US : nullptr;
    if (!T) return GG_EINVAL;
    if (!T->d.empty()) std::memcpy(d, T->d.data(), sizeof(double) * T->d.size());
    return GG_OK;
}

int gg_host_dd_shard_index(gg_dd_plan *pl, int part, int *iface, int *rows)
{
    if (!pl || part < 0 || part >= pl->plan.P) return GG_EINVAL;
    DDShardHost &S = pl->shard(part);
    if (iface && !S.iface.empty()) std::memcpy(iface, S.iface.data(), sizeof(int) * S.iface.size());
    if (rows && !S.rows.empty()) std::memcpy(rows, S.rows.data(), sizeof(int) * S.rows.size());
    return GG_OK;
}

void gg_host_dd_plan_free(gg_dd_plan *pl) { delete pl; }

}  // extern "C"
