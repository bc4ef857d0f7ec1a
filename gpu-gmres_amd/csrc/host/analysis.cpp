// analysis.cpp -- setup-time analysis for the device triangular solves / SpMV.
//
//  * canonical solve forms: the off-diagonal terms of each row in exactly the
//    summation order the reference uses, plus the divisor, so the device
//    kernels reproduce the reference arithmetic order:
//      LUSolve_ignoreZero           src/SpMV_compute.cpp:92-136
//      MyILUPP::HostPrecond_left    src/preconditioner.cu:1094-1114
//      MyILUPP::HostPrecond_right   src/preconditioner.cu:1117-1137
//  * level sets (replaces cusparse*csrsv_analysis, src/preconditioner.cu:1313-1316)
//  * 2D structured-grid detection for the wavefront solve
//  * CSR-stream row blocks for SpMV
#include <cstdlib>
#include <algorithm>
#include <cmath>

#include "../gg_internal.h"

namespace gg {

namespace {
inline bool near_zero(double a) { return std::fabs(a) < 1e-9; }
void push(Csr &C, int c, double v) { C.ci.push_back(c); C.v.push_back(v); }
CanonTri start(const Csr &T, bool lower)
{
    CanonTri C;
    C.lower = lower;
    C.off.n = T.n;
    C.off.rp.assign(T.n + 1, 0);
    C.off.ci.reserve(T.nnz());
    C.off.v.reserve(T.nnz());
    C.d.assign(T.n, 1.0);
    return C;
}
}  // namespace

CanonTri canon_lower_unit(const Csr &L)
{
    CanonTri C = start(L, true);
    for (int r = 0; r < L.n; r++) {
        for (int k = L.rp[r]; k < L.rp[r + 1]; k++) {
            if (L.ci[k] >= r) break;          // forward loop stops at the diagonal
            push(C.off, L.ci[k], L.v[k]);
        }
        C.off.rp[r + 1] = (int)C.off.ci.size();
    }
    return C;
}

CanonTri canon_upper_ignorezero(const Csr &U)
{
    CanonTri C = start(U, false);
    for (int r = 0; r < U.n; r++) {
        int lb = U.rp[r], j = U.rp[r + 1] - 1;
        for (; j >= lb; j--) {                // backward loop from the row end
            if (U.ci[j] <= r) break;
            push(C.off, U.ci[j], U.v[j]);
        }
        if (j >= lb && U.ci[j] == r && !near_zero(U.v[j])) C.d[r] = U.v[j];
        C.off.rp[r + 1] = (int)C.off.ci.size();
    }
    return C;
}

CanonTri canon_lower_lastdiag(const Csr &L)
{
    CanonTri C = start(L, true);
    for (int r = 0; r < L.n; r++) {
        int lb = L.rp[r], ub = L.rp[r + 1];
        GG_REQUIRE(ub > lb, GG_EINVAL, "split L: empty row " + std::to_string(r));
        for (int k = lb; k < ub - 1; k++) push(C.off, L.ci[k], L.v[k]);
        C.d[r] = L.v[ub - 1];
        C.off.rp[r + 1] = (int)C.off.ci.size();
    }
    return C;
}

CanonTri canon_upper_firstdiag(const Csr &U)
{
    CanonTri C = start(U, false);
    for (int r = 0; r < U.n; r++) {
        int lb = U.rp[r], ub = U.rp[r + 1];
        GG_REQUIRE(ub > lb, GG_EINVAL, "split U: empty row " + std::to_string(r));
        for (int k = lb + 1; k < ub; k++) push(C.off, U.ci[k], U.v[k]);
        C.d[r] = U.v[lb];
        C.off.rp[r + 1] = (int)C.off.ci.size();
    }
    return C;
}

Levels level_sets(const CanonTri &T, bool ext_cols)
{
    const int n = T.off.n;
    std::vector<int> lev(n, 0);
    int maxlev = 0;
    auto row = [&](int r) {
        int l = 0;
        for (int k = T.off.rp[r]; k < T.off.rp[r + 1]; k++) {
            int c = T.off.ci[k];
            GG_REQUIRE(T.lower ? c < r : c > r, GG_EINVAL,
                       std::string(T.lower ? "lower" : "upper") + " factor has an entry on the wrong side of the diagonal at row " +
                           std::to_string(r));
            if (ext_cols && c >= n) continue;
            l = std::max(l, lev[c] + 1);
        }
        lev[r] = l;
        maxlev = std::max(maxlev, l);
    };
    if (T.lower) for (int r = 0; r < n; r++) row(r);
    else for (int r = n - 1; r >= 0; r--) row(r);
    Levels L;
    L.ptr.assign(maxlev + 2, 0);
    for (int r = 0; r < n; r++) L.ptr[lev[r] + 1]++;
    for (int l = 0; l <= maxlev; l++) L.ptr[l + 1] += L.ptr[l];
    L.rows.resize(n);
    std::vector<int> pos(L.ptr.begin(), L.ptr.end() - 1);
    for (int r = 0; r < n; r++) L.rows[pos[lev[r]]++] = r;
    if (n == 0) L.ptr.assign(1, 0);
    return L;
}

Wave2D detect_wave2d(const CanonTri &L, const CanonTri &U, bool split_u)
{
    Wave2D w;
    const int n = L.off.n;
    if (n < 128 || U.off.n != n) return w;
    int nx = 0;
    for (int r = 0; r < n; r++)
        for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) nx = std::max(nx, r - L.off.ci[k]);
    if (nx < 2 || n % nx != 0 || n / nx < 2) return w;
    // the fill depth K: the smallest offset above 1 is nx - K
    int K = 0;
    for (int r = 0; r < n; r++)
        for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) {
            const int o = r - L.off.ci[k];
            if (o > 1) K = std::max(K, nx - o);
        }
    if (K > 2 || nx < K + 3 || (split_u && K > 0)) return w;
    // L rows: [r-nx][r-nx+1]..[r-nx+K][r-1] in this order (each may be absent),
    // no wrap: (j-1, i+a) needs i + a < nx, (j, i-1) needs i > 0
    for (int r = 0; r < n; r++) {
        int lb = L.off.rp[r], ub = L.off.rp[r + 1], k = lb;
        for (int a = 0; a <= K; a++)
            if (k < ub && L.off.ci[k] == r - nx + a && (r % nx) + a < nx) k++;
        if (k < ub && L.off.ci[k] == r - 1 && (r % nx) != 0) k++;
        if (k != ub) return w;
    }
    // U rows (LUSolve_ignoreZero walks from the row end): [r+nx][r+nx-1]..[r+nx-K][r+1];
    // split_u: [r+1][r+nx] (ascending, diag-first split U)
    for (int r = 0; split_u && r < n; r++) {
        int lb = U.off.rp[r], ub = U.off.rp[r + 1], k = lb;
        if (k < ub && U.off.ci[k] == r + 1 && (r % nx) != nx - 1) k++;
        if (k < ub && U.off.ci[k] == r + nx) k++;
        if (k != ub) return w;
    }
    for (int r = 0; !split_u && r < n; r++) {
        int lb = U.off.rp[r], ub = U.off.rp[r + 1], k = lb;
        for (int a = 0; a <= K; a++)
            if (k < ub && U.off.ci[k] == r + nx - a && (r % nx) - a >= 0) k++;
        if (k < ub && U.off.ci[k] == r + 1 && (r % nx) != nx - 1) k++;
        if (k != ub) return w;
    }
    w.ok = true;
    w.nx = nx;
    w.ny = n / nx;
    w.skew = K + 1;
    w.u_inline_first = split_u;
    w.nbands = (w.ny + 63) / 64;
    // the lane skew, plus skew-1 lead-in and run-out steps (Wave2D::slot)
    w.T = (nx + 63 * w.skew + 2 * (w.skew - 1) + kWaveTAlign - 1) / kWaveTAlign * kWaveTAlign;
    w.P2 = (long long)w.nbands * w.T * 64;
    w.P = w.P2;
    return w;
}

Wave2D detect_border2d(const CanonTri &L, const CanonTri &U, bool split_u, CanonTri &gl, CanonTri &gu)
{
    Wave2D w;
    const int n = L.off.n;
    if (n < 256 || U.off.n != n) return w;
    // the line length: the most frequent L offset above 1
    std::vector<int> cnt;
    for (int r = 0; r < n; r++)
        for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) {
            const int o = r - L.off.ci[k];
            if (o > 1 && o <= 65536) {
                if ((int)cnt.size() <= o) cnt.resize(o + 1, 0);
                cnt[o]++;
            }
        }
    int nx = 0;
    for (int o = 2; o < (int)cnt.size(); o++)
        if (cnt[o] > (nx ? cnt[nx] : 0)) nx = o;
    if (nx < 3 || cnt[nx] < n / 4) return w;
    // the tail: every row with a U term off the grid pattern, and every row
    // with an off-pattern L term into the grid block, lies in it (a fixed point:
    // the tail grows until the grid rows' odd L terms all point into it)
    int nt = 0;
    for (int r = 0; r < n; r++)
        for (int k = U.off.rp[r]; k < U.off.rp[r + 1]; k++) {
            const int o = U.off.ci[k] - r;
            if (o != 1 && o != nx) nt = std::max(nt, r + 1);
        }
    for (bool grew = true; grew;) {
        grew = false;
        for (int r = nt; r < n; r++)
            for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) {
                const int c = L.off.ci[k], o = r - c;
                if (o != 1 && o != nx && c >= nt) {
                    nt = r + 1;
                    grew = true;
                    break;
                }
            }
    }
    const int ng = n - nt;
    if (nt == 0 || nt > n / 8 || ng % nx != 0 || ng / nx < 2) return w;
    // the grid block; the tail terms of its L rows must lead the row
    auto block = [&](const CanonTri &T, CanonTri &B) -> bool {
        B = CanonTri{};
        B.lower = T.lower;
        B.off.n = ng;
        B.off.rp.assign(ng + 1, 0);
        B.d.assign(T.d.begin() + nt, T.d.end());
        for (int r = nt; r < n; r++) {
            bool grid = false;
            for (int k = T.off.rp[r]; k < T.off.rp[r + 1]; k++) {
                const int c = T.off.ci[k];
                if (c < nt) {
                    if (grid) return false;
                    continue;
                }
                grid = true;
                B.off.ci.push_back(c - nt);
                B.off.v.push_back(T.off.v[k]);
            }
            B.off.rp[r - nt + 1] = (int)B.off.ci.size();
        }
        return true;
    };
    if (!block(L, gl) || !block(U, gu)) return w;
    w = detect_wave2d(gl, gu, split_u);
    if (!w.ok || w.skew != 1) return Wave2D{};
    w.bnt = nt;
    w.bofs = (nt + 63LL) / 64 * 64;      // the grid's arrays stay 512-B aligned
    w.P = w.bofs + w.P2;
    return w;
}

Wave2D detect_wave3d(const CanonTri &L, const CanonTri &U)
{
    Wave2D w;
    const int n = L.off.n;
    if (n < 128 || U.off.n != n) return w;
    long long nxy = 0;
    for (int r = 0; r < n; r++)
        for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) nxy = std::max<long long>(nxy, r - L.off.ci[k]);
    long long nx = 0;
    for (int r = 0; r < n; r++)
        for (int k = L.off.rp[r]; k < L.off.rp[r + 1]; k++) {
            const long long o = r - L.off.ci[k];
            if (o < nxy) nx = std::max(nx, o);
        }
    if (nx < 2 || nxy <= nx || nxy % nx != 0 || nxy / nx < 2 || n % nxy != 0 || n / nxy < 2) return w;
    // L rows: [r-nxy][r-nx][r-1] in this order (each may be absent), no wrap
    for (int r = 0; r < n; r++) {
        int k = L.off.rp[r];
        const int ub = L.off.rp[r + 1];
        if (k < ub && L.off.ci[k] == r - nxy) k++;
        if (k < ub && L.off.ci[k] == r - nx && (r % nxy) >= nx) k++;
        if (k < ub && L.off.ci[k] == r - 1 && (r % nx) != 0) k++;
        if (k != ub) return w;
    }
    // U rows (LUSolve_ignoreZero walks from the row end): [r+nxy][r+nx][r+1]
    for (int r = 0; r < n; r++) {
        int k = U.off.rp[r];
        const int ub = U.off.rp[r + 1];
        if (k < ub && U.off.ci[k] == r + nxy) k++;
        if (k < ub && U.off.ci[k] == r + nx && (r % nxy) + nx < nxy) k++;
        if (k < ub && U.off.ci[k] == r + 1 && (r % nx) != nx - 1) k++;
        if (k != ub) return w;
    }
    w.ok = true;
    w.nx = (int)nx;
    w.ny = (int)(nxy / nx);
    w.nz = (int)(n / nxy);
    const char *pl = std::getenv("GG_WAVE3D_PLANES");     // the (plane, band) pipeline instead
    if (!(pl && pl[0] == '1')) {
        // 8-line x 8-plane tiles (Wave2D::slot); the lane skew is a + c <= 14 steps
        w.tile = true;
        w.NJ = (w.ny + 7) / 8;
        w.NK = (w.nz + 7) / 8;
        w.nbands = w.NJ * w.NK;
        w.T = (w.nx + 14 + kTileTAlign - 1) / kTileTAlign * kTileTAlign;
        w.P2 = (long long)w.nbands * w.T * 64;
        w.P = w.P2;
        return w;
    }
    w.nbands = (w.ny + 63) / 64;
    w.T = (w.nx + 63 + kWaveTAlign - 1) / kWaveTAlign * kWaveTAlign;
    w.P2 = (long long)w.nbands * w.T * 64;
    w.P = w.P2 * w.nz;
    return w;
}

std::vector<int> spmv_blocks(const Csr &A, std::vector<int> &long_rows)
{
    std::vector<int> b;
    b.push_back(0);
    long_rows.clear();
    int r = 0;
    const int n = A.n;
    while (r < n) {
        int len = A.rp[r + 1] - A.rp[r];
        if (len > kSpmvCap) {           // a row alone, handled by the long-row path
            long_rows.push_back(r);
            r++;
            b.push_back(r);
            continue;
        }
        int start = r, nnz = 0;
        while (r < n && r - start < 256) {
            int l = A.rp[r + 1] - A.rp[r];
            if (l > kSpmvCap || nnz + l > kSpmvCap) break;
            nnz += l;
            r++;
        }
        b.push_back(r);
    }
    return b;
}


Wave2D select_split_layout(const CanonTri &L, const CanonTri &U, CanonTri &gl, CanonTri &gu)
{
    Wave2D w;
    const char *env = std::getenv("GG_NO_WAVEFRONT");
    if (env && env[0] == '1') return w;
    w = detect_wave2d(L, U, true);
    if (!w.ok) {
        const char *nb = std::getenv("GG_NO_BORDER");
        if (!(nb && nb[0] == '1')) w = detect_border2d(L, U, true, gl, gu);
    }
    if (w.ok && w.nbands > 512) w.ok = false;
    return w;
}


std::vector<int> rcm_order(const CanonTri &L, const CanonTri &U)
{
    const int n = L.off.n;
    // symmetric adjacency of L + U (off-diagonal terms only)
    std::vector<int> deg(n, 0);
    auto each = [&](auto &&f) {
        for (const CanonTri *T : {&L, &U})
            for (int r = 0; r < n; r++)
                for (int k = T->off.rp[r]; k < T->off.rp[r + 1]; k++) {
                    const int c = T->off.ci[k];
                    if (c >= 0 && c < n && c != r) f(r, c);
                }
    };
    each([&](int r, int c) {
        deg[r]++;
        deg[c]++;
    });
    std::vector<long long> ap(n + 1, 0);
    for (int r = 0; r < n; r++) ap[r + 1] = ap[r] + deg[r];
    std::vector<int> adj(ap[n]);
    std::vector<long long> fill(ap.begin(), ap.end() - 1);
    each([&](int r, int c) {
        adj[fill[r]++] = c;
        adj[fill[c]++] = r;
    });
    // neighbours sorted by (degree, index), duplicates dropped
    std::vector<int> ndeg(n);
    for (int r = 0; r < n; r++) {
        auto b = adj.begin() + ap[r], e = adj.begin() + ap[r + 1];
        std::sort(b, e);
        e = std::unique(b, e);
        ndeg[r] = (int)(e - b);
        std::sort(b, e, [&](int a, int c) { return deg[a] != deg[c] ? deg[a] < deg[c] : a < c; });
    }
    std::vector<int> order;
    order.reserve(n);
    std::vector<char> seen(n, 0);
    std::vector<int> lvl(n, -1);
    auto bfs = [&](int root, std::vector<int> &out) {     // one component from root
        size_t h = out.size();
        out.push_back(root);
        seen[root] = 1;
        while (h < out.size()) {
            const int r = out[h++];
            for (long long k = ap[r]; k < ap[r] + ndeg[r]; k++) {
                const int c = adj[k];
                if (!seen[c]) {
                    seen[c] = 1;
                    out.push_back(c);
                }
            }
        }
    };
    // components in order of their lowest-(degree, index) node
    std::vector<int> byd(n);
    for (int r = 0; r < n; r++) byd[r] = r;
    std::sort(byd.begin(), byd.end(), [&](int a, int c) { return ndeg[a] != ndeg[c] ? ndeg[a] < ndeg[c] : a < c; });
    std::vector<int> comp;
    for (int start : byd) {
        if (seen[start]) continue;
        // pseudo-peripheral root: two BFS sweeps, the last node of the first
        // (lowest degree in its last level) starts the second
        comp.clear();
        bfs(start, comp);
        int root = comp.back();
        for (int c : comp) seen[c] = 0;
        comp.clear();
        bfs(root, comp);
        order.insert(order.end(), comp.begin(), comp.end());
    }
    std::reverse(order.begin(), order.end());
    return order;
}

void relabel_tri(const CanonTri &C, const std::vector<long long> &nat2lay, CanonTri &out, Levels &lv)
{
    const int n = C.off.n;
    std::vector<int> l2n(n, -1);
    for (int r = 0; r < n; r++) l2n[nat2lay[r]] = r;
    out.lower = C.lower;
    out.off.n = n;
    out.off.rp.assign(n + 1, 0);
    out.d.assign(n, 1.0);
    for (int p = 0; p < n; p++) {
        const int r = l2n[p];
        out.off.rp[p + 1] = out.off.rp[p] + (C.off.rp[r + 1] - C.off.rp[r]);
        out.d[p] = C.d[r];
    }
    out.off.ci.resize(C.off.ci.size());
    out.off.v.resize(C.off.v.size());
    for (int p = 0; p < n; p++) {
        const int r = l2n[p];
        int o = out.off.rp[p];
        for (int k = C.off.rp[r]; k < C.off.rp[r + 1]; k++, o++) {
            out.off.ci[o] = (int)nat2lay[C.off.ci[k]];
            out.off.v[o] = C.off.v[k];
        }
    }
    const Levels nl = level_sets(C);
    lv.ptr = nl.ptr;
    lv.rows.resize(n);
    for (size_t l = 0; l + 1 < nl.ptr.size(); l++) {
        for (int q = nl.ptr[l]; q < nl.ptr[l + 1]; q++) lv.rows[q] = (int)nat2lay[nl.rows[q]];
        std::sort(lv.rows.begin() + nl.ptr[l], lv.rows.begin() + nl.ptr[l + 1]);
    }
}

}  // namespace gg
