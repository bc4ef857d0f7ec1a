// factor.cpp -- host-side ILU(0) / ILU(k) setup for the MI355X solver.
//
// Setup phase only (factored once, reused for every solve / time step,
// SURVEY.md 2.2).  Arithmetic follows the reference entry-for-entry in fp64:
//   ilu0_left   leftILU                 src/leftILU.cu:27-336 (column kernel of
//                                       cpuSequentialTriSolve :769-825, level
//                                       order generateLevel :339-368, split
//                                       splitLU_csr :481-541)
//   iluk_itsol  lofC + ilukC            src/iluk.cpp:56-334
#include <algorithm>
#include <memory>
#include <atomic>
#include <cmath>
#include <numeric>
#include <thread>

#include "../gg_internal.h"

namespace gg {

namespace {

inline bool near_zero(double a) { return std::fabs(a) < 1e-9; }  // Equal(a,0), src/defs.h:45-47

// transpose a square CSR (row order inside each output row ascending)
void transpose(int n, const std::vector<int> &rp, const std::vector<int> &ci,
               const std::vector<double> &v, std::vector<int> &tp, std::vector<int> &ti,
               std::vector<double> &tv)
{
    const int nnz = rp[n];
    tp.assign(n + 1, 0);
    ti.resize(nnz);
    tv.resize(nnz);
    for (int k = 0; k < nnz; k++) tp[ci[k] + 1]++;
    for (int c = 0; c < n; c++) tp[c + 1] += tp[c];
    std::vector<int> pos(tp.begin(), tp.end() - 1);
    for (int r = 0; r < n; r++)
        for (int k = rp[r]; k < rp[r + 1]; k++) {
            int p = pos[ci[k]]++;
            ti[p] = r;
            tv[p] = v[k];
        }
}

}  // namespace

void ilu0_left(const Csr &A, Csr &L, Csr &U)
{
    const int n = A.n;
    // dependency levels on the original values (generateLevel)
    std::vector<int> level(n, 0);
    for (int r = 0; r < n; r++)
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
            int c = A.ci[k];
            if (c > r && !near_zero(A.v[k]) && level[c] < level[r] + 1) level[c] = level[r] + 1;
        }
    std::vector<int> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return level[a] < level[b]; });

    // CSC image of A (rows ascending per column)
    std::vector<int> cp, ri;
    std::vector<double> cv;
    transpose(n, A.rp, A.ci, A.v, cp, ri, cv);

    // left-looking column elimination, merge-based L lookup
    for (int tgt : order) {
        const int lb = cp[tgt], ub = cp[tgt + 1];
        double u_diag = 0.0;
        for (int k = lb; k < ub - 1; k++) {
            const int cr = ri[k];
            if (cr > tgt) break;
            if (cr == tgt) { u_diag = cv[k]; break; }
            // column cr: entries with row > cr are its (final) L part
            int q = cp[cr];
            const int qe = cp[cr + 1];
            const double ukt = cv[k];
            for (int p = k + 1; p < ub; p++) {
                const int r2 = ri[p];
                while (q < qe && ri[q] < r2) q++;
                if (q == qe) break;
                if (ri[q] == r2) cv[p] -= cv[q] * ukt;
            }
        }
        for (int k = lb; k < ub; k++) {
            if (ri[k] <= tgt) continue;
            cv[k] = near_zero(u_diag) ? 0.0 : cv[k] / u_diag;
        }
    }

    // back to CSR, split with the 1e-9 drop, unit diagonal appended LAST in L
    Csr F;
    F.n = n;
    transpose(n, cp, ri, cv, F.rp, F.ci, F.v);
    split_lu_drop(F, L, U);
}

void split_lu_drop(const Csr &F, Csr &L, Csr &U)
{
    const int n = F.n;
    L.n = U.n = n;
    L.rp.assign(n + 1, 0);
    U.rp.assign(n + 1, 0);
    L.ci.clear(); L.v.clear(); U.ci.clear(); U.v.clear();
    L.ci.reserve(F.rp[n] / 2 + n); L.v.reserve(F.rp[n] / 2 + n);
    U.ci.reserve(F.rp[n] / 2 + n); U.v.reserve(F.rp[n] / 2 + n);
    for (int r = 0; r < n; r++) {
        for (int k = F.rp[r]; k < F.rp[r + 1]; k++) {
            if (near_zero(F.v[k])) continue;
            if (F.ci[k] < r) { L.ci.push_back(F.ci[k]); L.v.push_back(F.v[k]); }
            else { U.ci.push_back(F.ci[k]); U.v.push_back(F.v[k]); }
        }
        L.ci.push_back(r);
        L.v.push_back(1.0);
        L.rp[r + 1] = (int)L.ci.size();
        U.rp[r + 1] = (int)U.ci.size();
    }
}

void csc_pattern(const Csr &A, std::vector<int> &cp, std::vector<int> &ri,
                 std::vector<long long> &csc2csr, std::vector<long long> &csr2csc)
{
    const int n = A.n, nnz = A.rp[n];
    cp.assign(n + 1, 0);
    ri.resize(nnz);
    csc2csr.resize(nnz);
    csr2csc.resize(nnz);
    for (int k = 0; k < nnz; k++) cp[A.ci[k] + 1]++;
    for (int c = 0; c < n; c++) cp[c + 1] += cp[c];
    std::vector<int> pos(cp.begin(), cp.end() - 1);
    for (int r = 0; r < n; r++)
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
            const int p = pos[A.ci[k]]++;
            ri[p] = r;
            csc2csr[p] = k;
            csr2csc[k] = p;
        }
}

void iluk_symbolic(const Csr &A, int lof, std::vector<std::vector<int>> &Lja,
                   std::vector<std::vector<int>> &Uja)
{
    const int n = A.n;
    // ---- symbolic (lofC): per row, L part in leftmost-pivot order, U part in
    //      insertion order, with levels of fill
    Lja.assign(n, {});
    Uja.assign(n, {});
    std::vector<std::vector<int>> ulvl(n);
    std::vector<int> jbuf(n + 1), levls(n + 1), iw(n, -1);
    for (int i = 0; i < n; i++) {
        int incl = 0, incu = i;
        for (int k = A.rp[i]; k < A.rp[i + 1]; k++) {
            int col = A.ci[k];
            if (col < i) { jbuf[incl] = col; levls[incl] = 0; iw[col] = incl++; }
            else if (col > i) { jbuf[incu] = col; levls[incu] = 0; iw[col] = incu++; }
        }
        int jpiv = -1;
        while (++jpiv < incl) {
            int k = jbuf[jpiv], kmin = k, jmin = jpiv;
            for (int j = jpiv + 1; j < incl; j++)
                if (jbuf[j] < kmin) { kmin = jbuf[j]; jmin = j; }
            if (jmin != jpiv) {
                jbuf[jpiv] = kmin; jbuf[jmin] = k;
                iw[kmin] = jpiv; iw[k] = jmin;
                std::swap(levls[jpiv], levls[jmin]);
                k = kmin;
            }
            const std::vector<int> &uk = Uja[k];
            const std::vector<int> &lk = ulvl[k];
            for (size_t j = 0; j < uk.size(); j++) {
                int col = uk[j];
                int it = lk[j] + levls[jpiv] + 1;
                if (it > lof) continue;
                int ip = iw[col];
                if (ip == -1) {
                    if (col < i) { jbuf[incl] = col; levls[incl] = it; iw[col] = incl++; }
                    else if (col > i) { jbuf[incu] = col; levls[incu] = it; iw[col] = incu++; }
                } else if (it < levls[ip]) {
                    levls[ip] = it;
                }
            }
        }
        for (int j = 0; j < incl; j++) iw[jbuf[j]] = -1;
        for (int j = i; j < incu; j++) iw[jbuf[j]] = -1;
        Lja[i].assign(jbuf.begin(), jbuf.begin() + incl);
        Uja[i].assign(jbuf.begin() + i, jbuf.begin() + incu);
        ulvl[i].assign(levls.begin() + i, levls.begin() + incu);
    }
}

// Row i of the ILU(k) pattern for k >= 2 without any other row's result, by
// incomplete fill paths (Hysom & Pothen, "Level-based incomplete LU
// factorization: graph model and algorithms", the incomplete fill-path
// theorem): entry (i, j) has level L - 1 exactly when the shortest path
// i -> ... -> j in G(A) whose interior vertices are all below min(i, j) has L
// edges -- lofC's sum rule lev(i,j) = min_k lev(i,k) + lev(k,j) + 1 unrolled.
// Per row a layered min-max search: M_L(x) = the smallest largest interior
// vertex over walks of exactly L edges from i to x with every interior vertex
// below i (M_1 = -1 on row i of A), M_{L+1}(y) = min over edges x -> y, x < i,
// of max(M_L(x), x); j > i joins at the first L where M_L(j) exists, j < i at
// the first L with M_L(j) < j (a walk shortens to a path with no larger
// interior, so walks never report a level below the true one).  Rows are
// independent: built over host threads like k = 1.
struct FillPathScratch {
    std::vector<int> mcur, mnext, lev;          // per vertex; kUnset outside the row's search
    std::vector<int> fcur, fnext, touched;
    static constexpr int kUnset = 0x7fffffff;
    explicit FillPathScratch(int n) : mcur(n, kUnset), mnext(n, kUnset), lev(n, kUnset) {}
};
static void fillpath_row(const Csr &A, int lof, int i, FillPathScratch &w, std::vector<int> &row)
{
    constexpr int U = FillPathScratch::kUnset;
    w.fcur.clear();
    w.touched.clear();
    for (int e = A.rp[i]; e < A.rp[i + 1]; e++) {
        const int x = A.ci[e];
        if (x == i || w.mcur[x] != U) continue;
        w.mcur[x] = -1;                             // an original entry: level 0
        w.fcur.push_back(x);
        if (w.lev[x] == U) {
            w.lev[x] = 0;
            w.touched.push_back(x);
        }
    }
    for (int L = 1; L <= lof && !w.fcur.empty(); L++) {
        w.fnext.clear();
        for (int x : w.fcur) {
            if (x >= i) continue;                   // only vertices below i are interior
            const int m = std::max(w.mcur[x], x);
            for (int e = A.rp[x]; e < A.rp[x + 1]; e++) {
                const int y = A.ci[e];
                if (y == i || m >= w.mnext[y]) continue;
                if (w.mnext[y] == U) w.fnext.push_back(y);
                w.mnext[y] = m;
            }
        }
        for (int x : w.fcur) w.mcur[x] = U;
        for (int y : w.fnext) {
            if (w.lev[y] == U && (y > i || w.mnext[y] < y)) {
                w.lev[y] = L;
                w.touched.push_back(y);
            }
            w.mcur[y] = w.mnext[y];
            w.mnext[y] = U;
        }
        w.fcur.swap(w.fnext);
    }
    for (int x : w.fcur) w.mcur[x] = U;
    row.clear();
    row.push_back(i);
    for (int x : w.touched) {
        row.push_back(x);                           // every recorded level is <= lof
        w.lev[x] = U;
    }
    std::sort(row.begin(), row.end());
}

// The ILU(k) pattern as flat rows (each row ascending: L part, the diagonal,
// U part) -- the order-free content of lofC's output (src/iluk.cpp:193-334:
// its L part is built in leftmost-pivot = ascending order, its U part is
// sorted by the emission; ilukC's arithmetic per entry only depends on the
// ascending pivot order, not on where an entry is stored).
//   k = 1: a fill entry has level 1 exactly when it comes from an ORIGINAL L
//     entry (i, k) of row i and an ORIGINAL U entry (k, c) of row k (every other
//     path has level >= 2), so row i's pattern is A(i) united with U_A(k) over
//     k in L_A(i): independent of every other row's fill, built row-parallel
//     over `threads` host threads (dynamic blocks of 1024 rows);
//   k >= 2: the incomplete fill paths of each row (fillpath_row), row-parallel
//     the same way (GG_ILUK_SERIAL=1: lofC itself, serial, flattened).
void iluk_pattern(const Csr &A, int lof, int threads, std::vector<long long> &prow, std::vector<int> &nl,
                  std::vector<int> &pcol)
{
    const int n = A.n;
    prow.assign((size_t)n + 1, 0);
    nl.assign(n, 0);
    const char *ser = std::getenv("GG_ILUK_SERIAL");
    if (lof == 0 || (lof >= 2 && ser && ser[0] == '1')) {
        std::vector<std::vector<int>> Lja, Uja;
        iluk_symbolic(A, lof, Lja, Uja);
        for (int i = 0; i < n; i++) {
            nl[i] = (int)Lja[i].size();
            prow[i + 1] = prow[i] + nl[i] + 1 + (long long)Uja[i].size();
        }
        pcol.resize((size_t)prow[n]);
        for (int i = 0; i < n; i++) {
            int *o = pcol.data() + prow[i];
            std::copy(Lja[i].begin(), Lja[i].end(), o);        // ascending (leftmost pivot first)
            o[nl[i]] = i;
            std::vector<int> u = Uja[i];
            std::sort(u.begin(), u.end());
            std::copy(u.begin(), u.end(), o + nl[i] + 1);
        }
        return;
    }
    constexpr int kRows = 1024;
    const int nblk = (n + kRows - 1) / kRows;
    std::vector<std::vector<int>> bcols(nblk), blen(nblk);
    std::atomic<int> next{0};
    auto work = [&]() {
        std::vector<int> mark(n, -1), row;
        std::unique_ptr<FillPathScratch> fp(lof >= 2 ? new FillPathScratch(n) : nullptr);
        for (int b; (b = next.fetch_add(1)) < nblk;) {
            const int r0 = b * kRows, r1 = std::min(n, r0 + kRows);
            std::vector<int> &cols = bcols[b], &len = blen[b];
            len.resize(r1 - r0);
            for (int i = r0; i < r1; i++) {
                if (fp) {
                    fillpath_row(A, lof, i, *fp, row);
                    len[i - r0] = (int)row.size();
                    cols.insert(cols.end(), row.begin(), row.end());
                    continue;
                }
                row.clear();
                mark[i] = i;
                row.push_back(i);
                for (int e = A.rp[i]; e < A.rp[i + 1]; e++) {
                    const int c = A.ci[e];
                    if (mark[c] != i) { mark[c] = i; row.push_back(c); }
                }
                for (int e = A.rp[i]; e < A.rp[i + 1]; e++) {
                    const int k = A.ci[e];
                    if (k >= i) continue;
                    for (int f = A.rp[k]; f < A.rp[k + 1]; f++) {
                        const int c = A.ci[f];
                        if (c > k && mark[c] != i) { mark[c] = i; row.push_back(c); }
                    }
                }
                std::sort(row.begin(), row.end());
                len[i - r0] = (int)row.size();
                cols.insert(cols.end(), row.begin(), row.end());
            }
        }
    };
    const int nt = std::max(1, std::min(threads, nblk));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (std::thread &t : pool) t.join();
    for (int b = 0; b < nblk; b++)
        for (size_t q = 0; q < blen[b].size(); q++) {
            const int i = b * kRows + (int)q;
            prow[i + 1] = prow[i] + blen[b][q];
        }
    pcol.resize((size_t)prow[n]);
    for (int b = 0; b < nblk; b++) {
        std::copy(bcols[b].begin(), bcols[b].end(), pcol.data() + prow[(size_t)b * kRows]);
        std::vector<int>().swap(bcols[b]);
    }
    for (int i = 0; i < n; i++) {
        const int *r = pcol.data() + prow[i];
        nl[i] = (int)(std::lower_bound(r, r + (prow[i + 1] - prow[i]), i) - r);
    }
}

// ilukC's factors from the flat pattern (iluk_pattern) and the factored
// values (the diagonal position holds the un-inverted pivot): L strict
// ascending + unit diagonal last, U diagonal first + strict ascending --
// iluk_emit's forms
void iluk_emit_flat(int n, const std::vector<long long> &prow, const std::vector<int> &nl,
                    const std::vector<int> &pcol, const std::vector<double> &val, Csr &L, Csr &U)
{
    L.n = U.n = n;
    L.rp.assign((size_t)n + 1, 0);
    U.rp.assign((size_t)n + 1, 0);
    for (int i = 0; i < n; i++) {
        L.rp[i + 1] = L.rp[i] + nl[i] + 1;
        U.rp[i + 1] = U.rp[i] + (int)(prow[i + 1] - prow[i] - nl[i]);
    }
    L.ci.resize(L.rp[n]);
    L.v.resize(L.rp[n]);
    U.ci.resize(U.rp[n]);
    U.v.resize(U.rp[n]);
    for (int i = 0; i < n; i++) {
        const long long p0 = prow[i], d0 = p0 + nl[i];
        std::copy(pcol.begin() + p0, pcol.begin() + d0, L.ci.begin() + L.rp[i]);
        std::copy(val.begin() + p0, val.begin() + d0, L.v.begin() + L.rp[i]);
        L.ci[L.rp[i + 1] - 1] = i;
        L.v[L.rp[i + 1] - 1] = 1.0;
        std::copy(pcol.begin() + d0, pcol.begin() + prow[i + 1], U.ci.begin() + U.rp[i]);
        std::copy(val.begin() + d0, val.begin() + prow[i + 1], U.v.begin() + U.rp[i]);
    }
}

int iluk_itsol(const Csr &A, int lof, Csr &L, Csr &U)
{
    const int n = A.n;
    std::vector<std::vector<int>> Lja, Uja;
    iluk_symbolic(A, lof, Lja, Uja);

    // ---- numeric (ilukC): D kept inverted, multipliers scaled by D[jrow]
    std::vector<std::vector<double>> Lma(n), Uma(n);
    std::vector<double> D(n), Draw(n);
    std::vector<int> jw(n, -1);
    for (int i = 0; i < n; i++) {
        Lma[i].assign(Lja[i].size(), 0.0);
        Uma[i].assign(Uja[i].size(), 0.0);
        for (size_t j = 0; j < Lja[i].size(); j++) jw[Lja[i][j]] = (int)j;
        jw[i] = i;
        D[i] = 0.0;
        for (size_t j = 0; j < Uja[i].size(); j++) jw[Uja[i][j]] = (int)j;
        for (int k = A.rp[i]; k < A.rp[i + 1]; k++) {
            int col = A.ci[k], jpos = jw[col];
            if (col < i) Lma[i][jpos] = A.v[k];
            else if (col == i) D[i] = A.v[k];
            else Uma[i][jpos] = A.v[k];
        }
        for (size_t j = 0; j < Lja[i].size(); j++) {
            int jrow = Lja[i][j];
            Lma[i][j] *= D[jrow];
            const double lij = Lma[i][j];
            for (size_t k = 0; k < Uja[jrow].size(); k++) {
                int col = Uja[jrow][k], jpos = jw[col];
                if (jpos == -1) continue;
                if (col < i) Lma[i][jpos] -= lij * Uma[jrow][k];
                else if (col == i) D[i] -= lij * Uma[jrow][k];
                else Uma[i][jpos] -= lij * Uma[jrow][k];
            }
        }
        for (int c : Lja[i]) jw[c] = -1;
        jw[i] = -1;
        for (int c : Uja[i]) jw[c] = -1;
        if (D[i] == 0.0) return GG_EZEROPIVOT;
        Draw[i] = D[i];
        D[i] = 1.0 / D[i];
    }

    iluk_emit(Lja, Uja, Lma, Uma, Draw, L, U);
    return 0;
}

void iluk_emit(const std::vector<std::vector<int>> &Lja, const std::vector<std::vector<int>> &Uja,
               const std::vector<std::vector<double>> &Lma, const std::vector<std::vector<double>> &Uma,
               const std::vector<double> &Draw, Csr &L, Csr &U)
{
    const int n = (int)Lja.size();
    // ---- emit: L strict ascending + unit diag last; U diag (un-inverted)
    //      first + strict upper ascending
    L.n = U.n = n;
    L.rp.assign(n + 1, 0);
    U.rp.assign(n + 1, 0);
    L.ci.clear(); L.v.clear(); U.ci.clear(); U.v.clear();
    std::vector<int> idx;
    for (int i = 0; i < n; i++) {
        for (size_t j = 0; j < Lja[i].size(); j++) { L.ci.push_back(Lja[i][j]); L.v.push_back(Lma[i][j]); }
        L.ci.push_back(i);
        L.v.push_back(1.0);
        L.rp[i + 1] = (int)L.ci.size();
        U.ci.push_back(i);
        U.v.push_back(Draw[i]);
        idx.resize(Uja[i].size());
        std::iota(idx.begin(), idx.end(), 0);
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return Uja[i][a] < Uja[i][b]; });
        for (int t : idx) { U.ci.push_back(Uja[i][t]); U.v.push_back(Uma[i][t]); }
        U.rp[i + 1] = (int)U.ci.size();
    }
}

}  // namespace gg
