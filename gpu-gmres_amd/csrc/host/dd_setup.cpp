// dd_setup.cpp -- host setup of the sharded (domain-decomposed) solve, SURVEY.md 8(e).
//
// The reference's DD path (etbr_dd: partition4 src/partition3.cpp:122-194,
// dd_form src/form_dd.cpp:32-110) orders a P-way partition as an ARROW matrix:
// interiors 0..P-1 first, the separator S (every endpoint of a cut edge) last.
// Interiors are mutually uncoupled, so with B = P A P^T:
//
//   ILU(0) of B has B's pattern (no fill); row-wise, in the reference's own
//   summation orders (LUSolve_ignoreZero, src/SpMV_compute.cpp:92-136):
//     interior row of part p   L: interior-p columns only
//                              U (walked from the row end): separator columns
//                                FIRST, then interior-p columns
//     separator row            L (walked from the row start): interior columns
//                                FIRST (any part), then separator columns
//                              U: separator columns only
//
// so the global triangular solves split EXACTLY (same operations, same order)
// into, per part p,
//     forward   y_I = L_II^-1 b_I                              (local)
//               y_S = L_SS^-1 (b_S - L_SI y_I)                 (needs interface y of every part)
//     backward  x_S = U_SS^-1 y_S                              (local, separator replicated)
//               x_I = U_II^-1 (y_I - U_IS x_S)                 (local)
// where the "- L_SI y_I" / "- U_IS x_S" terms are subtracted first, in the
// reference order, before the pure triangle runs.  Every part keeps a REPLICA
// of the separator (computed identically on every part); the only data every
// part needs from the others are the interface values: interior nodes that a
// separator row references.  One all-gather of those per SpMV and per L solve.
//
// A shard's local index space: [0, nI) its interior rows, [nI, nI + nS) the
// separator, then P * maxI halo slots (part q's interface at q * maxI + k).
#include <algorithm>

#include "../gg_internal.h"

namespace gg {

DDPlan dd_plan(const Csr &A, int P, int method)
{
    GG_REQUIRE(P >= 1 && P <= kMaxShards, GG_EINVAL,
               "dd: nparts must be in [1, " + std::to_string(kMaxShards) + "]");
    DDPlan D;
    D.n = A.n;
    D.P = P;
    std::vector<int> node_part;
    partition_arrow(A, P, method, node_part, D.part_size, D.pinv, D.q);
    D.begin.assign(P + 2, 0);
    for (int i = 0; i <= P; i++) D.begin[i + 1] = D.begin[i] + D.part_size[i];
    D.B = arrow_permute(A, D.pinv, D.q);
    Csr Lf, Uf;
    ilu0_left(D.B, Lf, Uf);
    D.cl = canon_lower_unit(Lf);
    D.cu = canon_upper_ignorezero(Uf);
    // interface lists: interior columns of separator rows of B (L's pattern is a subset)
    const int s0 = D.begin[P], n = D.n;
    D.iface.assign(P, {});
    D.hidx.assign(n, -1);
    std::vector<char> mark(s0, 0);
    for (int r = s0; r < n; r++)
        for (int k = D.B.rp[r]; k < D.B.rp[r + 1]; k++) {
            const int c = D.B.ci[k];
            if (c < s0) mark[c] = 1;
        }
    int part = 0;
    for (int c = 0; c < s0; c++) {
        if (!mark[c]) continue;
        while (c >= D.begin[part + 1]) part++;
        D.iface[part].push_back(c);
    }
    D.maxI = 0;
    for (int p = 0; p < P; p++) D.maxI = std::max(D.maxI, (int)D.iface[p].size());
    for (int p = 0; p < P; p++)
        for (size_t k = 0; k < D.iface[p].size(); k++)
            D.hidx[D.iface[p][k]] = p * D.maxI + (int)k;
    return D;
}

namespace {
CanonTri empty_tri(int n, bool lower)
{
    CanonTri T;
    T.lower = lower;
    T.off.n = n;
    T.off.rp.assign(n + 1, 0);
    T.d.assign(n, 1.0);
    return T;
}
void close_row(Csr &C) { C.rp.push_back((int)C.ci.size()); }
}  // namespace

DDShardHost dd_shard(const DDPlan &D, int p)
{
    GG_REQUIRE(p >= 0 && p < D.P, GG_EINVAL, "dd: part out of range");
    const int b0 = D.begin[p], b1 = D.begin[p + 1], s0 = D.begin[D.P], n = D.n;
    DDShardHost S;
    S.p = p;
    S.nI = b1 - b0;
    S.nS = n - s0;
    const int nI = S.nI, nS = S.nS;
    auto loc_int = [&](int c) { return c - b0; };
    auto loc_sep = [&](int c) { return c - s0; };
    // rows: interior of p, then the separator
    S.rows.reserve(nI + nS);
    for (int g = b0; g < b1; g++) S.rows.push_back(g);
    for (int g = s0; g < n; g++) S.rows.push_back(g);
    // A, local column space [I | S | halo]
    S.A.n = nI + nS;
    S.A.rp.assign(1, 0);
    for (int g : S.rows) {
        const bool sep = g >= s0;
        for (int k = D.B.rp[g]; k < D.B.rp[g + 1]; k++) {
            const int c = D.B.ci[k];
            int lc;
            if (c >= s0) lc = nI + loc_sep(c);
            else if (!sep) {
                GG_REQUIRE(c >= b0 && c < b1, GG_EINVAL, "dd: interior rows of two parts are coupled");
                lc = loc_int(c);
            } else {
                GG_REQUIRE(D.hidx[c] >= 0, GG_EINVAL, "dd: interface list incomplete");
                lc = nI + nS + D.hidx[c];
            }
            S.A.ci.push_back(lc);
            S.A.v.push_back(D.B.v[k]);
        }
        close_row(S.A);
    }
    // lower triangle
    S.LI = empty_tri(0, true);
    S.LI.off.rp.assign(1, 0);
    S.LI.d.clear();
    for (int g = b0; g < b1; g++) {
        for (int k = D.cl.off.rp[g]; k < D.cl.off.rp[g + 1]; k++) {
            const int c = D.cl.off.ci[k];
            GG_REQUIRE(c >= b0 && c < g, GG_EINVAL, "dd: interior L row leaves its part");
            S.LI.off.ci.push_back(loc_int(c));
            S.LI.off.v.push_back(D.cl.off.v[k]);
        }
        close_row(S.LI.off);
        S.LI.d.push_back(D.cl.d[g]);
    }
    S.LI.off.n = nI;
    S.LS = empty_tri(0, true);
    S.LS.off.rp.assign(1, 0);
    S.LS.d.clear();
    S.LSH.n = nS;
    S.LSH.rp.assign(1, 0);
    for (int g = s0; g < n; g++) {
        int k = D.cl.off.rp[g];
        const int ke = D.cl.off.rp[g + 1];
        for (; k < ke && D.cl.off.ci[k] < s0; k++) {      // interior terms come first
            const int c = D.cl.off.ci[k];
            GG_REQUIRE(D.hidx[c] >= 0, GG_EINVAL, "dd: L couples a non-interface node");
            S.LSH.ci.push_back(D.hidx[c]);
            S.LSH.v.push_back(D.cl.off.v[k]);
        }
        for (; k < ke; k++) {
            const int c = D.cl.off.ci[k];
            GG_REQUIRE(c >= s0 && c < g, GG_EINVAL, "dd: separator L row out of order");
            S.LS.off.ci.push_back(loc_sep(c));
            S.LS.off.v.push_back(D.cl.off.v[k]);
        }
        close_row(S.LSH);
        close_row(S.LS.off);
        S.LS.d.push_back(D.cl.d[g]);
    }
    S.LS.off.n = nS;
    // upper triangle (canonical order walks each row from its end)
    S.UI = empty_tri(0, false);
    S.UI.off.rp.assign(1, 0);
    S.UI.d.clear();
    S.UIS.n = nI;
    S.UIS.rp.assign(1, 0);
    for (int g = b0; g < b1; g++) {
        int k = D.cu.off.rp[g];
        const int ke = D.cu.off.rp[g + 1];
        for (; k < ke && D.cu.off.ci[k] >= s0; k++) {      // separator terms come first
            S.UIS.ci.push_back(loc_sep(D.cu.off.ci[k]));
            S.UIS.v.push_back(D.cu.off.v[k]);
        }
        for (; k < ke; k++) {
            const int c = D.cu.off.ci[k];
            GG_REQUIRE(c > g && c < b1, GG_EINVAL, "dd: interior U row out of order");
            S.UI.off.ci.push_back(loc_int(c));
            S.UI.off.v.push_back(D.cu.off.v[k]);
        }
        close_row(S.UIS);
        close_row(S.UI.off);
        S.UI.d.push_back(D.cu.d[g]);
    }
    S.UI.off.n = nI;
    S.US = empty_tri(0, false);
    S.US.off.rp.assign(1, 0);
    S.US.d.clear();
    for (int g = s0; g < n; g++) {
        for (int k = D.cu.off.rp[g]; k < D.cu.off.rp[g + 1]; k++) {
            const int c = D.cu.off.ci[k];
            GG_REQUIRE(c > g, GG_EINVAL, "dd: separator U row couples an interior node");
            S.US.off.ci.push_back(loc_sep(c));
            S.US.off.v.push_back(D.cu.off.v[k]);
        }
        close_row(S.US.off);
        S.US.d.push_back(D.cu.d[g]);
    }
    S.US.off.n = nS;
    // own interface nodes (interior-local), ascending
    for (int c : D.iface[p]) S.iface.push_back(loc_int(c));
    return S;
}

}  // namespace gg
