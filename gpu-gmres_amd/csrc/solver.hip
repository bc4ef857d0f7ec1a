// solver.hip -- device-resident restarted GMRES(m) for MI355X and its C ABI.
//
// Engines:
//   left  : GMRES_GPU_leftILU0 / GMRES_leftILU0   src/gmres.cu:1438-1696, :566-717
//   split : GMRESilu_GPU / GMRESilu               src/gmres.cu:2254-2446, :2069-2252
// Differences from the reference, all deliberate:
//   * fp64 everywhere; H, Givens, s on the device; one host sync per restart
//     cycle instead of (i+2) blocking scalar reads per inner iteration;
//   * Update uses the last filled column when max_iter cuts a cycle short;
//   * lucky breakdown (H[i+1,i] == 0) does not divide by zero.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <atomic>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>

#include "kernels.h"
#include "gg_solver.h"

namespace gg {

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }

void DevCsr::upload(const Csr &A, hipStream_t st)
{
    n = A.n;
    nnz = A.nnz();
    rp.upload(A.rp, st);
    // two spare entries: the SpMV reads entries in aligned pairs and may touch
    // the one after a block's last entry (never used)
    ci.alloc(A.ci.size() + 2);
    v.alloc(A.v.size() + 2);
    GG_HIP(hipMemsetAsync(ci.p, 0, ci.n * sizeof(int), st));
    GG_HIP(hipMemsetAsync(v.p, 0, v.n * sizeof(double), st));
    if (!A.ci.empty()) {
        GG_HIP(hipMemcpyAsync(ci.p, A.ci.data(), A.ci.size() * sizeof(int), hipMemcpyHostToDevice, st));
        GG_HIP(hipMemcpyAsync(v.p, A.v.data(), A.v.size() * sizeof(double), hipMemcpyHostToDevice, st));
    }
    std::vector<int> lr;
    std::vector<int> b = spmv_blocks(A, lr);
    nblk = (int)b.size() - 1;
    blk.upload(b, st);
    nlong = (int)lr.size();
    long_rows.upload(lr, st);
    // sliced ELL when every 64-row slice is short and evenly filled (grids,
    // banded / stencil matrices): padded entries <= 1.25 nnz + one slice
    sell = false;
    const char *force_csr = std::getenv("GG_SPMV_CSR");
    if (n > 0 && !(force_csr && force_csr[0] == '1')) {
        nslice = (n + 63) / 64;
        std::vector<int> sp(nslice + 1, 0);
        long long tot = 0;
        int wmax = 0;
        bool fits = true;                        // int32 entry offsets
        for (int s_ = 0; s_ < nslice && fits; s_++) {
            int w = 0;
            for (int r = s_ * 64; r < std::min(n, s_ * 64 + 64); r++) w = std::max(w, A.rp[r + 1] - A.rp[r]);
            wmax = std::max(wmax, w);
            tot += 64LL * w;
            fits = tot < (1LL << 31);
            sp[s_ + 1] = (int)std::min<long long>(tot, 1LL << 30);
        }
        if (fits && wmax <= 64 && tot <= (long long)(1.25 * nnz) + 64LL * wmax) {
            std::vector<int> c(tot, -1);
            std::vector<double> vv(tot, 0.0);
            for (int r = 0; r < n; r++) {
                const int s_ = r / 64, l = r % 64;
                for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
                    const long long e = sp[s_] + 64LL * (k - A.rp[r]) + l;
                    c[e] = A.ci[k];
                    vv[e] = A.v[k];
                }
            }
            sptr.upload(sp, st);
            sci.upload(c, st);
            sv.upload(vv, st);
            sell = true;
            GG_HIP(hipStreamSynchronize(st));   // the host staging vectors go out of scope
        }
    }
    build_panels(A, st);
}

// Column panels for the CSR-stream matrices whose gathers scatter over an x
// far larger than an XCD's L2 (the C3 stand-in: 44 MB of x, uniform columns,
// one 64-B line fetched per 8-B term, profiles/pmc_traffic_c3.json).  Panel
// width GG_SPMV_PANEL doubles (default 786,432 = 6 MiB; the XCD's L2 is 4 MiB:
// the C3 stand-in's SpMV 971 us unpanelled, 702 / 648 / 652 / 716 / 921 us at
// 3 / 4 / 6 / 8 / 22 MiB panels with cached entry loads, 640 / 626 / 692 us at
// 4 / 6 / 8 MiB with the entries streamed non-temporally (GG_PANEL_NT),
// profiles/r06/c3_panel_ab.txt); used when the matrix
// has at least GG_SPMV_PANEL_MIN rows (default 2^21), more than one panel, and
// every row's columns strictly ascending (the panel order is then the CSR
// order).  GG_SPMV_PANEL=0 turns it off.
void DevCsr::build_panels(const Csr &A, hipStream_t st)
{
    panel = false;
    const char *pe = std::getenv("GG_SPMV_PANEL");
    const long long w = pe ? atoll(pe) : 786432;
    const char *me = std::getenv("GG_SPMV_PANEL_MIN");
    const long long nmin = me ? atoll(me) : (1LL << 21);
    if (sell || w <= 0 || n < nmin || n <= w || nnz == 0) return;
    for (int r = 0; r < n; r++)
        for (int k = A.rp[r] + 1; k < A.rp[r + 1]; k++)
            if (A.ci[k] <= A.ci[k - 1]) return;            // not ascending: the panel order would differ
    pw = (int)w;
    npanel = (int)((n + w - 1) / w);
    rtile = 0;
    const char *rte = std::getenv("GG_SPMV_RTILE");
    const int rtb = rte ? atoi(rte) : 0;
    if (rtb > 0) {
        // Row tiles: rtb contiguous row ranges of about equal cost (entries +
        // a y access per row), each one block of ONE launch that walks its
        // rows' segments panel by panel -- a row's segments in column order,
        // its running sum in y touched only by its own block, and every block
        // in about the same panel at the same time (x's slice shared in L2).
        // Measured slower than the panel-major launches, so off by default
        // (C3 stand-in, one box, profiles/r06/c3_rtile_ab.txt: 670-865 us at
        // 512-2048 row blocks and 2-6 MiB panels against 623 us): a block's
        // sub-blocks run one after another, each a dependent load -> gather ->
        // sum -> store chain, where the panel-major launch keeps 8 of them in
        // flight per CU
        long long cost = 0;
        for (int r = 0; r < n; r++) cost += (A.rp[r + 1] - A.rp[r]) + 4;
        const long long target = std::max<long long>(1, (cost + rtb - 1) / rtb);
        std::vector<int> rb{0};
        long long acc = 0;
        for (int r = 0; r < n; r++) {
            acc += (A.rp[r + 1] - A.rp[r]) + 4;
            if (acc >= target && r + 1 < n) {
                rb.push_back(r + 1);
                acc = 0;
            }
        }
        rb.push_back(n);
        const int nb = (int)rb.size() - 1;
        std::vector<int> srow, sptr_h, pc(nnz), pb, rts, zr;
        std::vector<double> pvv(nnz);
        srow.reserve((size_t)n * 2);
        sptr_h.reserve((size_t)n * 2 + 1);
        std::vector<int> cur(A.rp.begin(), A.rp.end() - 1);
        long long e = 0;
        for (int b = 0; b < nb; b++) {
            rts.push_back((int)pb.size());
            for (int p = 0; p < npanel; p++) {
                const long long hi = std::min<long long>((long long)(p + 1) * w, n);
                int nseg_sb = 0, nent_sb = 0;
                for (int r = rb[b]; r < rb[b + 1]; r++) {
                    int k = cur[r];
                    const int k1 = A.rp[r + 1];
                    while (k < k1 && A.ci[k] < hi) {
                        // one segment (or a piece of it) of at most kSpmvCap entries
                        int kend = k;
                        while (kend < k1 && A.ci[kend] < hi && kend - k < kSpmvCap) kend++;
                        const int len = kend - k;
                        if (nseg_sb == 0 || nseg_sb == 256 || nent_sb + len > kSpmvCap) {
                            pb.push_back((int)srow.size());       // a new sub-block
                            nseg_sb = 0;
                            nent_sb = 0;
                        }
                        srow.push_back(k == A.rp[r] ? ~r : r);
                        sptr_h.push_back((int)e);
                        for (; k < kend; k++, e++) {
                            pc[e] = A.ci[k];
                            pvv[e] = A.v[k];
                        }
                        nseg_sb++;
                        nent_sb += len;
                    }
                    cur[r] = k;
                }
            }
        }
        rts.push_back((int)pb.size());
        pb.push_back((int)srow.size());
        sptr_h.push_back((int)e);
        for (int r = 0; r < n; r++)
            if (A.rp[r + 1] == A.rp[r]) zr.push_back(r);    // empty rows: y = 0
        nseg = (long long)srow.size();
        nzero = (int)zr.size();
        seg_row.upload(srow, st);
        seg_ptr.upload(sptr_h, st);
        pci.upload(pc, st);
        pv.upload(pvv, st);
        zero_rows.upload(zr.empty() ? std::vector<int>{0} : zr, st);
        pblk.upload(pb, st);
        rt_sub.upload(rts, st);
        pan_blk_h.assign(npanel + 1, 0);
        rtile = nb;
        panel = true;
        GG_HIP(hipStreamSynchronize(st));
        return;
    }
    std::vector<int> cur(A.rp.begin(), A.rp.end() - 1);  // per row: its next entry
    std::vector<int> ps(npanel + 1, 0), srow, sptr_h, pc(nnz);
    std::vector<double> pvv(nnz);
    std::vector<char> seen(n, 0);
    srow.reserve((size_t)n * 4);
    sptr_h.reserve((size_t)n * 4 + 1);
    long long e = 0;
    for (int p = 0; p < npanel; p++) {
        ps[p] = (int)srow.size();
        const long long hi = std::min<long long>((long long)(p + 1) * w, n);
        for (int r = 0; r < n; r++) {
            int k = cur[r];
            const int k1 = A.rp[r + 1];
            if (k >= k1 || A.ci[k] >= hi) continue;
            srow.push_back(seen[r] ? r : ~r);
            seen[r] = 1;
            sptr_h.push_back((int)e);
            for (; k < k1 && A.ci[k] < hi; k++, e++) {
                pc[e] = A.ci[k];
                pvv[e] = A.v[k];
            }
            cur[r] = k;
        }
    }
    ps[npanel] = (int)srow.size();
    sptr_h.push_back((int)e);
    // per panel, blocks of <= 256 segments holding <= kSpmvCap entries (a
    // longer segment: no panels)
    std::vector<int> pb;
    pan_blk_h.assign(npanel + 1, 0);
    for (int p = 0; p < npanel; p++) {
        pan_blk_h[p] = (int)pb.size();
        int sg = ps[p];
        while (sg < ps[p + 1]) {
            pb.push_back(sg);
            const int start = sg;
            while (sg < ps[p + 1] && sg - start < 256 && sptr_h[sg + 1] - sptr_h[start] <= kSpmvCap) sg++;
            if (sg == start) return;                       // one segment beyond a block's capacity
        }
    }
    pan_blk_h[npanel] = (int)pb.size();
    pb.push_back(ps[npanel]);
    std::vector<int> zr;
    for (int r = 0; r < n; r++)
        if (!seen[r]) zr.push_back(r);                    // empty rows: y = 0
    nseg = (long long)srow.size();
    nzero = (int)zr.size();
    pan_seg.upload(ps, st);
    seg_row.upload(srow, st);
    seg_ptr.upload(sptr_h, st);
    pci.upload(pc, st);
    pv.upload(pvv, st);
    zero_rows.upload(zr.empty() ? std::vector<int>{0} : zr, st);
    pblk.upload(pb, st);
    panel = true;
    GG_HIP(hipStreamSynchronize(st));
}

void DevCsr::copy_from(const DevCsr &o, hipStream_t st)
{
    n = o.n;
    nnz = o.nnz;
    nblk = o.nblk;
    nlong = o.nlong;
    sell = o.sell;
    nslice = o.nslice;
    auto dup = [&](auto &dst, const auto &src) {
        dst.alloc(src.n);
        GG_HIP(hipMemcpyAsync(dst.p, src.p, src.n * sizeof(*src.p), hipMemcpyDeviceToDevice, st));
    };
    dup(rp, o.rp);
    dup(ci, o.ci);
    dup(v, o.v);
    dup(blk, o.blk);
    dup(long_rows, o.long_rows);
    if (sell) {
        dup(sptr, o.sptr);
        dup(sci, o.sci);
        dup(sv, o.sv);
    }
    panel = o.panel;
    npanel = o.npanel;
    pw = o.pw;
    nseg = o.nseg;
    nzero = o.nzero;
    rtile = o.rtile;
    if (rtile) dup(rt_sub, o.rt_sub);
    if (panel && !rtile) dup(pan_seg, o.pan_seg);
    if (panel) {
        dup(seg_row, o.seg_row);
        dup(seg_ptr, o.seg_ptr);
        dup(pci, o.pci);
        dup(pv, o.pv);
        dup(zero_rows, o.zero_rows);
        dup(pblk, o.pblk);
    }
    pan_blk_h = o.pan_blk_h;
}

long long round_up(long long a, long long b) { return (a + b - 1) / b * b; }

// Tiles of a 3D layout in a forward dependency order: tile (J, K) waits on
// (J-1, K) and (J, K-1), whose hand-offs lag it by about the same time since
// planes are skewed by one step like lines (k_trsv_tile3d, traced: 3.7-4.2 and
// 4.2-4.8 us), so tiles are taken by that expected start, 7J + 8K, then J
// (round 2's two-step plane skew: 2J + 3K).
// Any order that lists a tile after both its sources keeps the persistent grid
// deadlock-free (every workgroup takes its tiles in list order).
std::vector<int> tile_order(const Wave2D &w)
{
    std::vector<int> ord(w.nbands);
    for (int q = 0; q < w.nbands; q++) ord[q] = q;
    auto key = [&](int q) { return 7LL * (q % w.NJ) + 8LL * (q / w.NJ); };
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
        const long long ka = key(a), kb = key(b);
        return ka != kb ? ka < kb : (a % w.NJ) < (b % w.NJ);
    });
    return ord;
}

// Build a device triangular solve from a canonical triangle.  WAVE2D when a
// grid layout is active, else LEVEL (one launch per dependency level).
void build_level(DevTri &T, const CanonTri &C, const Levels &lv, hipStream_t st, bool no_long = false);

bool identity_map(const std::vector<long long> &m, int n)
{
    for (int r = 0; r < n; r++)
        if (m[r] != r) return false;
    return true;
}

void build_tri(DevTri &T, const CanonTri &C, const Wave2D *wl, const std::vector<long long> *nat2lay,
               long long Ppad, hipStream_t st)
{
    T.tail.reset();
    T.tail_fma.reset();
    T.bofs = 0;
    T.ncoup = 0;
    T.cbytes = 0;
    T.lower = C.lower;
    T.n = C.off.n;
    T.il = !C.lower && wl && wl->ok && wl->u_inline_first;
    const int n = C.off.n;
    if (wl && wl->ok) {
        T.kind = DevTri::WAVE2D;
        T.wl = *wl;
        const bool d3 = wl->nz > 1;
        std::vector<double> c1(Ppad, 0.0), c2(Ppad, 0.0), dv(Ppad, 1.0), rv(Ppad, 1.0);
        std::vector<double> c0(d3 ? Ppad : 0, 0.0);
        const int K = wl->skew - 1;              // fill offsets nx-1 .. nx-K (2D)
        std::vector<double> ce1(K >= 1 ? Ppad : 0, 0.0), ce2(K >= 2 ? Ppad : 0, 0.0);
        bool unit = true, rcp_ok = true, mul_ok = true;
        const int nx = wl->nx;
        const long long nxy = (long long)wl->nx * wl->ny;
        for (int r = 0; r < n; r++) {
            const long long p = (*nat2lay)[r];
            for (int k = C.off.rp[r]; k < C.off.rp[r + 1]; k++) {
                const long long off = std::abs((long long)C.off.ci[k] - r);
                if (d3 && off == nxy) c0[p] = C.off.v[k];
                else if (K >= 1 && off == nx - 1) ce1[p] = C.off.v[k];
                else if (K >= 2 && off == nx - 2) ce2[p] = C.off.v[k];
                else (off == nx ? c1 : c2)[p] = C.off.v[k];
            }
            const double d = C.d[r];
            dv[p] = d;
            rv[p] = 1.0 / d;
            if (d != 1.0) unit = false;
            // WD_RCP keeps every intermediate normal for 2^-100 <= |d| <= 2^100
            if (!(std::fabs(d) >= 0x1p-100 && std::fabs(d) <= 0x1p100)) rcp_ok = false;
            // WD_MUL: 1/d finite and normal
            if (!(std::fabs(d) >= 0x1p-1020 && std::fabs(d) <= 0x1p1020)) mul_ok = false;
        }
        T.c1.upload(c1, st);
        T.c2.upload(c2, st);
        if (K >= 1) T.ce1.upload(ce1, st);
        if (K >= 2) T.ce2.upload(ce2, st);
        if (d3) T.c0.upload(c0, st);
        if (d3 && !wl->tile) {
            T.prog.alloc((size_t)wl->nz * wl->nbands);
            GG_HIP(hipMemsetAsync(T.prog.p, 0, T.prog.n * sizeof(unsigned long long), st));
        }
        if (wl->tile) T.order.upload(tile_order(*wl), st);
        T.rcp_ok = false;
        T.mul_ok = false;
        if (unit) {
            T.div = WD_UNIT;
        } else {
            T.dw.upload(dv, st);
            const char *hw = std::getenv("GG_WAVE_HWDIV");
            T.rcp_ok = rcp_ok && !(hw && hw[0] == '1');
            T.mul_ok = mul_ok;
            if (T.rcp_ok || T.mul_ok) T.rw.upload(rv, st);
            T.div = T.rcp_ok ? WD_RCP : WD_HW;
        }
        // GG_DIV_FMA: unskewed 2D grids and 3D tiles in the canonical row order
        // (the plane term, the line term, the in-line term), the unit L or a U
        // whose 1/d are normal
        // GG_FMA_TILE (diagnostics, default 3): bit 0 / 1 admits the 3D tiles' L / U
        const char *ft = std::getenv("GG_FMA_TILE");
        const int ftm = ft ? atoi(ft) : 3;
        const bool tile_ok = wl->tile && (ftm & (C.lower ? 1 : 2)) && (!C.lower || unit);
        // (the fused rows take the in-line term first whatever the canonical
        // order, so the split engine's in-line-first U is admitted too, and
        // its non-unit L as a pre-scaled lower triangle)
        // Round 6: skewed 2D grids (ILU(1) / ILU(2) factors, GG_FMA_SKEW default
        // 1) too -- nearest term first: the in-line term, then the fills
        // (nx-2, nx-1), then the line term (nx); the fills pre-scaled for U
        const char *fs = std::getenv("GG_FMA_SKEW");
        const bool skew_ok = !d3 && !(fs && fs[0] == '0');
        T.fma_ok = (!d3 || tile_ok) && (K == 0 || skew_ok) && (unit ? C.lower : mul_ok);
        if (T.fma_ok && !unit) {
            std::vector<double> s1(Ppad, 0.0), s2(Ppad, 0.0), s0(d3 ? Ppad : 0, 0.0);
            std::vector<double> se1(K >= 1 ? Ppad : 0, 0.0), se2(K >= 2 ? Ppad : 0, 0.0);
            for (long long p = 0; p < Ppad; p++) {
                s1[p] = c1[p] * rv[p];
                s2[p] = c2[p] * rv[p];
                if (d3) s0[p] = c0[p] * rv[p];
                if (K >= 1) se1[p] = ce1[p] * rv[p];
                if (K >= 2) se2[p] = ce2[p] * rv[p];
            }
            T.c1s.upload(s1, st);
            T.c2s.upload(s2, st);
            if (d3) T.c0s.upload(s0, st);
            if (K >= 1) T.ce1s.upload(se1, st);
            if (K >= 2) T.ce2s.upload(se2, st);
        }
        // one hand-off granule per band (tile) and step, then per workgroup 64
        // zero granules (dummy reads) and 64 write-only ones (dummy re-arms),
        // for up to kTileDummyBlocks workgroups: one line that every boundary
        // wave polled and re-armed would be a hot spot on one memory channel
        // (+ 64 words: the 3D tile kernel's task queue, k_trsv_tile3d)
        const long long ngran = wl->ngran();
        const long long ndummy = 128LL * kTileDummyBlocks;
        T.bnd.alloc((size_t)(ngran + ndummy + 64));
        launch_fill_u64(T.bnd.p, ngran, kSentinel, st);
        launch_fill_u64(T.bnd.p + ngran, ndummy + 64, 0ull, st);
        // algorithmic bytes: this triangle's share of B_ilu --
        // its CSR entries (a stored diagonal included), one row-pointer array, b
        // read and x written -- the reference's formulation of the same solve
        T.bytes = T.bytes_mul = 12.0 * ((double)C.off.nnz() + (unit ? 0.0 : (double)n)) + 4.0 * (n + 1) + 16.0 * n;
        // what the wavefront kernel itself streams (no indices): b, two
        // coefficients, (divisor (, reciprocal)), x per grid point
        T.stream_bytes = (double)n * (8.0 * ((unit ? 4 : T.rcp_ok ? 6 : 5) + (d3 ? (wl->tile ? 1 : 2) : 0) + K));
        T.stream_bytes_mul = (double)n * (8.0 * ((unit ? 4 : 5) + (d3 ? (wl->tile ? 1 : 2) : 0) + K));
    } else if (nat2lay && !identity_map(*nat2lay, n)) {
        // a relabeled (RCM) layout: the triangle in layout space
        CanonTri Cr;
        Levels lv;
        relabel_tri(C, *nat2lay, Cr, lv);
        build_level(T, Cr, lv, st);
    } else {
        build_level(T, C, level_sets(C), st);
    }
}

// LEVEL triangle: the flow kernel's tasks over the level sets `lv` of C
// (no_long: every row one lane's -- GG_DIV_FMA's rows have no long-row form)
void build_level(DevTri &T, const CanonTri &C, const Levels &lv, hipStream_t st, bool no_long)
{
    const int n = C.off.n;
    {
        T.kind = DevTri::LEVEL;
        T.off.upload(C.off, st);
        T.d.upload(C.d, st);
        T.lev_ptr = lv.ptr;
        T.lev_rows.upload(lv.rows, st);
        // flow tasks in level order: runs of up to 64 short rows, long rows alone
        const char *fl = std::getenv("GG_FLOW_LONG");       // tuning: terms above which a row is long
        const int flow_long = no_long ? INT_MAX : fl ? std::max(0, atoi(fl)) : kFlowLong;
        std::vector<int4> tasks;
        int run0 = 0, runn = 0;
        auto flush = [&]() {
            if (runn) tasks.push_back(make_int4(run0, runn, 0, 0));
            runn = 0;
        };
        for (int q = 0; q < (int)lv.rows.size(); q++) {
            const int r = lv.rows[q];
            if (C.off.rp[r + 1] - C.off.rp[r] > flow_long) {
                flush();
                tasks.push_back(make_int4(q, -1, 0, 0));
            } else {
                if (runn == 0) run0 = q;
                if (++runn == 64) flush();
            }
        }
        flush();
        // the sliced copy, where its padding stays within 2x the short rows'
        // terms (GG_FLOW_ELL=0: the CSR form only)
        long long groups = 0, terms = 0;
        for (int4 &tk : tasks) {
            if (tk.y < 0) continue;
            int w = 0;
            for (int j = 0; j < tk.y; j++) {
                const int r = lv.rows[tk.x + j];
                w = std::max(w, C.off.rp[r + 1] - C.off.rp[r]);
                terms += C.off.rp[r + 1] - C.off.rp[r];
            }
            tk.z = (int)groups;
            tk.w = w;
            groups += w;
        }
        const char *fe = std::getenv("GG_FLOW_ELL");
        T.ell = !(fe && fe[0] == '0') && groups * 64 <= 2 * terms + 64LL * (long long)tasks.size() &&
                groups * 64 < INT_MAX;
        T.eci.release();
        T.ev.release();
        std::vector<int> eci;
        std::vector<double> ev;
        if (T.ell) {
            eci.assign((size_t)std::max<long long>(groups, 1) * 64, -1);
            ev.assign(eci.size(), 0.0);
            for (const int4 &tk : tasks) {
                if (tk.y < 0) continue;
                for (int j = 0; j < tk.y; j++) {
                    const int r = lv.rows[tk.x + j];
                    for (int k = C.off.rp[r]; k < C.off.rp[r + 1]; k++) {
                        const size_t e = ((size_t)tk.z + (k - C.off.rp[r])) * 64 + j;
                        eci[e] = C.off.ci[k];
                        ev[e] = C.off.v[k];
                    }
                }
            }
            T.eci.upload(eci, st);
            T.ev.upload(ev, st);
        }
        T.ntask = (int)tasks.size();
        T.tasks.upload(tasks, st);
        GG_HIP(hipStreamSynchronize(st));       // the host vectors end here
        T.bytes = 12.0 * C.off.nnz() + 4.0 * (n + 1) + 24.0 * n;
    }
}

void build_tri_bordered(DevTri &T, const CanonTri &C, const CanonTri &Cg, const Wave2D &wl, hipStream_t st)
{
    const int nt = wl.bnt;
    // the grid block: a plain 2D wavefront in its own slot space
    Wave2D wg = wl;
    wg.bnt = 0;
    wg.bofs = 0;
    wg.P = wg.P2;
    std::vector<long long> gslot(Cg.off.n);
    for (int r = 0; r < Cg.off.n; r++) gslot[r] = wg.slot(r);
    build_tri(T, Cg, &wg, &gslot, round_up(wg.P2, 512), st);
    const bool grid_fma = T.fma_ok && T.wl.skew == 1, grid_unit = T.div == WD_UNIT;
    T.bofs = wl.bofs;
    // the tail over the whole layout (its columns are slots); level sets over
    // the tail's own rows only (an upper tail's grid columns are final before it runs)
    CanonTri Ct;
    Ct.lower = C.lower;
    Ct.off.n = nt;
    Ct.off.rp.assign(nt + 1, 0);
    Ct.d.assign(C.d.begin(), C.d.begin() + nt);
    for (int r = 0; r < nt; r++) {
        for (int k = C.off.rp[r]; k < C.off.rp[r + 1]; k++) {
            Ct.off.ci.push_back((int)wl.slot(C.off.ci[k]));
            Ct.off.v.push_back(C.off.v[k]);
        }
        Ct.off.rp[r + 1] = (int)Ct.off.ci.size();
    }
    T.tail = std::make_unique<DevTri>();
    T.tail->lower = C.lower;
    T.tail->n = nt;
    const Levels tlv = level_sets(Ct, true);
    build_level(*T.tail, Ct, tlv, st);
    // a small tail (an MNA system's pads and branches: hundreds of rows in a
    // few levels) runs in one workgroup, levels separated by barriers
    // (kernels.hip k_tail_small); GG_TAIL_SMALL=0 keeps the flow kernel
    const char *ts = std::getenv("GG_TAIL_SMALL");
    const bool small = !(ts && ts[0] == '0') && nt <= kTailSmallRows && (int)tlv.ptr.size() - 1 <= kTailSmallLevels;
    if (small) T.tail->lev_ptr_d.upload(tlv.ptr, st);
    // WD_MUL on the whole triangle needs every tail 1/d finite and normal too
    bool tail_mul = true;
    std::vector<double> ry(nt);
    for (int r = 0; r < nt; r++) {
        const double d = Ct.d[r];
        if (!(std::fabs(d) >= 0x1p-1020 && std::fabs(d) <= 0x1p1020)) tail_mul = false;
        ry[r] = 1.0 / d;
    }
    T.mul_ok = T.mul_ok && tail_mul;
    if (T.mul_ok) T.tail->rw.upload(ry, st);
    // GG_DIV_FMA: the mesh rows' tail terms lead the fused row (oracle
    // orc_set_fma_tail), so the forward solve forms them before the wavefront
    // as fused multiply-adds on the unit L (a non-unit L would need them
    // inside RN(b * y): that triangle takes WD_MUL instead); the tail rows as
    // their own fused rows -- pre-scaled by y = RN(1/d), nearest term first
    bool tail_unit = true;
    for (int r = 0; r < nt; r++) tail_unit = tail_unit && Ct.d[r] == 1.0;
    T.fma_ok = grid_fma && (C.lower ? (grid_unit && tail_unit) : tail_mul);
    if (T.fma_ok) {
        CanonTri Cf;
        Cf.lower = C.lower;
        Cf.off.n = nt;
        Cf.off.rp = Ct.off.rp;
        Cf.off.ci.resize(Ct.off.ci.size());
        Cf.off.v.resize(Ct.off.v.size());
        Cf.d.assign(nt, 1.0);
        for (int r = 0; r < nt; r++) {
            const int k0 = Ct.off.rp[r], k1 = Ct.off.rp[r + 1];
            for (int q = 0; q < k1 - k0; q++) {
                // lower: nearest first = descending columns; upper: ascending (canonical)
                const int k = C.lower ? k1 - 1 - q : k0 + q;
                Cf.off.ci[k0 + q] = Ct.off.ci[k];
                Cf.off.v[k0 + q] = Ct.off.v[k] * ry[r];
            }
        }
        T.tail_fma = std::make_unique<DevTri>();
        T.tail_fma->lower = C.lower;
        T.tail_fma->n = nt;
        build_level(*T.tail_fma, Cf, tlv, st, true);
        T.tail_fma->fmrow = true;
        T.tail_fma->rw.upload(ry, st);
        if (small) T.tail_fma->lev_ptr_d.upload(tlv.ptr, st);
    }
    // the grid rows' tail terms (lower: the leading terms of the row, detect_border2d)
    std::vector<long long> cs;
    std::vector<int> crp(1, 0), cci;
    std::vector<double> cv;
    for (int r = nt; r < C.off.n; r++) {
        const int k0 = C.off.rp[r];
        int k = k0;
        while (k < C.off.rp[r + 1] && C.off.ci[k] < nt) k++;
        if (k == k0) continue;
        GG_REQUIRE(C.lower, GG_EINVAL, "bordered grid: an upper grid row references the tail");
        cs.push_back(wl.slot(r));
        for (int q = k0; q < k; q++) {
            cci.push_back(C.off.ci[q]);
            cv.push_back(C.off.v[q]);
        }
        crp.push_back((int)cci.size());
    }
    T.ncoup = (int)cs.size();
    if (T.ncoup) {
        T.cslot.upload(cs, st);
        T.crp.upload(crp, st);
        T.cci.upload(cci, st);
        T.cv.upload(cv, st);
    }
    // coupling: per row its slot, b read + written; per term column, value, x
    T.cbytes = 24.0 * T.ncoup + 4.0 * (T.ncoup + 1) + 20.0 * cci.size();
    // the uploads above (ry, tlv.ptr, cs / crp / cci / cv) are asynchronous
    // copies from these local vectors: they must have been taken before the
    // vectors go out of scope (as build_level)
    GG_HIP(hipStreamSynchronize(st));
}

}  // namespace gg

using namespace gg;

// struct gg_solver: gg_solver.h (shared with batch.hip)

namespace {

int fail(const Error &e)
{
    set_error(e.msg);
    return e.code;
}

#define GG_API_BEGIN try {
#define GG_API_END                                                   \
    }                                                                \
    catch (const gg::Error &e) { return fail(e); }                   \
    catch (const std::bad_alloc &) { return fail({GG_ENOMEM, "host allocation failed"}); } \
    catch (const std::exception &e) { return fail({GG_EINVAL, e.what()}); }

void check_csr(int n, const int *rp, const int *ci, const double *v, const char *what)
{
    GG_REQUIRE(n >= 0, GG_EINVAL, std::string(what) + ": negative n");
    GG_REQUIRE(rp && (n == 0 || (ci && v) || rp[n] == 0), GG_EINVAL, std::string(what) + ": null array");
    GG_REQUIRE(rp[0] == 0, GG_EINVAL, std::string(what) + ": row_ptr[0] != 0");
    for (int r = 0; r < n; r++) {
        GG_REQUIRE(rp[r + 1] >= rp[r], GG_EINVAL, std::string(what) + ": row_ptr not monotone");
        for (int k = rp[r]; k < rp[r + 1]; k++)
            GG_REQUIRE(ci[k] >= 0 && ci[k] < n, GG_EINVAL,
                       std::string(what) + ": column index out of range at row " + std::to_string(r));
    }
}

Csr make_csr(int n, const int *rp, const int *ci, const double *v)
{
    Csr C;
    C.n = n;
    C.rp.assign(rp, rp + n + 1);
    C.ci.assign(ci, ci + rp[n]);
    C.v.assign(v, v + rp[n]);
    return C;
}

void set_device(gg_solver *s) { GG_HIP(hipSetDevice(s->device)); }

// choose the vector space and upload A in it
// The solver's vector space.  prow / pcol (split engine): A' has row lay(j) =
// A row prow[j] and column c -> lay(pcol[c]); null: A in layout space.
// order (off the wavefront): the layout places row order[k] at slot k (RCM,
// gg_set_precond_split); natural when null
void setup_space(gg_solver *s, const Wave2D *wl, const int *prow = nullptr, const int *pcol = nullptr,
                 const std::vector<int> *order = nullptr)
{
    const int n = s->A.n;
    s->wave = wl && wl->ok;
    if (s->wave) {
        s->wl = *wl;
        s->P = wl->P;
    } else {
        s->wl = Wave2D{};
        s->P = n;
    }
    s->Ppad = round_up(std::max<long long>(s->P, 1), 512);
    s->nat2lay_h.resize(n);
    std::vector<long long> l2n(s->Ppad, -1);
    if (!s->wave && order) {
        GG_REQUIRE((int)order->size() == n, GG_EINVAL, "layout order: wrong length");
        for (int k = 0; k < n; k++) s->nat2lay_h[(*order)[k]] = k;
    }
    for (int r = 0; r < n; r++) {
        long long p = s->wave ? wl->slot(r) : order ? s->nat2lay_h[r] : r;
        s->nat2lay_h[r] = p;
        l2n[p] = r;
    }
    s->relabeled = !s->wave && order;
    s->lay2nat.upload(l2n, s->st);
    s->nat2lay.upload(s->nat2lay_h, s->st);
    s->G = reduce_grid(s->Ppad / 2);
    const char *wf = std::getenv("GG_WIDE_FORCE");     // tests: k_arnoldi_wide at any size
    if (wf && wf[0] == '1') s->G = kWideG;
    // A in layout space: row p = A row nat(p) (split: prow[nat(p)]), columns
    // remapped (split: through pcol), entry order kept
    if (!s->wave && !prow && !order) {
        Csr Ap = s->A;
        Ap.n = (int)s->P;
        s->dA.upload(Ap, s->st);
    } else {
        auto src = [&](long long p) -> long long {
            const long long r = l2n[p];
            return (r < 0 || !prow) ? r : prow[r];
        };
        Csr Ap;
        Ap.n = (int)s->P;
        Ap.rp.assign(s->P + 1, 0);
        for (long long p = 0; p < s->P; p++) {
            const long long r = src(p);
            Ap.rp[p + 1] = Ap.rp[p] + (r >= 0 ? s->A.rp[r + 1] - s->A.rp[r] : 0);
        }
        Ap.ci.resize(s->A.nnz());
        Ap.v.resize(s->A.nnz());
        for (long long p = 0; p < s->P; p++) {
            const long long r = src(p);
            if (r < 0) continue;
            int o = Ap.rp[p];
            for (int k = s->A.rp[r]; k < s->A.rp[r + 1]; k++, o++) {
                const int c = s->A.ci[k];
                Ap.ci[o] = (int)s->nat2lay_h[pcol ? pcol[c] : c];
                Ap.v[o] = s->A.v[k];
            }
        }
        s->dA.upload(Ap, s->st);
    }
    s->m_alloc = -1;   // workspace follows the space
}

void ensure_workspace(gg_solver *s, int m)
{
    if (s->m_alloc == m) return;
    const long long P = s->Ppad;
    s->V.alloc((size_t)(m + 1) * P);
    GG_HIP(hipMemsetAsync(s->V.p, 0, (size_t)(m + 1) * P * sizeof(double), s->st));
    for (DBuf<double> *b : {&s->w, &s->ww, &s->r, &s->rr, &s->bb, &s->t1, &s->t2, &s->z, &s->xv,
                            &s->bv, &s->y}) {
        b->alloc(P);
        GG_HIP(hipMemsetAsync(b->p, 0, P * sizeof(double), s->st));
    }
    s->partA.alloc(1024);
    s->partB.alloc(1024);
    {
        const char *e = std::getenv("GG_NO_PERSIST");
        const bool off = e && e[0] == '1';
        const char *wf = std::getenv("GG_WIDE_FORCE");
        const bool force_wide = wf && wf[0] == '1';
        const int pj = arnoldi_persist_units(s->G, s->Ppad);
        // (GG_MGS_GATHER 3: kXcds reducer-only blocks beside the G)
        const int xr = (mgs_gather_form() == 3 && mgs_prefetch()) ? kMgsXcds : 0;
        s->persist = !off && !force_wide && pj != 0 && s->G + xr <= arnoldi_persist_max_blocks(pj);
        s->wide = !off && !s->persist && arnoldi_wide_ok(s->G, s->Ppad);   // long vectors: w on chip
        if (s->persist || s->wide) s->gran.alloc((size_t)m * (m + 2) * (s->G + 1));
        if (s->persist) {
            s->xgran.alloc((size_t)m * (m + 2) * kMgsXcdWords);
            if (!s->elect.p) {
                s->elect.alloc(kMgsElectWords);
                GG_HIP(hipMemsetAsync(s->elect.p, 0, kMgsElectWords * sizeof(unsigned long long), s->st));
            }
        }
    }
    s->H.alloc((size_t)(m + 1) * m);
    GG_HIP(hipMemsetAsync(s->H.p, 0, (size_t)(m + 1) * m * sizeof(double), s->st));
    s->s.alloc(m + 1);
    s->cs.alloc(m + 1);
    s->sn.alloc(m + 1);
    s->ysm.alloc(m + 1);
    if (!s->ds.p) s->ds.alloc(1);
    if (!s->err.p) s->err.alloc(1);
    s->m_alloc = m;
}

int prof_begin(gg_solver *s, int kind, int i);
void prof_end(gg_solver *s, int mark);

// one triangular solve, bracketed for in-solve timing when `i` >= 0
void trsv(gg_solver *s, Gate g, DevTri &T, int kind, int i, const double *in, double *out)
{
    const int mk = i >= 0 ? prof_begin(s, kind, i) : -1;
    // a bordered forward solve forms its grid rows' heads in b (DevTri::tail)
    GG_REQUIRE(!T.tail || !T.lower || in == s->t1.p, GG_EINVAL, "bordered forward solve: input must be scratch");
    T.fast = s->div_mode;
    launch_trsv(g, T, in, out, s->err.p, s->st);
    prof_end(s, mk);
}

bool user_kind(const gg_solver *s) { return s->pkind == GG_PRECOND_USER || s->pkind == GG_PRECOND_USER_SPLIT; }

// the control block as of the work enqueued so far (host round trip)
DevState read_state(gg_solver *s)
{
    DevState h{};
    GG_HIP(hipMemcpyAsync(&h, s->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    return h;
}

// One application of the caller's operator `op` (the reference engines' calls of
// Preconditioner::DevPrecond*, src/gmres.cu:2294-2406, 2592-2690): the gate is
// evaluated on the host (the device is synchronized around the call anyway), the
// fp64 input rounded to the fp32 staging array, the callback run, its fp32
// output promoted.
void apply_user(gg_solver *s, Gate g, int op, const double *in, double *out)
{
    const int n = s->A.n;
    if (g.done || g.nit) {
        const DevState h = read_state(s);
        if ((g.done && (h.done & g.mask)) || (g.nit && g.i >= h.nit)) return;
    }
    launch_f64_to_f32(Gate{}, in, s->fin.p, n, s->st);
    GG_HIP(hipStreamSynchronize(s->st));
    const int rc = s->ufn(s->uctx, op, s->fin.p, s->fout.p, n);
    GG_HIP(hipDeviceSynchronize());
    GG_REQUIRE(rc == 0, GG_EINVAL, "user preconditioner (op " + std::to_string(op) + ") returned " +
                                       std::to_string(rc));
    launch_f32_to_f64(Gate{}, s->fout.p, out, n, s->st);
}

// ---- preconditioner operators (enqueue only; graph-capturable) ----------
void apply_minv(gg_solver *s, Gate g, const double *in, double *out, int i = -1)
{
    if (s->pkind == GG_PRECOND_USER) {
        apply_user(s, g, GG_APPLY_MINV, in, out);
        return;
    }
    if (s->pkind == GG_PRECOND_NONE) {
        Gate g2 = g;
        (void)g2;
        launch_copy(in, out, s->Ppad, s->st);   // copy is not gated: harmless
        return;
    }
    trsv(s, g, s->L, GG_PROF_TRSV_L, i, in, s->t1.p);
    trsv(s, g, s->U, GG_PROF_TRSV_U, i, s->t1.p, out);
}
// Split engine (see gg_solver): every operand in layout space.
// Ml(v) = L^-1 P_r D_l^-1 v (DevPrecond_left, src/preconditioner.cu:1592-1626),
// `in` already in A' row order (b, or nothing: the SpMV folds it, spmv_left)
void apply_left(gg_solver *s, Gate g, const double *in, double *out, int i = -1)
{
    launch_div(g, in, s->ls_l.p, s->t1.p, (int)s->P, s->st);
    trsv(s, g, s->L, GG_PROF_TRSV_L, i, s->t1.p, out);
}
// Mr(v) = D_r^-1 P_c U^-1 M v (DevPrecond_right, :1629-1657), out in the
// column convention: with the column permutation in A' the gather is gone and
// D_r^-1 is a contiguous pass (folding it into the 2D wavefront U solve's
// writer wave cost more than the pass: U 99.7 -> 142 us at C2)
void apply_right(gg_solver *s, Gate g, const double *in, double *out, int i = -1, bool t1_ready = false,
                 bool no_div = false)
{
    // t1_ready: t1 = M v already formed by the previous iteration's persistent MGS;
    // no_div: leave U^-1 M v in t2, the consumer divides by D_r per gathered term
    if (!t1_ready) launch_mul(g, in, s->mid_l.p, s->t1.p, (int)s->P, s->st);
    trsv(s, g, s->U, GG_PROF_TRSV_U, i, s->t1.p, s->t2.p);
    if (!no_div) launch_div(g, s->t2.p, s->rs_l.p, out, (int)s->P, s->st);
}
// the split engine's inner iteration folds Mr's D_r^-1 into the SpMV when A'
// has its sliced copy (GG_SPMV_XDIV=0: the separate pass, apply_right)
static bool xdiv_fold()
{
    static const bool on = [] {
        const char *e = std::getenv("GG_SPMV_XDIV");
        return !(e && e[0] == '0');
    }();
    return on;
}
// Ml(A' z) with Ml's row gather and D_l^-1 in the SpMV (resid: Ml(b - A x))
void spmv_left(gg_solver *s, Gate g, const double *z, const double *b, double *out, int i = -1,
               bool fuse = false, const double *xdiv = nullptr)
{
    if (fuse && !b) {
        // A' z and its row scaling computed inside the forward solve's launch
        // (GG_FUSE_SPMV); xdiv: z[c] / xdiv[c] per gathered term (D_r^-1 folded)
        const int mk = prof_begin(s, GG_PROF_PRECOND, i);
        const int ml = prof_begin(s, GG_PROF_TRSV_L, i);
        launch_trsv_spmv(g, s->L, s->dA, z, s->t1.p, out, s->err.p, s->st, s->ls_l.p, xdiv);
        prof_end(s, ml);
        prof_end(s, mk);
        return;
    }
    int mk = prof_begin(s, GG_PROF_SPMV, i);
    launch_spmv(g, s->dA, z, b, s->t1.p, b != nullptr, s->st, s->ls_l.p);
    prof_end(s, mk);
    mk = prof_begin(s, GG_PROF_PRECOND, i);
    trsv(s, g, s->L, GG_PROF_TRSV_L, i, s->t1.p, out);
    prof_end(s, mk);
}
// Mr^-1(x) = M^-1 U P_c^-1 D_r x (DevPrecond_starting_value, :1561-1589), x in
// the column convention
void apply_start(gg_solver *s, Gate g, const double *in, double *out)
{
    launch_mul(g, in, s->rs_l.p, s->t1.p, (int)s->P, s->st);
    launch_spmv(g, s->dUfull, s->t1.p, nullptr, s->t2.p, false, s->st);
    launch_div(g, s->t2.p, s->mid_l.p, out, (int)s->P, s->st);
}
void apply_rhs(gg_solver *s, Gate g, const double *in, double *out)
{
    if (s->pkind == GG_PRECOND_SPLIT) apply_left(s, g, in, out);
    else if (s->pkind == GG_PRECOND_USER_SPLIT) apply_user(s, g, GG_APPLY_RHS, in, out);
    else apply_minv(s, g, in, out);
}

// ---- in-solve profiling ---------------------------------------------------------
int prof_event(gg_solver *s)
{
    // slots of collected marks first (the pipelined cycle loop always has a
    // cycle's marks pending, so the pool would otherwise grow with the solve)
    int idx;
    if (!s->prof_free.empty()) {
        idx = s->prof_free.back();
        s->prof_free.pop_back();
    } else {
        if (s->prof_used == s->prof_pool.size()) {
            hipEvent_t e;
            GG_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));   // timing only
            s->prof_pool.push_back(e);
        }
        idx = (int)s->prof_used++;
    }
    GG_HIP(hipEventRecord(s->prof_pool[idx], s->st));
    return idx;
}
int prof_begin(gg_solver *s, int kind, int i)
{
    if (!((s->prof_mask >> kind) & 1)) return -1;
    s->marks.push_back({kind, i, prof_event(s), -1});
    return (int)s->marks.size() - 1;
}
void prof_end(gg_solver *s, int mark)
{
    if (mark < 0) return;
    s->marks[mark].e1 = prof_event(s);
}
// after a cycle has completed: account marks of iterations that really ran
// (the first `upto` marks -- the pipelined loop keeps the next cycle's, whose
// events are still pending; the pool is reused once no mark is left)
void prof_collect(gg_solver *s, int executed, size_t upto = (size_t)-1)
{
    if (!s->prof_mask) {
        s->marks.clear();
        s->prof_used = 0;
        s->prof_free.clear();
        return;
    }
    upto = std::min(upto, s->marks.size());
    for (size_t q = 0; q < upto; q++) {
        const auto &mk = s->marks[q];
        if (mk.i < executed && mk.e1 >= 0) {
            float ms = 0.f;
            GG_HIP(hipEventElapsedTime(&ms, s->prof_pool[mk.e0], s->prof_pool[mk.e1]));
            s->prof_ms[mk.kind] += ms;
            s->prof_cnt[mk.kind]++;
        }
        // the cycle these marks belong to has completed: their events are free
        s->prof_free.push_back(mk.e0);
        if (mk.e1 >= 0) s->prof_free.push_back(mk.e1);
    }
    s->marks.erase(s->marks.begin(), s->marks.begin() + upto);
    if (s->marks.empty()) {
        s->prof_used = 0;
        s->prof_free.clear();
    }
}

// ---- GMRES phases ------------------------------------------------------------
void enqueue_init(gg_solver *s)
{
    Gate none;
    DevState *ds = s->ds.p;
    const bool split = s->pkind == GG_PRECOND_SPLIT;
    const bool usplit = s->pkind == GG_PRECOND_USER_SPLIT;
    apply_rhs(s, none, s->bv.p, s->bb.p);                                     // bb = M b
    launch_dot(none, s->bb.p, s->bb.p, s->partA.p, s->G, s->Ppad, s->st);
    launch_set_normb(s->partA.p, s->G, ds, s->st);
    if (split) {
        apply_start(s, none, s->xv.p, s->y.p);                                 // y = Mr^-1 x0
        spmv_left(s, none, s->xv.p, s->bv.p, s->r.p);                          // r = Ml (b - A x)
    } else if (usplit) {
        apply_user(s, none, GG_APPLY_START, s->xv.p, s->y.p);                  // y = Mr^-1 x0
        launch_spmv(none, s->dA, s->xv.p, s->bv.p, s->rr.p, true, s->st);     // rr = b - A x
        apply_rhs(s, none, s->rr.p, s->r.p);                                  // r = Ml rr
    } else {
        launch_spmv(none, s->dA, s->xv.p, s->bv.p, s->rr.p, true, s->st);     // rr = b - A x
        apply_rhs(s, none, s->rr.p, s->r.p);                                  // r = M rr
    }
    launch_dot(none, s->r.p, s->r.p, s->partA.p, s->G, s->Ppad, s->st);
    launch_init_beta(s->partA.p, s->G, ds, s->hist.p, s->st);
}

// inner iteration i's sum granules (gather_h): after the m * (m+2) * G partials
unsigned long long *hgran(gg_solver *s, int m, int i)
{
    return s->gran.p + (size_t)m * (m + 2) * s->G + (size_t)i * (m + 2);
}

// The inner iteration's SpMV runs inside the forward solve's launch (FusedSpmv,
// kernels.hip) on the 2D wavefront with GG_DIV_FMA's unit L; GG_FUSE_SPMV=0 keeps
// the separate k_spmv_sell launch.  Same bits either way (the rows summed alike).
bool fuse_spmv_active(gg_solver *s)
{
    const char *e = std::getenv("GG_FUSE_SPMV");
    if (e && e[0] == '0') return false;
    if (s->shared || s->pkind == GG_PRECOND_NONE || user_kind(s)) return false;
    s->L.fast = s->div_mode;
    return fused_spmv_ok(s->L, s->dA);
}

// the padding map of the solver's vector space (kernels.h UnitMap)
UnitMap unit_map(const gg_solver *s)
{
    UnitMap um;
    const char *e = std::getenv("GG_NO_PADSKIP");           // A/B: every unit
    if (e && e[0] == '1') return um;
    if (!s->wave) {
        um.kind = 0;
        um.n = s->A.n;
        return um;
    }
    const Wave2D &w = s->wl;
    um.kind = w.tile ? 2 : 1;
    um.tbase = w.bofs / 2;                                  // bordered grid: the tail's units first
    um.tn = w.bnt;
    um.nx = w.nx;
    um.ny = w.ny;
    um.nz = w.nz;
    um.T = w.T;
    um.skew = w.skew;
    um.NJ = w.NJ;
    um.nbands = w.nbands;
    um.n = s->A.n;
    return um;
}

// diagnostics: GG_MGS_TRACE=N -- device time stamps of the N-th persistent
// orthogonalization launch (k_arnoldi_persist: per step start / h known /
// partial formed / published, for unit-block 0 and XCD 0's reducer)
long long *mgs_trace_for(gg_solver *s, int i, int m)
{
    static const long long at = [] {
        const char *e = std::getenv("GG_MGS_TRACE");
        return e ? atoll(e) : -1LL;
    }();
    if (at < 0 || (long long)s->mgs_seq + 1 != at) return nullptr;
    s->mgs_trace.alloc((size_t)2 * (m + 2) * 4);
    GG_HIP(hipMemsetAsync(s->mgs_trace.p, 0, s->mgs_trace.n * sizeof(long long), s->st));
    s->mgs_trace_i = i;
    return s->mgs_trace.p;
}
void mgs_trace_print(gg_solver *s)
{
    if (s->mgs_trace_i < 0) return;
    const int i = s->mgs_trace_i;
    std::vector<long long> h((size_t)2 * (i + 2) * 4);
    GG_HIP(hipMemcpy(h.data(), s->mgs_trace.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    for (int row = 0; row < 2; row++)
        for (int k = 0; k <= i + 1; k++) {
            const long long *t = &h[((size_t)row * (i + 2) + k) * 4];
            std::fprintf(stderr, "mgs_trace i=%d row=%d k=%d %lld %lld %lld %lld\n", i, row, k, t[0], t[1], t[2], t[3]);
        }
    s->mgs_trace_i = -1;
}

// GG_SPLIT_DIVFOLD=0: the split engine keeps k_div (Mr's D_r^-1) as its own
// launch on the fused-SpMV path
static bool divfold_on()
{
    const char *e = std::getenv("GG_SPLIT_DIVFOLD");
    return !(e && e[0] == '0');
}
// GG_FLOW_FILLFOLD=0: the flow solves fill their x themselves (own launch)
static bool fill_fold_on()
{
    const char *e = std::getenv("GG_FLOW_FILLFOLD");
    return !(e && e[0] == '0');
}
// GG_SPLIT_MULFOLD=0: the split engine keeps k_mul as its own launch
static bool mulfold_on()
{
    const char *e = std::getenv("GG_SPLIT_MULFOLD");
    return !(e && e[0] == '0');
}

// One restart cycle: its start (i0 = 0), inner iterations [i0, i1) and, with
// tail, its end (update, residual).  The default is the whole cycle; the
// transient loop enqueues a cycle's first iterations alone when the previous
// step says the solve will converge within them (solve_device_once).
void enqueue_cycle(gg_solver *s, int m, int i0 = 0, int i1 = -1, bool tail = true)
{
    if (i1 < 0) i1 = m;
    const UnitMap um = unit_map(s);
    DevState *ds = s->ds.p;
    const long long P = s->Ppad;
    const bool split = s->pkind == GG_PRECOND_SPLIT;
    const bool usplit = s->pkind == GG_PRECOND_USER_SPLIT;
    const bool user = user_kind(s);
    if (i0 == 0) launch_init_cycle(ds, s->r.p, s->V.p, s->s.p, s->G, P, s->st);
    const bool persist = s->persist && !s->shared;
    const bool wide = s->wide && !s->shared;
    // the split engine: the persistent MGS of iteration i also forms Mr's first
    // pass for iteration i + 1, t1 = M v_{i+1} (k_mul's product, one launch fewer)
    const bool mulfold = persist && split && mulfold_on();
    // the permuted split on the flow kernels (the x-division fold path): the
    // fills of the U / L solves' outputs move into the MGS / SpMV launches
    const bool xpath = split && !fuse_spmv_active(s) && s->dA.sell && xdiv_fold() &&
                       (s->U.kind == DevTri::WAVE2D || s->split_local);
    const bool lfill = xpath && fill_fold_on() && s->L.kind == DevTri::LEVEL && !s->L.tail && s->L.bofs == 0 &&
                       !s->L.lev_ptr.empty();
    const bool ufill = xpath && mulfold && fill_fold_on() && s->U.kind == DevTri::LEVEL && !s->U.tail &&
                       s->U.bofs == 0 && !s->U.lev_ptr.empty();
    if (i0 == 0 && (persist || wide)) launch_fill_u64(s->gran.p, (long long)s->gran.n, kSentinel, s->st);
    if (i0 == 0 && persist) launch_fill_u64(s->xgran.p, (long long)s->xgran.n, kSentinel, s->st);
    const bool fuse = fuse_spmv_active(s);
    for (int i = i0; i < i1; i++) {
        Gate gi;
        gi.done = &ds->done;
        gi.mask = ~0;
        gi.nit = &ds->nit;
        gi.i = i;
        double *vi = s->V.p + (long long)i * P;
        if (user) {
            // host-driven: stop enqueueing once the cycle is over (the caller's
            // operator would run on vectors nobody reads)
            const DevState h = read_state(s);
            if ((h.done & ~0) || i >= h.nit) break;
        }
        int mk;
        if (usplit) {
            apply_user(s, gi, GG_APPLY_RIGHT, vi, s->z.p);                    // z = Mr v_i
            launch_spmv(gi, s->dA, s->z.p, nullptr, s->ww.p, false, s->st);   // ww = A z
            apply_user(s, gi, GG_APPLY_LEFT, s->ww.p, s->w.p);                // w = Ml ww
        } else if (fuse && !split) {
            // ww = A v_i computed inside the forward solve's launch (GG_FUSE_SPMV)
            mk = prof_begin(s, GG_PROF_PRECOND, i);
            const int ml = prof_begin(s, GG_PROF_TRSV_L, i);
            launch_trsv_spmv(gi, s->L, s->dA, vi, s->ww.p, s->t1.p, s->err.p, s->st);
            prof_end(s, ml);
            trsv(s, gi, s->U, GG_PROF_TRSV_U, i, s->t1.p, s->w.p);              // w = M^-1 ww
            prof_end(s, mk);
        } else if (!split) {
            mk = prof_begin(s, GG_PROF_SPMV, i);
            launch_spmv(gi, s->dA, vi, nullptr, s->ww.p, false, s->st);        // ww = A v_i
            prof_end(s, mk);
            mk = prof_begin(s, GG_PROF_PRECOND, i);
            apply_minv(s, gi, s->ww.p, s->w.p, i);                             // w = M^-1 ww
            prof_end(s, mk);
        } else if (!fuse && s->dA.sell && (s->U.kind == DevTri::WAVE2D || s->split_local) && xdiv_fold()) {
            // z = Mr v_i without its last pass: D_r^-1 goes into the SpMV's
            // gathers (the same division per term, k_spmv_sell<.., XDIV>) --
            // on grid-ordered or RCM-placed factors, whose gathers are local
            // (netlist 3,595 -> 3,635 it/s; on the randomly permuted split in
            // its natural order the second gather doubled the SpMV's misses,
            // 49.8 -> 112.7 us: profiles/r04/r04p_*_x*.json)
            if (!(mulfold && i > 0)) launch_mul(gi, vi, s->mid_l.p, s->t1.p, (int)s->P, s->st);
            // flow solves' sentinel fills ride on the launch before each: the
            // previous iteration's MGS filled t2, the SpMV fills w
            s->U.prefilled = ufill && i > 0;
            trsv(s, gi, s->U, GG_PROF_TRSV_U, i, s->t1.p, s->t2.p);
            s->U.prefilled = false;
            mk = prof_begin(s, GG_PROF_SPMV, i);
            const bool sx = launch_spmv_xdiv(gi, s->dA, s->t2.p, s->rs_l.p, s->t1.p, s->st, s->ls_l.p,
                                             lfill ? s->w.p : nullptr, lfill ? s->L.lev_ptr.back() : 0);
            GG_REQUIRE(sx, GG_EINVAL, "split engine: the x-division SpMV needs A's sliced copy");
            prof_end(s, mk);
            mk = prof_begin(s, GG_PROF_PRECOND, i);
            s->L.prefilled = lfill;     // launch_spmv_xdiv performed the fill (riding or its own launch)
            trsv(s, gi, s->L, GG_PROF_TRSV_L, i, s->t1.p, s->w.p);              // w = Ml A z
            s->L.prefilled = false;
            prof_end(s, mk);
        } else {
            if (fuse && divfold_on()) {
                // D_r^-1 (Mr's last pass) in the fused SpMV's gathers: z stays U^-1 M v
                apply_right(s, gi, vi, nullptr, i, mulfold && i > 0, true);   // t2 = U^-1 M v_i
                spmv_left(s, gi, s->t2.p, nullptr, s->w.p, i, fuse, s->rs_l.p); // w = Ml A D_r^-1 t2
            } else {
                apply_right(s, gi, vi, s->z.p, i, mulfold && i > 0);          // z = Mr v_i
                spmv_left(s, gi, s->z.p, nullptr, s->w.p, i, fuse);            // w = Ml A z
            }
        }
        mk = prof_begin(s, GG_PROF_MGS, i);
        if (persist) {
            launch_arnoldi_persist(gi, i, m, ds, s->w.p, s->V.p, P, s->H.p, s->cs.p, s->sn.p, s->s.p,
                                   s->hist.p, s->gran.p + (size_t)i * (m + 2) * s->G, hgran(s, m, i), s->G,
                                   P, s->err.p, s->xgran.p + (size_t)i * (m + 2) * kMgsXcdWords, s->elect.p,
                                   ++s->mgs_seq, um, s->st, mgs_trace_for(s, i, m), mulfold ? s->mid_l.p : nullptr,
                                   mulfold ? s->t1.p : nullptr, ufill ? s->t2.p : nullptr,
                                   ufill ? s->U.lev_ptr.back() : 0);
        } else if (wide) {
            launch_arnoldi_wide(gi, i, m, ds, s->w.p, s->V.p, P, s->H.p, s->cs.p, s->sn.p, s->s.p,
                                s->hist.p, s->gran.p + (size_t)i * (m + 2) * s->G, hgran(s, m, i), s->G,
                                P, s->err.p, um, s->st);
        } else {
            double *pin = s->partA.p, *pout = s->partB.p;
            launch_dot(gi, s->w.p, s->V.p, pin, s->G, P, s->st);               // <w, v_0>
            for (int k = 0; k <= i; k++) {
                const double *vk = s->V.p + (long long)k * P;
                const double *vn = (k < i) ? s->V.p + (long long)(k + 1) * P : s->w.p;
                launch_mgs_step(gi, i, k, m, s->w.p, vk, vn, pin, pout, s->H.p, s->G, P, s->st);
                std::swap(pin, pout);
            }
            launch_arnoldi_finalize(gi, i, m, ds, pin, s->G, s->w.p,
                                    s->V.p + (long long)(i + 1) * P, s->H.p, s->cs.p, s->sn.p,
                                    s->s.p, s->hist.p, P, s->st);
        }
        prof_end(s, mk);
    }
    if (!tail) return;
    Gate gu;
    gu.done = &ds->done;
    gu.mask = DONE_RESTART | DONE_INIT | DONE_ABORT | DONE_FINAL | DONE_EXH;
    launch_update(gu, m, ds, s->H.p, s->s.p, s->ysm.p, s->V.p, P, split || usplit ? s->y.p : s->xv.p, s->G, P,
                  s->st, um);
    if (split) apply_right(s, gu, s->y.p, s->xv.p);                            // x = Mr y
    if (usplit) apply_user(s, gu, GG_APPLY_RIGHT, s->y.p, s->xv.p);
    Gate gr;
    gr.done = &ds->done;
    gr.mask = ~0;
    if (split) {
        spmv_left(s, gr, s->xv.p, s->bv.p, s->r.p);                            // r = Ml (b - A x)
    } else {
        launch_spmv(gr, s->dA, s->xv.p, s->bv.p, s->rr.p, true, s->st);       // rr = b - A x
        apply_rhs(s, gr, s->rr.p, s->r.p);
    }
    launch_dot(gr, s->r.p, s->r.p, s->partA.p, s->G, P, s->st);
    launch_end_cycle(s->partA.p, s->G, ds, s->hist.p, s->st);
}


// re-arm a wavefront triangle's hand-off state (granules, 3D progress words)
void reset_wave(DevTri *T, hipStream_t st)
{
    launch_fill_u64(T->bnd.p, T->wl.ngran(), kSentinel, st);
    if (T->wl.tile)     // the tile kernel's task queue (a launch cut short would leave it armed)
        GG_HIP(hipMemsetAsync(T->bnd.p + T->wl.ngran() + 128LL * kTileDummyBlocks, 0, 64 * sizeof(unsigned long long), st));
    if (T->fcnt.p) GG_HIP(hipMemsetAsync(T->fcnt.p, 0, T->fcnt.n * sizeof(unsigned long long), st));
    if (T->prog.p) GG_HIP(hipMemsetAsync(T->prog.p, 0, T->prog.n * sizeof(unsigned long long), st));
}

// Device error word: bit 0 = wavefront boundary wait timed out, bit 1 = a
// WD_RCP step saw a numerator outside its safe range (repeat with WD_HW), bit
// 3 = a statically dealt tile grid was not co-resident (repeat with the tile
// queue, k_trsv_tile3d).  Bits 1 and 3 throw Fallback: the caller applies it
// (apply_fallback) and repeats the solve / apply.
struct Fallback {
    int bits;
};
void check_err(gg_solver *s)
{
    // on the solver's stream: a plain hipMemcpy would not wait for its kernels
    int err = 0;
    GG_HIP(hipMemcpyAsync(&err, s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    if (err & 8) throw Fallback{err};              // (the residency timeout also left garbage)
    GG_REQUIRE((err & 1) == 0, GG_ETIMEOUT, "wavefront triangular solve: boundary wait timed out");
    if (err & 2) throw Fallback{err};
}
// the control block and the error word in one round trip (after a cycle)
DevState read_state_checked(gg_solver *s)
{
    if (!s->h_state) {
        GG_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_state), sizeof(DevState), hipHostMallocDefault));
        GG_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_err), sizeof(int), hipHostMallocDefault));
    }
    GG_HIP(hipMemcpyAsync(s->h_state, s->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipMemcpyAsync(s->h_err, s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    const int err = *s->h_err;
    if (err & 8) throw Fallback{err};
    GG_REQUIRE((err & 1) == 0, GG_ETIMEOUT, "wavefront triangular solve: boundary wait timed out");
    if (err & 2) throw Fallback{err};
    return *s->h_state;
}
// for the rest of the solver's life: every WD_RCP triangle divides (bit 1),
// every 3D tile triangle claims its tiles from the queue (bit 3)
void apply_fallback(gg_solver *s, const Fallback &f)
{
    for (DevTri *T : {&s->L, &s->U}) {
        if ((f.bits & 2) && T->kind == DevTri::WAVE2D && T->div == WD_RCP) T->div = WD_HW;
        if ((f.bits & 8) && T->kind == DevTri::WAVE2D && T->wl.tile) T->tile_queue = true;
    }
}

// A persistent orthogonalization grid that was not co-resident aborted the
// cycle (DONE_ABORT, kernels.hip gather_first): everything after the abort
// point was gated off and x, r, j, hist_len are as before the cycle.  Restore
// the control block (done = 0, resid = beta / normb as k_init_beta /
// k_end_cycle left it), drop the persistent kernels for the solver's life and
// run the cycle again on the per-step kernels (the same reduction tree: the
// same bits).  Returns the state after the cycle.
DevState rerun_aborted_cycle(gg_solver *s, int m, DevState h)
{
    s->persist = false;
    s->wide = false;
    s->resid_fallbacks++;
    prof_collect(s, 0);                 // the aborted cycle's marks
    h.done = 0;
    h.resid = h.beta / h.normb;
    GG_HIP(hipMemcpyAsync(s->ds.p, &h, sizeof(DevState), hipMemcpyHostToDevice, s->st));
    enqueue_cycle(s, m);
    h = read_state_checked(s);
    GG_REQUIRE((h.done & DONE_ABORT) == 0, GG_EHIP, "gg_solve: per-step cycle aborted");
    return h;
}

int solve_device_once(gg_solver *s, const double *d_b, double *d_x, const gg_options *opt,
                 gg_result *res)
{
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_solve: no matrix (call gg_set_matrix)");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "gg_solve: no preconditioner (call gg_set_precond_*)");
    GG_REQUIRE(opt, GG_EINVAL, "gg_solve: null options");
    const int m = opt->restart;
    GG_REQUIRE(m >= 1 && m <= 512, GG_EINVAL, "gg_solve: restart must be in [1, 512]");
    GG_REQUIRE(opt->max_iter >= 0, GG_EINVAL, "gg_solve: negative max_iter");
    GG_REQUIRE((opt->flags & ~GG_SOLVE_SHARED_DEVICE) == 0, GG_EINVAL,
               (opt->flags & GG_SOLVE_CGS2) ? "gg_solve: GG_SOLVE_CGS2 is a sharded-solve (gg_dd_solve) mode"
                                            : "gg_solve: unknown flags");
    s->shared = (opt->flags & GG_SOLVE_SHARED_DEVICE) != 0;
    if (s->shared) {
        // only kernels whose workgroups wait on earlier-dispatched ones
        bool ok = s->pkind == GG_PRECOND_NONE;
        if (s->pkind != GG_PRECOND_SPLIT && s->pkind != GG_PRECOND_NONE)
            ok = s->L.kind == DevTri::WAVE2D && s->U.kind == DevTri::WAVE2D && s->L.wl.nz == 1;
        GG_REQUIRE(ok, GG_EINVAL, "gg_solve: GG_SOLVE_SHARED_DEVICE needs the 2D wavefront path "
                                  "(or no preconditioner)");
    }
    const int n = s->A.n;
    set_device(s);
    ensure_workspace(s, m);
    const long long need = (long long)opt->max_iter + opt->max_iter / m + 4;
    if (need > s->hist_cap) {
        s->hist.alloc(need);
        s->hist_cap = need;
    }
    // inputs into the solver's vector space (split: b in A' row order, x in
    // the column convention)
    const bool split = s->pkind == GG_PRECOND_SPLIT;
    launch_gather(d_b, split ? s->sb_map.p : s->lay2nat.p, s->bv.p, s->Ppad, s->st);
    launch_gather(d_x, split ? s->sx_map.p : s->lay2nat.p, s->xv.p, s->Ppad, s->st);
    if (split || s->pkind == GG_PRECOND_USER_SPLIT)
        GG_HIP(hipMemsetAsync(s->y.p, 0, s->Ppad * sizeof(double), s->st));
    for (DevTri *T : {&s->L, &s->U})
        if (T->kind == DevTri::WAVE2D)
            reset_wave(T, s->st);
    DevState h{};
    h.tol = opt->tol;
    h.max_iter = opt->max_iter;
    h.m = m;
    h.j = 1;
    GG_HIP(hipMemcpyAsync(s->ds.p, &h, sizeof(DevState), hipMemcpyHostToDevice, s->st));
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));

    GG_HIP(hipEventRecord(s->ev0, s->st));
    enqueue_init(s);
    int ret = 1, iters = 0, inner = 0, restarts = 0;
    long long hist_len = 1;
    double relres = 0.0;
    // Pipelined cycles (GG_CYCLE_PIPE, default on): cycle c+1 is enqueued before
    // the state after cycle c is read, so the device never waits for the host's
    // round trip between restart cycles (C2: ~59 us a cycle).  The cycle behind
    // the last one runs gated off (DONE_* bits: its init, Arnoldi, update and
    // residual do nothing).  Host-driven operators (user plug-ins) keep one cycle
    // at a time.
    const char *pe = std::getenv("GG_CYCLE_PIPE");
    const bool pipe = !(pe && pe[0] == '0') && !user_kind(s) && opt->max_iter >= 1;
    if (pipe) {
        for (int k = 0; k < 2; k++)
            if (!s->p_state[k]) {
                GG_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->p_state[k]), sizeof(DevState), hipHostMallocDefault));
                GG_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->p_err[k]), sizeof(int), hipHostMallocDefault));
                GG_HIP(hipEventCreateWithFlags(&s->p_ev[k], hipEventDisableTiming));
            }
        s->mark_ends.clear();
        auto enqueue = [&](int slot) {          // one cycle and the read of the state after it
            enqueue_cycle(s, m);
            s->mark_ends.push_back(s->marks.size());
            GG_HIP(hipMemcpyAsync(s->p_state[slot], s->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipMemcpyAsync(s->p_err[slot], s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipEventRecord(s->p_ev[slot], s->st));
        };
        auto collect = [&](int executed) {      // the oldest enqueued cycle's marks
            const size_t upto = s->mark_ends.empty() ? s->marks.size() : s->mark_ends.front();
            prof_collect(s, executed, upto);
            if (!s->mark_ends.empty()) {
                s->mark_ends.erase(s->mark_ends.begin());
                for (size_t &e : s->mark_ends) e -= upto;
            }
        };
        auto drain = [&]() {                    // the speculative cycle behind the last (gated off)
            GG_HIP(hipStreamSynchronize(s->st));
            while (!s->mark_ends.empty()) collect(0);
            prof_collect(s, 0);
        };
        // cycle 1 is gated on DONE_INIT (converged at the start) like the rest.
        // The transient loop's hint (the previous step's inner iterations, h):
        // cycle 1's first h + 2 iterations go in alone and their state is read;
        // when the solve converged in them only the cycle's end follows, else
        // the rest of the cycle and cycle 2 -- the launches a converged step
        // would have run gated off (up to 2m - h iterations' worth, each a
        // launch that reads its gate and returns) are never enqueued.  The
        // kernels that do run are the same, in the same order: the same bits.
        const int hint = s->iter_hint;
        if (hint > 0 && hint + 2 < m) {
            const int K = hint + 2;
            enqueue_cycle(s, m, 0, K, false);
            GG_HIP(hipMemcpyAsync(s->p_state[0], s->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipMemcpyAsync(s->p_err[0], s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipEventRecord(s->p_ev[0], s->st));
            GG_HIP(hipEventSynchronize(s->p_ev[0]));
            const DevState hp = *s->p_state[0];
            const bool conv = *s->p_err[0] == 0 && (hp.done & (DONE_INIT | DONE_INNER)) != 0 &&
                              (hp.done & DONE_ABORT) == 0;
            enqueue_cycle(s, m, conv ? m : K, m, true);
            s->mark_ends.push_back(s->marks.size());
            GG_HIP(hipMemcpyAsync(s->p_state[0], s->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipMemcpyAsync(s->p_err[0], s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
            GG_HIP(hipEventRecord(s->p_ev[0], s->st));
            if (!conv) enqueue(1);
        } else {
            enqueue(0);
            enqueue(1);
        }
        int cur = 0;
        DevState prev{};
        prev.j = 1;
        prev.hist_len = 1;
        while (true) {
            GG_HIP(hipEventSynchronize(s->p_ev[cur]));
            const int err = *s->p_err[cur];
            DevState h = *s->p_state[cur];
            if (err & 8) {
                drain();
                throw Fallback{err};
            }
            if (err & 1) {
                drain();
                GG_REQUIRE(false, GG_ETIMEOUT, "wavefront triangular solve: boundary wait timed out");
            }
            if (err & 2) {
                drain();
                throw Fallback{err};
            }
            if (h.done & DONE_ABORT) {
                // this cycle aborted, the one behind it ran gated off: rerun this
                // one on the per-step kernels, then refill the pipeline
                drain();
                h = rerun_aborted_cycle(s, m, h);
                prof_collect(s, (h.done & DONE_INNER) ? h.conv_i + 1 : h.nit);   // the rerun's marks
                s->mark_ends.clear();
                enqueue(cur ^ 1);
            } else {
                collect((h.done & DONE_INNER) ? h.conv_i + 1 : (h.done & DONE_INIT) ? 0 : h.nit);
            }
            relres = h.resid;
            if (h.done & DONE_INIT) {
                ret = 0;
                iters = 0;
                hist_len = 1;
                break;
            }
            restarts++;
            if (h.done & DONE_INNER) {
                ret = 0;
                iters = prev.j + h.conv_i;
                inner += h.conv_i + 1;
                hist_len = h.hist_len + h.conv_i + 1;
                break;
            }
            inner += h.nit;
            hist_len = h.hist_len;
            if (h.done & DONE_RESTART) {
                ret = 0;
                iters = h.j;
                break;
            }
            if (h.j > opt->max_iter) {          // while (j <= *max_iter) exhausted
                ret = 1;
                iters = opt->max_iter;          // the reference leaves *max_iter untouched
                break;
            }
            prev = h;
            enqueue(cur);                       // the cycle after the one in flight
            cur ^= 1;
        }
        drain();
    } else {
    // The first cycle goes in before the state after the initial residual is
    // read: its kernels are gated on DONE_INIT (converged at the start), so a
    // solve costs one host round trip less.  The state after init is j = 1,
    // hist_len = 1 (k_init_beta).
    bool first = opt->max_iter >= 1;
    if (first) enqueue_cycle(s, m);
    DevState h = read_state_checked(s);
    if (first && (h.done & DONE_ABORT)) h = rerun_aborted_cycle(s, m, h);
    relres = h.resid;
    if (h.done & DONE_INIT) {
        ret = 0;
        iters = 0;
        if (first) prof_collect(s, 0);
    } else {
        DevState prev = h;
        prev.j = 1;
        prev.hist_len = 1;
        if (!first) h = prev;
        while (true) {
            if (first) {
                first = false;               // cycle 1: enqueued and read above
                restarts++;
            } else {
                if (h.j > opt->max_iter) {   // while (j <= *max_iter) exhausted
                    ret = 1;
                    relres = h.resid;
                    iters = opt->max_iter;   // the reference leaves *max_iter untouched
                    hist_len = h.hist_len;
                    break;
                }
                restarts++;
                enqueue_cycle(s, m);
                prev = h;
                h = read_state_checked(s);
                if (h.done & DONE_ABORT) h = rerun_aborted_cycle(s, m, h);
            }
            prof_collect(s, (h.done & DONE_INNER) ? h.conv_i + 1 : h.nit);
            if (h.done & DONE_INNER) {
                ret = 0;
                iters = prev.j + h.conv_i;
                inner += h.conv_i + 1;
                relres = h.resid;
                hist_len = h.hist_len + h.conv_i + 1;
                break;
            }
            inner += h.nit;
            if (h.done & DONE_RESTART) {
                ret = 0;
                iters = h.j;
                relres = h.resid;
                hist_len = h.hist_len;
                break;
            }
            hist_len = h.hist_len;
            relres = h.resid;
        }
    }
    }
    GG_HIP(hipEventRecord(s->ev1, s->st));
    check_err(s);
    mgs_trace_print(s);
    launch_gather(s->xv.p, split ? s->sx_out.p : s->nat2lay.p, d_x, n, s->st);
    GG_HIP(hipStreamSynchronize(s->st));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_hist.resize(hist_len);
    if (hist_len)
        GG_HIP(hipMemcpy(s->last_hist.data(), s->hist.p, hist_len * sizeof(double),
                         hipMemcpyDeviceToHost));
    if (res) {
        res->status = ret;
        res->iters = iters;
        res->inner_iters = inner;
        res->restarts = restarts;
        res->relres = relres;
        res->solve_ms = ms;
    }
    return ret;
}

int solve_device(gg_solver *s, const double *d_b, double *d_x, const gg_options *opt,
                 gg_result *res)
{
    // d_x is written only at the very end, so a fallback simply starts over
    // (each fallback at most once: the bits it applies do not come back)
    for (int attempt = 0;; attempt++) {
        try {
            return solve_device_once(s, d_b, d_x, opt, res);
        } catch (Fallback &f) {
            if (attempt >= 2) throw Error{GG_EHIP, "gg_solve: fallbacks exhausted"};
            apply_fallback(s, f);
        }
    }
}

void stage_in(gg_solver *s, const double *h, DBuf<double> &d)
{
    const int n = s->A.n;
    if (d.n < (size_t)std::max(n, 1)) d.alloc(std::max(n, 1));
    if (n) GG_HIP(hipMemcpyAsync(d.p, h, n * sizeof(double), hipMemcpyHostToDevice, s->st));
}
void stage_out(gg_solver *s, const DBuf<double> &d, double *h)
{
    const int n = s->A.n;
    if (n) GG_HIP(hipMemcpyAsync(h, d.p, n * sizeof(double), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
}

}  // namespace

// for the many-RHS driver (batch.hip, gg_solver.h)
namespace gg {
int solve_one(gg_solver *s, const double *d_b, double *d_x, const gg_options *opt, gg_result *res)
{
    return solve_device(s, d_b, d_x, opt, res);
}
UnitMap solver_unit_map(const gg_solver *s) { return unit_map(s); }
}  // namespace gg

// ======================================================================= C ABI
extern "C" {

int gg_abi_version(void) { return GG_ABI_VERSION; }

const char *gg_strerror(int status)
{
    switch (status) {
    case GG_OK: return "converged";
    case GG_NOT_CONVERGED: return "not converged";
    case GG_EINVAL: return "invalid argument";
    case GG_EHIP: return "HIP runtime error";
    case GG_EZEROPIVOT: return "zero pivot in factorization";
    case GG_ENOMEM: return "out of memory";
    case GG_ESTATE: return "invalid call order";
    case GG_ETIMEOUT: return "device wait timed out";
    case GG_ECOMM: return "communication error";
    default: return "unknown status";
    }
}

const char *gg_last_error(void) { return g_last_error.c_str(); }

int gg_device_count(int *count)
{
    GG_API_BEGIN
    GG_REQUIRE(count, GG_EINVAL, "null count");
    int c = 0;
    GG_HIP(hipGetDeviceCount(&c));
    *count = c;
    return GG_OK;
    GG_API_END
}

int gg_create(int device, gg_solver **out)
{
    GG_API_BEGIN
    GG_REQUIRE(out, GG_EINVAL, "null out");
    std::unique_ptr<gg_solver> s(new gg_solver());
    s->device = device;
    set_device(s.get());
    GG_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    GG_HIP(hipEventCreate(&s->ev0));
    GG_HIP(hipEventCreate(&s->ev1));
    *out = s.release();
    return GG_OK;
    GG_API_END
}

int gg_destroy(gg_solver *s)
{
    if (!s) return GG_OK;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    for (hipEvent_t e : s->prof_pool) (void)hipEventDestroy(e);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    gg::batch_release(s);
    if (s->h_state) (void)hipHostFree(s->h_state);
    if (s->h_err) (void)hipHostFree(s->h_err);
    for (int k = 0; k < 2; k++) {
        if (s->p_state[k]) (void)hipHostFree(s->p_state[k]);
        if (s->p_err[k]) (void)hipHostFree(s->p_err[k]);
        if (s->p_ev[k]) (void)hipEventDestroy(s->p_ev[k]);
    }
    hipStream_t st = s->st;
    delete s;
    if (st) (void)hipStreamDestroy(st);
    return GG_OK;
}

static std::atomic<long long> g_set_matrix_calls{0};
long long gg_set_matrix_count(void) { return g_set_matrix_calls.load(); }

int gg_set_matrix(gg_solver *s, int n, const int *row_ptr, const int *col_idx, const double *val)
{
    GG_API_BEGIN
    GG_REQUIRE(s, GG_EINVAL, "null solver");
    g_set_matrix_calls++;
    check_csr(n, row_ptr, col_idx, val, "A");
    set_device(s);
    s->A = make_csr(n, row_ptr, col_idx, val);
    s->have_A = true;
    s->pkind = -1;
    s->L.kind = s->U.kind = DevTri::NONE;
    return GG_OK;
    GG_API_END
}

int gg_set_precond_none(gg_solver *s)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    set_device(s);
    setup_space(s, nullptr);
    s->L.kind = s->U.kind = DevTri::NONE;
    s->pkind = GG_PRECOND_NONE;
    GG_HIP(hipStreamSynchronize(s->st));
    return GG_OK;
    GG_API_END
}

static void setup_left(gg_solver *s, const Csr &Lf, const Csr &Uf, int kind)
{
    CanonTri cl = canon_lower_unit(Lf);
    CanonTri cu = canon_upper_ignorezero(Uf);
    Wave2D wl;
    const char *env = std::getenv("GG_NO_WAVEFRONT");
    if (!(env && env[0] == '1')) {
        wl = detect_wave2d(cl, cu);
        if (wl.ok && wl.nbands > 512) wl.ok = false;   // every band must be co-resident
        const char *e3 = std::getenv("GG_NO_WAVE3D");
        if (!wl.ok && !(e3 && e3[0] == '1')) wl = detect_wave3d(cl, cu);
    }
    setup_space(s, &wl);
    build_tri(s->L, cl, &wl, &s->nat2lay_h, s->Ppad, s->st);
    build_tri(s->U, cu, &wl, &s->nat2lay_h, s->Ppad, s->st);
    s->pkind = kind;
    GG_HIP(hipStreamSynchronize(s->st));
}

int gg_set_precond_ilu0(gg_solver *s)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    set_device(s);
    Csr Lf, Uf;
    ilu0_left(s->A, Lf, Uf);
    setup_left(s, Lf, Uf, GG_PRECOND_ILU0);
    return GG_OK;
    GG_API_END
}

// ILU(0) numeric factorization on the device (k_ilu0_columns): the factored
// matrix in A's CSR order, bit-identical to ilu0_left before its split.  The
// CSC pattern and position maps are built on the host (O(nnz)), as leftILU
// builds its CSC and level lists on the host before its device kernels.
void ilu0_device_values(gg_solver *s, std::vector<double> &fv, double *ms)
{
    const Csr &A = s->A;
    const int n = A.n, nnz = A.rp[n];
    std::vector<int> cp, ri;
    std::vector<long long> c2r, r2c;
    csc_pattern(A, cp, ri, c2r, r2c);
    DBuf<int> dcp, dri, dlev, ddone;
    DBuf<long long> dc2r, dr2c;
    DBuf<double> dv, dcv0, dcv, dout;
    dcp.upload(cp, s->st);
    dri.upload(ri, s->st);
    dc2r.upload(c2r, s->st);
    dr2c.upload(r2c, s->st);
    dv.upload(A.v, s->st);
    dcv0.alloc(nnz);
    dcv.alloc(nnz);
    dout.alloc(nnz);
    dlev.alloc(n);
    ddone.alloc(n);
    if (!s->err.p) s->err.alloc(1);
    GG_HIP(hipMemsetAsync(dlev.p, 0xFF, (size_t)n * sizeof(int), s->st));     // level -1: not known
    GG_HIP(hipMemsetAsync(ddone.p, 0, (size_t)n * sizeof(int), s->st));
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));
    const int maxb = ilu0_columns_max_blocks();
    GG_REQUIRE(maxb > 0, GG_EHIP, "ILU(0) device: occupancy query failed");
    const long long need = ((long long)n + kBlock - 1) / kBlock;
    const int blocks = (int)std::max<long long>(1, std::min<long long>(maxb, need));
    GG_HIP(hipEventRecord(s->ev0, s->st));
    launch_gather(dv.p, dc2r.p, dcv0.p, nnz, s->st);
    launch_gather(dv.p, dc2r.p, dcv.p, nnz, s->st);
    launch_ilu0_columns(n, dcp.p, dri.p, dcv0.p, dcv.p, dlev.p, ddone.p, s->err.p, blocks, s->st);
    launch_gather(dcv.p, dr2c.p, dout.p, nnz, s->st);
    GG_HIP(hipEventRecord(s->ev1, s->st));
    fv.resize(nnz);
    GG_HIP(hipMemcpyAsync(fv.data(), dout.p, (size_t)nnz * sizeof(double), hipMemcpyDeviceToHost, s->st));
    int err = 0;
    GG_HIP(hipMemcpyAsync(&err, s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    GG_REQUIRE(err == 0, GG_ETIMEOUT, "ILU(0) device: a column wait timed out");
    float t = 0.f;
    GG_HIP(hipEventElapsedTime(&t, s->ev0, s->ev1));
    if (ms) *ms = t;
}

int gg_ilu0_device_values(gg_solver *s, double *val, double *ms)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A && val, GG_ESTATE, "gg_ilu0_device_values: call gg_set_matrix first");
    set_device(s);
    std::vector<double> fv;
    ilu0_device_values(s, fv, ms);
    std::copy(fv.begin(), fv.end(), val);
    return GG_OK;
    GG_API_END
}

int gg_set_precond_ilu0_device(gg_solver *s)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    set_device(s);
    Csr F;
    F.n = s->A.n;
    F.rp = s->A.rp;
    F.ci = s->A.ci;
    ilu0_device_values(s, F.v, nullptr);
    Csr Lf, Uf;
    split_lu_drop(F, Lf, Uf);
    setup_left(s, Lf, Uf, GG_PRECOND_ILU0);
    return GG_OK;
    GG_API_END
}

// ILU(k) with the numeric phase on the device (k_iluk_wave): the pattern on
// the host (iluk_pattern: row-parallel for k = 1, lofC for k >= 2; the
// reference runs lofC on the host too), A's values scattered into it and the
// rows factored on the device, the factors emitted in iluk_itsol's forms;
// bit-identical to iluk_itsol.  Host threads: GG_HOST_THREADS (default: the
// hardware threads, at most 16).
void iluk_device_factor(gg_solver *s, int level, Csr &L, Csr &U, double *ms)
{
    const Csr &A = s->A;
    const int n = A.n;
    static const int threads = [] {
        const char *e = std::getenv("GG_HOST_THREADS");
        const int hw = (int)std::thread::hardware_concurrency();
        return e ? std::max(1, atoi(e)) : std::max(1, std::min(hw, 16));
    }();
    std::vector<long long> prow;
    std::vector<int> nl, pcol;
    iluk_pattern(A, level, threads, prow, nl, pcol);
    const long long np = prow[n];
    // rows of more than the kernel's LDS capacity take the long-row path
    // (GG_ILUK_LONG: a lower threshold, to exercise that path on small systems)
    const char *lg = std::getenv("GG_ILUK_LONG");
    const int cap = lg ? std::max(0, std::min(iluk_wave_cap(), atoi(lg))) : iluk_wave_cap();
    std::vector<int> rshort, rlong;
    for (int i = 0; i < n; i++) (prow[i + 1] - prow[i] > cap ? rlong : rshort).push_back(i);
    const int maxb = iluk_wave_max_blocks();
    GG_REQUIRE(maxb > 1, GG_EHIP, "ILU(k) device: occupancy query failed");
    const int wpb = kBlock / 64;
    int long_blocks = 0;
    if (!rlong.empty()) {
        // long-row waves: the long rows' share of the entries, at most half
        // the grid and 16 GiB of position maps (n ints per wave)
        long long long_nnz = 0;
        for (int i : rlong) long_nnz += prow[i + 1] - prow[i];
        const long long want = std::max<long long>(1, (long long)((double)maxb * long_nnz / std::max<long long>(np, 1)));
        const long long by_mem = std::max<long long>(1, (16LL << 30) / ((long long)wpb * n * (long long)sizeof(int)));
        long_blocks = (int)std::min<long long>({want, std::max(1, maxb / 2), by_mem,
                                                (long long)(rlong.size() + wpb - 1) / wpb});
    }
    const int short_blocks = (int)std::min<long long>(maxb - long_blocks, std::max<long long>(1, ((long long)rshort.size() + wpb - 1) / wpb));
    const int blocks = long_blocks + (rshort.empty() ? 0 : short_blocks);
    DBuf<long long> dprow;
    DBuf<int> dnl, dpcol, ddone, drs, drl, darp, daci, dscr;
    DBuf<double> dav, dval, ddinv;
    dprow.upload(prow, s->st);
    dnl.upload(nl, s->st);
    dpcol.upload(pcol, s->st);
    darp.upload(A.rp, s->st);
    daci.upload(A.ci, s->st);
    dav.upload(A.v, s->st);
    drs.upload(rshort, s->st);
    drl.upload(rlong, s->st);
    dval.alloc(np);
    ddinv.alloc(n);
    ddone.alloc(n);
    dscr.alloc((size_t)std::max(long_blocks, 1) * wpb * (rlong.empty() ? 1 : (size_t)n));
    if (!s->err.p) s->err.alloc(1);
    GG_HIP(hipMemsetAsync(dval.p, 0, (size_t)np * sizeof(double), s->st));
    GG_HIP(hipMemsetAsync(ddone.p, 0, (size_t)n * sizeof(int), s->st));
    GG_HIP(hipMemsetAsync(dscr.p, 0xFF, dscr.n * sizeof(int), s->st));
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));
    GG_HIP(hipEventRecord(s->ev0, s->st));
    launch_iluk_scatter(n, darp.p, daci.p, dav.p, dprow.p, dpcol.p, dval.p, s->st);   // fill = 0
    launch_iluk_wave(n, dprow.p, dnl.p, dpcol.p, dval.p, ddinv.p, ddone.p, drs.p, (int)rshort.size(), drl.p,
                     (int)rlong.size(), long_blocks, dscr.p, s->err.p, blocks, s->st);
    GG_HIP(hipEventRecord(s->ev1, s->st));
    std::vector<double> val(np);
    GG_HIP(hipMemcpyAsync(val.data(), dval.p, (size_t)np * sizeof(double), hipMemcpyDeviceToHost, s->st));
    int err = 0;
    GG_HIP(hipMemcpyAsync(&err, s->err.p, sizeof(int), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    GG_REQUIRE((err & 1) == 0, GG_ETIMEOUT, "ILU(k) device: a row wait timed out");
    GG_REQUIRE((err & 2) == 0, GG_EZEROPIVOT, "ILU(k): zero pivot (src/iluk.cpp:175-185)");
    float t = 0.f;
    GG_HIP(hipEventElapsedTime(&t, s->ev0, s->ev1));
    if (ms) *ms = t;
    iluk_emit_flat(n, prow, nl, pcol, val, L, U);
}

int gg_set_precond_iluk_device(gg_solver *s, int level)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    GG_REQUIRE(level >= 0, GG_EINVAL, "ILU(k): negative level");
    set_device(s);
    Csr Lf, Uf;
    iluk_device_factor(s, level, Lf, Uf, nullptr);
    setup_left(s, Lf, Uf, GG_PRECOND_ILUK);
    return GG_OK;
    GG_API_END
}

int gg_iluk_device_factors(gg_solver *s, int level, int *l_row_ptr, int **l_col_idx, double **l_val,
                           int *u_row_ptr, int **u_col_idx, double **u_val, double *ms)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "gg_iluk_device_factors: call gg_set_matrix first");
    GG_REQUIRE(level >= 0, GG_EINVAL, "ILU(k): negative level");
    GG_REQUIRE(l_row_ptr && l_col_idx && l_val && u_row_ptr && u_col_idx && u_val, GG_EINVAL,
               "gg_iluk_device_factors: null output");
    set_device(s);
    Csr Lf, Uf;
    iluk_device_factor(s, level, Lf, Uf, ms);
    auto out = [](const Csr &F, int *rp, int **ci, double **v) {
        std::copy(F.rp.begin(), F.rp.end(), rp);
        const size_t nz = F.ci.size();
        *ci = static_cast<int *>(std::malloc(std::max<size_t>(nz, 1) * sizeof(int)));
        *v = static_cast<double *>(std::malloc(std::max<size_t>(nz, 1) * sizeof(double)));
        GG_REQUIRE(*ci && *v, GG_ENOMEM, "gg_iluk_device_factors: out of host memory");
        std::copy(F.ci.begin(), F.ci.end(), *ci);
        std::copy(F.v.begin(), F.v.end(), *v);
    };
    out(Lf, l_row_ptr, l_col_idx, l_val);
    out(Uf, u_row_ptr, u_col_idx, u_val);
    return GG_OK;
    GG_API_END
}

int gg_set_precond_iluk(gg_solver *s, int level)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    GG_REQUIRE(level >= 0, GG_EINVAL, "ILU(k): negative level");
    set_device(s);
    Csr Lf, Uf;
    int rc = iluk_itsol(s->A, level, Lf, Uf);
    GG_REQUIRE(rc == 0, GG_EZEROPIVOT, "ILU(k): zero pivot (src/iluk.cpp:175-185)");
    setup_left(s, Lf, Uf, GG_PRECOND_ILUK);
    return GG_OK;
    GG_API_END
}

int gg_set_precond_lu(gg_solver *s, const int *l_rp, const int *l_ci, const double *l_v,
                      const int *u_rp, const int *u_ci, const double *u_v)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    const int n = s->A.n;
    check_csr(n, l_rp, l_ci, l_v, "L");
    check_csr(n, u_rp, u_ci, u_v, "U");
    set_device(s);
    setup_left(s, make_csr(n, l_rp, l_ci, l_v), make_csr(n, u_rp, u_ci, u_v), GG_PRECOND_LU);
    return GG_OK;
    GG_API_END
}

int gg_set_precond_split(gg_solver *s, const int *l_rp, const int *l_ci, const double *l_v,
                         const int *u_rp, const int *u_ci, const double *u_v, const double *middle,
                         const int *perm_row, const int *perm_col, const double *lscale,
                         const double *rscale)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    const int n = s->A.n;
    check_csr(n, l_rp, l_ci, l_v, "L");
    check_csr(n, u_rp, u_ci, u_v, "U");
    GG_REQUIRE(middle && perm_row && perm_col && lscale && rscale, GG_EINVAL, "split: null vector");
    for (int i = 0; i < n; i++)
        GG_REQUIRE(perm_row[i] >= 0 && perm_row[i] < n && perm_col[i] >= 0 && perm_col[i] < n,
                   GG_EINVAL, "split: permutation index out of range");
    std::vector<int> pcinv(n, -1), prinv(n, -1);
    for (int i = 0; i < n; i++) {
        GG_REQUIRE(pcinv[perm_col[i]] < 0 && prinv[perm_row[i]] < 0, GG_EINVAL,
                   "split: perm_row / perm_col is not a permutation");
        pcinv[perm_col[i]] = i;
        prinv[perm_row[i]] = i;
    }
    set_device(s);
    Csr Lf = make_csr(n, l_rp, l_ci, l_v), Uf = make_csr(n, u_rp, u_ci, u_v);
    CanonTri cl = canon_lower_lastdiag(Lf);
    CanonTri cu = canon_upper_firstdiag(Uf);
    // grid-shaped factors (the split of a 5-point grid in natural order) take
    // the 2D wavefront: L rows ascending = the kernel's order, U rows ascending
    // = in-line term first (u_inline_first)
    // A power grid's MNA system pivoted with its pads and voltage-source
    // branches first (ggmres.matrices.mna_pivot_order) is a bordered grid:
    // the tail by the flow kernel, the mesh by the wavefront (GG_NO_BORDER=1:
    // the flow kernel for everything)
    CanonTri gl, gu;
    Wave2D wl = select_split_layout(cl, cu, gl, gu);
    // off the wavefront the flow kernel's rows and their terms' x sit where an
    // RCM order of the factors' pattern puts them (a randomly permuted split
    // has no locality in its own index order); GG_FLOW_RCM=0 keeps the natural
    // layout.  The rows' terms keep their order: the same arithmetic.
    std::vector<int> rcm;
    const char *fr = std::getenv("GG_FLOW_RCM");
    if (!wl.ok && !(fr && fr[0] == '0')) rcm = rcm_order(cl, cu);
    setup_space(s, &wl, perm_row, perm_col, rcm.empty() ? nullptr : &rcm);
    s->split_local = wl.ok || !rcm.empty();
    if (wl.ok && wl.bnt) {
        build_tri_bordered(s->L, cl, gl, wl, s->st);
        build_tri_bordered(s->U, cu, gu, wl, s->st);
    } else {
        build_tri(s->L, cl, &wl, &s->nat2lay_h, s->Ppad, s->st);
        build_tri(s->U, cu, &wl, &s->nat2lay_h, s->Ppad, s->st);
    }
    const long long Pp = s->Ppad;
    const std::vector<long long> &lay = s->nat2lay_h;
    // padding slots: every divisor and multiplier 1.0 (apply_start divides by
    // mid_l; a 0 there would put 0/0 into the padding of y and the wavefront
    // carries a padding NaN into real rows through 0 * NaN)
    std::vector<double> mid(Pp, 1.0), ls(Pp, 1.0), rs(Pp, 1.0);
    std::vector<long long> bmap(Pp, -1), xmap(Pp, -1), xout(n), yout(n);
    for (int r = 0; r < n; r++) {
        const long long p = lay[r];
        mid[p] = middle[r];
        ls[p] = lscale[perm_row[r]];
        rs[p] = rscale[pcinv[r]];
        bmap[p] = perm_row[r];
        xmap[p] = pcinv[r];
        xout[r] = lay[perm_col[r]];
        yout[r] = lay[prinv[r]];
    }
    s->mid_l.upload(mid, s->st);
    s->ls_l.upload(ls, s->st);
    s->rs_l.upload(rs, s->st);
    s->sb_map.upload(bmap, s->st);
    s->sx_map.upload(xmap, s->st);
    s->sx_out.upload(xout, s->st);
    s->sy_out.upload(yout, s->st);
    // the full U (diagonal first) in layout space, entry order kept
    Csr Ul;
    Ul.n = (int)s->P;
    Ul.rp.assign(s->P + 1, 0);
    std::vector<long long> l2n(s->P, -1);
    for (int r = 0; r < n; r++) l2n[lay[r]] = r;
    for (long long p = 0; p < s->P; p++)
        Ul.rp[p + 1] = Ul.rp[p] + (l2n[p] >= 0 ? Uf.rp[l2n[p] + 1] - Uf.rp[l2n[p]] : 0);
    Ul.ci.resize(Uf.nnz());
    Ul.v.resize(Uf.nnz());
    for (long long p = 0; p < s->P; p++) {
        if (l2n[p] < 0) continue;
        int o = Ul.rp[p];
        for (int k = Uf.rp[l2n[p]]; k < Uf.rp[l2n[p] + 1]; k++, o++) {
            Ul.ci[o] = (int)lay[Uf.ci[k]];
            Ul.v[o] = Uf.v[k];
        }
    }
    s->dUfull.upload(Ul, s->st);
    s->pkind = GG_PRECOND_SPLIT;
    GG_HIP(hipStreamSynchronize(s->st));
    return GG_OK;
    GG_API_END
}

int gg_set_precond_user(gg_solver *s, int split, gg_precond_fn fn, void *ctx)
{
    GG_API_BEGIN
    GG_REQUIRE(s && s->have_A, GG_ESTATE, "set_precond before set_matrix");
    GG_REQUIRE(fn, GG_EINVAL, "gg_set_precond_user: null callback");
    GG_REQUIRE(split == 0 || split == 1, GG_EINVAL, "gg_set_precond_user: split must be 0 or 1");
    set_device(s);
    setup_space(s, nullptr);
    s->L.kind = s->U.kind = DevTri::NONE;
    s->ufn = fn;
    s->uctx = ctx;
    s->fin.alloc(std::max(s->A.n, 1));
    s->fout.alloc(std::max(s->A.n, 1));
    s->pkind = split ? GG_PRECOND_USER_SPLIT : GG_PRECOND_USER;
    GG_HIP(hipStreamSynchronize(s->st));
    return GG_OK;
    GG_API_END
}

int gg_precond_kind(gg_solver *s) { return s ? s->pkind : GG_EINVAL; }
int gg_uses_wavefront(gg_solver *s) { return (s && s->wave) ? 1 : 0; }

long long gg_layout(gg_solver *s, long long *lay2nat, long long cap)
{
    if (!s || s->pkind < 0) return GG_ESTATE;
    if (lay2nat && cap > 0) {
        std::fill(lay2nat, lay2nat + std::min(cap, s->Ppad), -1LL);
        for (size_t r = 0; r < s->nat2lay_h.size(); r++)
            if (s->nat2lay_h[r] < cap) lay2nat[s->nat2lay_h[r]] = (long long)r;
    }
    return s->Ppad;
}
int gg_reduce_blocks(gg_solver *s, int *G)
{
    if (!s || !G) return GG_EINVAL;
    if (s->pkind < 0) return GG_ESTATE;
    *G = s->G;
    return GG_OK;
}
int gg_set_division(gg_solver *s, int mode)
{
    if (!s) return GG_EINVAL;
    if (mode != GG_DIV_EXACT && mode != GG_DIV_RCP && mode != GG_DIV_FMA) {
        set_error("gg_set_division: mode must be GG_DIV_EXACT, GG_DIV_RCP or GG_DIV_FMA");
        return GG_EINVAL;
    }
    s->div_mode = mode;
    return GG_OK;
}
int gg_trsv_levels(gg_solver *s, int which)
{
    if (!s || (which != 0 && which != 1)) return GG_EINVAL;
    const DevTri &T = which ? s->U : s->L;
    if (T.kind == DevTri::LEVEL) return (int)T.lev_ptr.size() - 1;
    if (T.kind == DevTri::WAVE2D) {
        const Wave2D &w = T.wl;
        // (bordered: the tail's levels run before / after the grid's)
        const int tail = T.tail ? (int)T.tail->lev_ptr.size() - 1 : 0;
        if (w.nz > 1) return w.nx + w.ny + w.nz - 2 + tail;
        return w.nx + w.skew * (w.ny - 1) + tail;
    }
    return 0;
}
int gg_mgs_kernel(gg_solver *s, char *name, int cap)
{
    if (!s || !name || cap <= 0) return GG_EINVAL;
    std::string k;
    if (s->m_alloc > 0 && !s->shared) {
        if (s->persist)
            k = "k_arnoldi_persist<" + std::to_string(arnoldi_persist_units(s->G, s->Ppad)) + ", " +
                std::to_string(mgs_gather_form()) + ", " + std::to_string(mgs_prefetch()) + ">";
        else if (s->wide) k = "k_arnoldi_wide";
    }
    std::snprintf(name, (size_t)cap, "%s", k.c_str());
    return (int)k.size();
}
int gg_trsv_kernel(gg_solver *s, int which, char *name, int cap)
{
    if (!s || (which != 0 && which != 1) || !name || cap <= 0) return GG_EINVAL;
    DevTri &T = which == 0 ? s->L : s->U;
    T.fast = s->div_mode;
    std::string k;
    if (which == 0 && fuse_spmv_active(s)) {
        k = "k_trsv_wave2d_spmv<" + std::to_string(T.eff_div()) + ">";
    } else if (T.kind == DevTri::WAVE2D) {
        const char *fwd = T.lower ? "true" : "false";
        const int div = T.eff_div();
        if (T.wl.tile)
            k = std::string("k_trsv_tile3d<") + fwd + ", " + std::to_string(div) + ", false>";
        else
            k = std::string("k_trsv_wave2d<") + fwd + ", " + std::to_string(div) + ", false, " +
                (T.wl.nz > 1 ? "true" : "false") + ", " + std::to_string(T.wl.nz > 1 ? 1 : T.wl.skew) + ", " +
                ((T.il && div != WD_UFMA && div != WD_SFMA) ? "true" : "false") + ">";   // fused rows: one order
    } else if (T.kind == DevTri::LEVEL) {
        const char *lv = std::getenv("GG_TRSV_LEVELS");
        k = (lv && atoi(lv) != 0) ? "k_trsv_level" : "k_trsv_flow";
    }
    std::snprintf(name, (size_t)cap, "%s", k.c_str());
    return (int)k.size();
}
int gg_division_active(gg_solver *s, int which)
{
    if (!s || (which != 0 && which != 1)) return GG_EINVAL;
    DevTri &T = which == 0 ? s->L : s->U;
    T.fast = s->div_mode;
    if (T.kind != DevTri::WAVE2D) return GG_DIV_EXACT;
    const int e = T.eff_div();
    return e == WD_MUL ? GG_DIV_RCP : (e == WD_UFMA || e == WD_SFMA) ? GG_DIV_FMA : GG_DIV_EXACT;
}
int gg_spmv_sliced(gg_solver *s) { return (s && s->dA.sell) ? 1 : 0; }
int gg_spmv_panels(gg_solver *s) { return (s && s->dA.panel) ? s->dA.npanel : 0; }
int gg_spmv_rtile(gg_solver *s) { return (s && s->dA.panel) ? s->dA.rtile : 0; }

int gg_solve_device(gg_solver *s, const double *d_b, double *d_x, const gg_options *opt,
                    gg_result *res)
{
    GG_API_BEGIN
    GG_REQUIRE(s, GG_EINVAL, "null solver");
    return solve_device(s, d_b, d_x, opt, res);
    GG_API_END
}

// the step loop behind gg_transient / gg_transient_src / gg_transient_mna (host
// source tables).  Step j = 1..nsteps evaluates the sources at time index
// it0 + j - 1.  The right-hand side is B u + (C/h) x with B an incidence matrix
// (src_node) and C/h diagonal (cdiag), or -- when Rm and Bm are given -- the
// general B u + R x of gg_transient_mna.
static int transient_loop(gg_solver *s, int it0, int nsteps, double h, const double *cdiag, int nsrc,
              const int *src_node, const std::vector<int> &kind, const std::vector<int> &dptr,
              const std::vector<double> &data, int nport, const int *port, double *x, const gg_options *opt,
              double *port_out, int *iters_total, const Csr *Rm = nullptr, const Csr *Bm = nullptr)
{
    GG_REQUIRE(nport == 0 || (port && port_out), GG_EINVAL, "null port arrays");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_transient: no matrix");
    set_device(s);
    const int n = s->A.n;
    const bool general = Rm && Bm;
    std::vector<int> sptr(n + 1, 0), sidx(general ? 0 : nsrc);
    if (!general) {
        // B^T by row: the sources of each row in ascending k (cs_dl_gaxpy column order)
        for (int k = 0; k < nsrc; k++) {
            GG_REQUIRE(src_node[k] >= 0 && src_node[k] < n, GG_EINVAL, "source node out of range");
            sptr[src_node[k] + 1]++;
        }
        for (int r = 0; r < n; r++) sptr[r + 1] += sptr[r];
        std::vector<int> fill(sptr.begin(), sptr.end() - 1);
        for (int k = 0; k < nsrc; k++) sidx[fill[src_node[k]]++] = k;
    }
    for (int j = 0; j < nport; j++) GG_REQUIRE(port[j] >= 0 && port[j] < n, GG_EINVAL, "port out of range");
    DBuf<int> d_sptr, d_sidx, d_port, d_kind, d_dptr;
    DBuf<double> d_data, d_u, d_c, d_w, d_pv;
    DevCsr d_R, d_B;
    if (general) {
        d_R.upload(*Rm, s->st);
        d_B.upload(*Bm, s->st);
    } else {
        d_sptr.upload(sptr, s->st);
        d_sidx.upload(sidx.data(), sidx.size(), s->st);
        d_c.upload(cdiag, n, s->st);
    }
    d_kind.upload(kind.data(), kind.size(), s->st);
    d_dptr.upload(dptr.data(), dptr.size(), s->st);
    d_data.upload(data.data(), std::max<size_t>(data.size(), 1), s->st);
    d_u.alloc(std::max(nsrc, 1));
    d_w.alloc(std::max(n, 1));
    d_port.upload(port, nport, s->st);
    d_pv.alloc((size_t)std::max(nport, 1) * (nsteps + 1));
    DBuf<double> xd;
    xd.upload(x, n, s->st);
    double *d_x = xd.p;
    launch_gather_ports(nport, d_port.p, d_x, d_pv.p, s->st);
    const int ntap = (int)s->taps.size();
    for (int t : s->taps) GG_REQUIRE(t >= 0 && t < n, GG_EINVAL, "tap node out of range");
    DBuf<int> d_tap;
    DBuf<double> d_tmax, d_tmin, d_tsum;
    if (ntap) {
        d_tap.upload(s->taps, s->st);
        d_tmax.alloc(ntap);
        d_tmin.alloc(ntap);
        d_tsum.alloc(ntap);
        launch_taps(ntap, d_tap.p, d_x, d_tmax.p, d_tmin.p, d_tsum.p, 0, 0.0, s->st);
    }
    int total = 0, status = GG_OK;
    // each step's solve is told how many inner iterations the previous one took
    // (solve_device_once: a short first chunk instead of two speculative cycles)
    struct HintReset {
        gg_solver *s;
        ~HintReset() { s->iter_hint = 0; }
    } hint_reset{s};
    const char *he = std::getenv("GG_TRANSIENT_HINT");
    const bool use_hint = !(he && he[0] == '0');
    s->iter_hint = 0;
    for (int it = 1; it <= nsteps; it++) {
        const int tidx = it0 + it - 1;              // time index of the sources
        if (general)
            launch_transient_step_csr(n, nsrc, d_kind.p, d_dptr.p, d_data.p, tidx, h, d_u.p, d_B.rp.p,
                                      d_B.ci.p, d_B.v.p, d_R.rp.p, d_R.ci.p, d_R.v.p, d_x, d_w.p, s->st);
        else
            launch_transient_step(n, nsrc, d_kind.p, d_dptr.p, d_data.p, tidx, h, d_u.p, d_sptr.p, d_sidx.p,
                                  d_c.p, d_x, d_w.p, s->st);
        gg_result r{};
        const int rc = solve_device(s, d_w.p, d_x, opt, &r);
        if (rc != GG_OK) status = rc;
        total += r.iters;
        s->iter_hint = use_hint && rc >= 0 ? r.inner_iters : 0;
        launch_gather_ports(nport, d_port.p, d_x, d_pv.p + (size_t)it * nport, s->st);
        launch_taps(ntap, d_tap.p, d_x, d_tmax.p, d_tmin.p, d_tsum.p, 1, 0.0, s->st);
    }
    if (ntap) {   // avg over the nsteps + 1 time points (ts.size()), src/mna_solve_gpu_gmres.cpp:782
        launch_taps(ntap, d_tap.p, d_x, d_tmax.p, d_tmin.p, d_tsum.p, 2, (double)(nsteps + 1), s->st);
        s->tap_max.resize(ntap);
        s->tap_min.resize(ntap);
        s->tap_avg.resize(ntap);
        GG_HIP(hipMemcpyAsync(s->tap_max.data(), d_tmax.p, ntap * sizeof(double), hipMemcpyDeviceToHost, s->st));
        GG_HIP(hipMemcpyAsync(s->tap_min.data(), d_tmin.p, ntap * sizeof(double), hipMemcpyDeviceToHost, s->st));
        GG_HIP(hipMemcpyAsync(s->tap_avg.data(), d_tsum.p, ntap * sizeof(double), hipMemcpyDeviceToHost, s->st));
    }
    if (nport) {
        std::vector<double> pv((size_t)nport * (nsteps + 1));
        GG_HIP(hipMemcpyAsync(pv.data(), d_pv.p, pv.size() * sizeof(double), hipMemcpyDeviceToHost, s->st));
        GG_HIP(hipStreamSynchronize(s->st));
        for (int it = 0; it <= nsteps; it++)
            for (int j = 0; j < nport; j++) port_out[(size_t)j * (nsteps + 1) + it] = pv[(size_t)it * nport + j];
    }
    GG_HIP(hipMemcpyAsync(x, d_x, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    *iters_total = total;
    return status;
}

int gg_transient(gg_solver *s, int nsteps, double h, const double *cdiag, int nsrc,
                 const int *src_node, const double *pulse, int nport, const int *port,
                 double *x, const gg_options *opt, double *port_out, int *iters_total)
{
    GG_API_BEGIN
    GG_REQUIRE(s && opt && x && cdiag && iters_total, GG_EINVAL, "null argument");
    GG_REQUIRE(nsteps >= 0 && nsrc >= 0 && nport >= 0, GG_EINVAL, "negative count");
    GG_REQUIRE(nsrc == 0 || (src_node && pulse), GG_EINVAL, "null source arrays");
    std::vector<int> kind(std::max(nsrc, 1), GG_SRC_PULSE), dptr(nsrc + 1);
    for (int k = 0; k <= nsrc; k++) dptr[k] = 7 * k;
    std::vector<double> data(pulse, pulse + (size_t)7 * nsrc);
    return transient_loop(s, 1, nsteps, h, cdiag, nsrc, src_node, kind, dptr, data, nport, port, x, opt,
                          port_out, iters_total);
    GG_API_END
}

int gg_transient_set_taps(gg_solver *s, int ntap, const int *tap_node)
{
    GG_API_BEGIN
    GG_REQUIRE(s && ntap >= 0 && (ntap == 0 || tap_node), GG_EINVAL, "null argument");
    s->taps.assign(tap_node, tap_node + ntap);
    s->tap_max.clear();
    s->tap_min.clear();
    s->tap_avg.clear();
    return GG_OK;
    GG_API_END
}

int gg_transient_get_taps(gg_solver *s, double *max_v, double *min_v, double *avg_v, double *ir)
{
    GG_API_BEGIN
    GG_REQUIRE(s, GG_EINVAL, "null argument");
    const size_t nt = s->taps.size();
    GG_REQUIRE(s->tap_max.size() == nt && nt > 0, GG_ESTATE, "gg_transient_get_taps: no transient run with taps");
    for (size_t j = 0; j < nt; j++) {
        if (max_v) max_v[j] = s->tap_max[j];
        if (min_v) min_v[j] = s->tap_min[j];
        if (avg_v) avg_v[j] = s->tap_avg[j];
        if (ir) ir[j] = s->tap_max[j] - s->tap_min[j];      // ir_value = max_value - min_value (:789)
    }
    return GG_OK;
    GG_API_END
}

// validated device tables of a gg_src_kind source list
static void source_tables(int nsrc, const int *src_kind, const int *src_ptr, const double *src_data,
                          std::vector<int> &kind, std::vector<int> &dptr, std::vector<double> &data)
{
    GG_REQUIRE(nsrc == 0 || (src_kind && src_ptr && src_data), GG_EINVAL, "null source arrays");
    kind.assign(std::max(nsrc, 1), GG_SRC_DC);
    dptr.assign(nsrc + 1, 0);
    for (int k = 0; k < nsrc; k++) {
        const int len = src_ptr[k + 1] - src_ptr[k];
        GG_REQUIRE(src_ptr[k] >= 0 && len >= 0, GG_EINVAL, "transient: bad src_ptr");
        const int need = src_kind[k] == GG_SRC_DC ? 1 : src_kind[k] == GG_SRC_PULSE ? 7 : -1;
        GG_REQUIRE(src_kind[k] == GG_SRC_DC || src_kind[k] == GG_SRC_PULSE || src_kind[k] == GG_SRC_PWL,
                   GG_EINVAL, "transient: unknown source kind");
        GG_REQUIRE(need < 0 ? (len >= 2 && len % 2 == 0) : len == need, GG_EINVAL,
                   "transient: DC takes 1 value, PULSE 7, PWL (time, value) pairs");
        kind[k] = src_kind[k];
        dptr[k + 1] = src_ptr[k + 1] - src_ptr[0];
    }
    data.assign(src_data + (nsrc ? src_ptr[0] : 0), src_data + (nsrc ? src_ptr[nsrc] : 0));
}

int gg_transient_src(gg_solver *s, int nsteps, double h, const double *cdiag, int nsrc,
                     const int *src_node, const int *src_kind, const int *src_ptr, const double *src_data,
                     int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                     int *iters_total)
{
    GG_API_BEGIN
    GG_REQUIRE(s && opt && x && cdiag && iters_total, GG_EINVAL, "null argument");
    GG_REQUIRE(nsteps >= 0 && nsrc >= 0 && nport >= 0, GG_EINVAL, "negative count");
    GG_REQUIRE(nsrc == 0 || src_node, GG_EINVAL, "null source arrays");
    std::vector<int> kind, dptr;
    std::vector<double> data;
    source_tables(nsrc, src_kind, src_ptr, src_data, kind, dptr, data);
    return transient_loop(s, 1, nsteps, h, cdiag, nsrc, src_node, kind, dptr, data, nport, port, x, opt,
                          port_out, iters_total);
    GG_API_END
}

int gg_transient_mna(gg_solver *s, int it0, int nsteps, double h, const int *r_row_ptr, const int *r_col_idx,
                     const double *r_val, int nsrc, const int *b_row_ptr, const int *b_col_idx,
                     const double *b_val, const int *src_kind, const int *src_ptr, const double *src_data,
                     int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                     int *iters_total)
{
    GG_API_BEGIN
    GG_REQUIRE(s && opt && x && iters_total, GG_EINVAL, "null argument");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_transient_mna: no matrix");
    GG_REQUIRE(it0 >= 0 && nsteps >= 0 && nsrc >= 0 && nport >= 0, GG_EINVAL, "negative count");
    const int n = s->A.n;
    Csr R, Bm;
    R.n = Bm.n = n;
    if (r_row_ptr) {
        check_csr(n, r_row_ptr, r_col_idx, r_val, "gg_transient_mna R");
        R = make_csr(n, r_row_ptr, r_col_idx, r_val);
    } else {
        R.rp.assign(n + 1, 0);                // R = 0 (a DC operating point)
    }
    GG_REQUIRE(b_row_ptr && b_row_ptr[0] == 0, GG_EINVAL, "gg_transient_mna: bad B row_ptr");
    for (int r = 0; r < n; r++) {
        GG_REQUIRE(b_row_ptr[r + 1] >= b_row_ptr[r], GG_EINVAL, "gg_transient_mna: B row_ptr not monotone");
        for (int k = b_row_ptr[r]; k < b_row_ptr[r + 1]; k++)
            GG_REQUIRE(b_col_idx && b_val && b_col_idx[k] >= 0 && b_col_idx[k] < nsrc, GG_EINVAL,
                       "gg_transient_mna: B column (source) index out of range");
    }
    Bm.rp.assign(b_row_ptr, b_row_ptr + n + 1);
    Bm.ci.assign(b_col_idx, b_col_idx + b_row_ptr[n]);
    Bm.v.assign(b_val, b_val + b_row_ptr[n]);
    std::vector<int> kind, dptr;
    std::vector<double> data;
    source_tables(nsrc, src_kind, src_ptr, src_data, kind, dptr, data);
    return transient_loop(s, it0, nsteps, h, nullptr, nsrc, nullptr, kind, dptr, data, nport, port, x, opt,
                          port_out, iters_total, &R, &Bm);
    GG_API_END
}

int gg_solve(gg_solver *s, const double *b, double *x, const gg_options *opt, gg_result *res)
{
    GG_API_BEGIN
    GG_REQUIRE(s && b && x, GG_EINVAL, "null argument");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_solve: no matrix");
    set_device(s);
    stage_in(s, b, s->nat_in);
    stage_in(s, x, s->nat_out);
    int rc = solve_device(s, s->nat_in.p, s->nat_out.p, opt, res);
    stage_out(s, s->nat_out, x);
    return rc;
    GG_API_END
}

int gg_solve_device_f32(gg_solver *s, const float *d_b, float *d_x, const gg_options *opt, gg_result *res)
{
    GG_API_BEGIN
    GG_REQUIRE(s && d_b && d_x, GG_EINVAL, "null argument");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_solve: no matrix");
    set_device(s);
    const int n = s->A.n;
    for (DBuf<double> *d : {&s->nat_in, &s->nat_out})
        if (d->n < (size_t)std::max(n, 1)) d->alloc(std::max(n, 1));
    launch_f32_to_f64(Gate{}, d_b, s->nat_in.p, n, s->st);
    launch_f32_to_f64(Gate{}, d_x, s->nat_out.p, n, s->st);
    const int rc = solve_device(s, s->nat_in.p, s->nat_out.p, opt, res);
    launch_f64_to_f32(Gate{}, s->nat_out.p, d_x, n, s->st);
    GG_HIP(hipStreamSynchronize(s->st));
    return rc;
    GG_API_END
}

int gg_device_fingerprint(const void *const *d_p, const unsigned long long *bytes, int count,
                          unsigned long long *fp)
{
    GG_API_BEGIN
    constexpr int kMax = 16;
    GG_REQUIRE(d_p && bytes && fp && count >= 0 && count <= kMax, GG_EINVAL, "gg_device_fingerprint: bad argument");
    for (int i = 0; i < count; i++)
        GG_REQUIRE((d_p[i] || bytes[i] == 0) && bytes[i] % 4 == 0, GG_EINVAL, "gg_device_fingerprint: bad buffer");
    if (count == 0) return GG_OK;
    // kMax accumulators per host thread and DEVICE (the kernel runs
    // on the current device, so its accumulator must live there too), never
    // freed (a thread_local destructor would run after the HIP runtime's own
    // teardown)
    constexpr int kDevs = 64;
    static thread_local unsigned long long *accs[kDevs] = {};
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_REQUIRE(dev >= 0 && dev < kDevs, GG_EINVAL, "gg_device_fingerprint: device index out of range");
    unsigned long long *&acc = accs[dev];
    if (!acc) GG_HIP(hipMalloc(reinterpret_cast<void **>(&acc), kMax * sizeof(unsigned long long)));
    GG_HIP(hipMemsetAsync(acc, 0, count * sizeof(unsigned long long), nullptr));
    for (int i = 0; i < count; i++) launch_fingerprint(d_p[i], (long long)(bytes[i] / 4), acc + i, nullptr);
    GG_HIP(hipMemcpy(fp, acc, count * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return GG_OK;
    GG_API_END
}

int gg_get_history(gg_solver *s, double *out, int cap)
{
    if (!s) return GG_EINVAL;
    int len = (int)s->last_hist.size();
    if (out && cap > 0) std::memcpy(out, s->last_hist.data(), sizeof(double) * std::min(len, cap));
    return len;
}

int gg_spmv(gg_solver *s, const double *x, double *y)
{
    GG_API_BEGIN
    GG_REQUIRE(s && x && y, GG_EINVAL, "null argument");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "gg_spmv: call gg_set_precond_* first (fixes the layout)");
    set_device(s);
    ensure_workspace(s, std::max(s->m_alloc, 1));
    stage_in(s, x, s->nat_in);
    const bool split = s->pkind == GG_PRECOND_SPLIT;      // A' = A with rows / columns permuted
    launch_gather(s->nat_in.p, split ? s->sx_map.p : s->lay2nat.p, s->xv.p, s->Ppad, s->st);
    launch_spmv(Gate{}, s->dA, s->xv.p, nullptr, s->ww.p, false, s->st);
    if (s->nat_out.n < (size_t)std::max(s->A.n, 1)) s->nat_out.alloc(std::max(s->A.n, 1));
    launch_gather(s->ww.p, split ? s->sy_out.p : s->nat2lay.p, s->nat_out.p, s->A.n, s->st);
    stage_out(s, s->nat_out, y);
    return GG_OK;
    GG_API_END
}

int gg_precond_apply(gg_solver *s, int op, const double *in, double *out)
{
    GG_API_BEGIN
    GG_REQUIRE(s && in && out, GG_EINVAL, "null argument");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "no preconditioner");
    const bool split = s->pkind == GG_PRECOND_SPLIT;
    const bool usplit = s->pkind == GG_PRECOND_USER_SPLIT;
    GG_REQUIRE(split || usplit ? (op >= GG_APPLY_LEFT && op <= GG_APPLY_RHS) : op == GG_APPLY_MINV, GG_EINVAL,
               "operator not defined for this preconditioner");
    set_device(s);
    ensure_workspace(s, std::max(s->m_alloc, 1));
    for (DevTri *T : {&s->L, &s->U})
        if (T->kind == DevTri::WAVE2D)
            reset_wave(T, s->st);
    stage_in(s, in, s->nat_in);
    // operator input spaces: LEFT takes an A-row vector (A' row order), START
    // an x (column convention), RIGHT / MINV a vector of the triangles' space
    const long long *in_map = !split || op == GG_APPLY_RIGHT ? s->lay2nat.p
                              : op == GG_APPLY_START        ? s->sx_map.p
                                                            : s->sb_map.p;
    launch_gather(s->nat_in.p, in_map, s->xv.p, s->Ppad, s->st);
    auto run = [&]() {
        GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));
        Gate none;
        switch (op) {
        case GG_APPLY_MINV: apply_minv(s, none, s->xv.p, s->ww.p); break;
        default:
            if (usplit) apply_user(s, none, op, s->xv.p, s->ww.p);
            else if (op == GG_APPLY_LEFT || op == GG_APPLY_RHS) apply_left(s, none, s->xv.p, s->ww.p);
            else if (op == GG_APPLY_RIGHT) apply_right(s, none, s->xv.p, s->ww.p);
            else apply_start(s, none, s->xv.p, s->ww.p);
        }
        check_err(s);
    };
    for (int attempt = 0;; attempt++) {
        try {
            run();
            break;
        } catch (Fallback &f) {
            if (attempt >= 2) throw Error{GG_EHIP, "gg_precond_apply: fallbacks exhausted"};
            apply_fallback(s, f);
            for (DevTri *T : {&s->L, &s->U})
                if (T->kind == DevTri::WAVE2D) reset_wave(T, s->st);   // a drained grid left granules set
        }
    }
    if (s->nat_out.n < (size_t)std::max(s->A.n, 1)) s->nat_out.alloc(std::max(s->A.n, 1));
    launch_gather(s->ww.p, split && op == GG_APPLY_RIGHT ? s->sx_out.p : s->nat2lay.p, s->nat_out.p,
                  s->A.n, s->st);
    stage_out(s, s->nat_out, out);
    return GG_OK;
    GG_API_END
}

int gg_time_spmv(gg_solver *s, int reps, int nrot, double *avg_ms)
{
    GG_API_BEGIN
    GG_REQUIRE(s && avg_ms && reps > 0 && nrot > 0, GG_EINVAL, "bad argument");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "no preconditioner / layout");
    set_device(s);
    if (nrot == 1) {
        // the solver's own A and workspace vectors: no copies (for matrices
        // far larger than the Infinity Cache, e.g. the C3 stand-in)
        ensure_workspace(s, std::max(s->m_alloc, 1));
        launch_fill_u64(reinterpret_cast<unsigned long long *>(s->xv.p), s->Ppad,
                        0x3FF0000000000000ull, s->st);              // x = 1.0
        launch_spmv(Gate{}, s->dA, s->xv.p, nullptr, s->ww.p, false, s->st);   // warm-up
        GG_HIP(hipEventRecord(s->ev0, s->st));
        for (int r = 0; r < reps; r++) launch_spmv(Gate{}, s->dA, s->xv.p, nullptr, s->ww.p, false, s->st);
        GG_HIP(hipEventRecord(s->ev1, s->st));
        GG_HIP(hipEventSynchronize(s->ev1));
        float ms = 0.f;
        GG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        *avg_ms = ms / reps;
        return GG_OK;
    }
    // nrot independent copies of (A, x, y) so repeats are not served on-die
    std::vector<std::unique_ptr<DevCsr>> As;
    std::vector<std::unique_ptr<DBuf<double>>> xs, ys;
    for (int k = 0; k < nrot; k++) {
        auto A = std::make_unique<DevCsr>();
        A->copy_from(s->dA, s->st);
        As.push_back(std::move(A));
        auto x = std::make_unique<DBuf<double>>();
        auto y = std::make_unique<DBuf<double>>();
        x->alloc(s->Ppad);
        y->alloc(s->Ppad);
        std::vector<double> h(s->Ppad, 1.0);
        GG_HIP(hipMemcpyAsync(x->p, h.data(), s->Ppad * 8, hipMemcpyHostToDevice, s->st));
        GG_HIP(hipStreamSynchronize(s->st));
        xs.push_back(std::move(x));
        ys.push_back(std::move(y));
    }
    for (int k = 0; k < nrot; k++)   // warm-up
        launch_spmv(Gate{}, *As[k], xs[k]->p, nullptr, ys[k]->p, false, s->st);
    GG_HIP(hipEventRecord(s->ev0, s->st));
    for (int r = 0; r < reps; r++) {
        int k = r % nrot;
        launch_spmv(Gate{}, *As[k], xs[k]->p, nullptr, ys[k]->p, false, s->st);
    }
    GG_HIP(hipEventRecord(s->ev1, s->st));
    GG_HIP(hipEventSynchronize(s->ev1));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    *avg_ms = ms / reps;
    return GG_OK;
    GG_API_END
}

int gg_time_precond(gg_solver *s, int reps, double *avg_ms)
{
    GG_API_BEGIN
    GG_REQUIRE(s && avg_ms && reps > 0, GG_EINVAL, "bad argument");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "no preconditioner");
    set_device(s);
    ensure_workspace(s, std::max(s->m_alloc, 1));
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));
    Gate none;
    auto once = [&]() {
        if (s->pkind == GG_PRECOND_SPLIT) apply_left(s, none, s->bv.p, s->ww.p);
        else apply_minv(s, none, s->bv.p, s->ww.p);
    };
    once();
    GG_HIP(hipEventRecord(s->ev0, s->st));
    for (int r = 0; r < reps; r++) once();
    GG_HIP(hipEventRecord(s->ev1, s->st));
    GG_HIP(hipEventSynchronize(s->ev1));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    *avg_ms = ms / reps;
    int err = 0;
    GG_HIP(hipMemcpy(&err, s->err.p, sizeof(int), hipMemcpyDeviceToHost));
    GG_REQUIRE((err & 1) == 0, GG_ETIMEOUT, "wavefront triangular solve: boundary wait timed out");
    return GG_OK;
    GG_API_END
}

int gg_trace_precond(gg_solver *s, int which, long long *out, long long cap, int *nbands,
                     int *nbatch)
{
    GG_API_BEGIN
    GG_REQUIRE(s && out && nbands && nbatch && (which == 0 || which == 1), GG_EINVAL, "bad argument");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "no preconditioner");
    DevTri &T = which == 0 ? s->L : s->U;
    GG_REQUIRE(T.kind == DevTri::WAVE2D && !T.tail && ((T.wl.nz == 1 && T.wl.skew == 1) || T.wl.tile), GG_ESTATE,
               "unskewed 2D or 3D tile wavefront path not active (bordered grids are not traced)");
    set_device(s);
    ensure_workspace(s, std::max(s->m_alloc, 1));
    // per band (2D) 3 nbatch + 8 words, per tile (3D tiles, k_trsv_tile3d) 5 nbatch + 8
    const int nb = T.wl.nbands, nbt = T.wl.tile ? T.wl.T / tile_batch_steps() : T.wl.T / wave_batch_steps(T.eff_div());
    const long long need = (long long)nb * ((T.wl.tile ? 5 : 3) * nbt + 8);
    GG_REQUIRE(cap >= need, GG_EINVAL, "trace buffer too small");
    DBuf<long long> buf;
    buf.alloc((size_t)need);
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), s->st));
    T.trace = buf.p;
    Gate none;
    T.fast = s->div_mode;
    launch_trsv(none, T, s->bv.p, s->t1.p, s->err.p, s->st);
    T.trace = nullptr;
    GG_HIP(hipMemcpyAsync(out, buf.p, need * sizeof(long long), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    *nbands = nb;
    *nbatch = nbt;
    return GG_OK;
    GG_API_END
}

int gg_profile_enable(gg_solver *s, int kinds)
{
    if (!s || (kinds & ~GG_PROF_ALL)) return GG_EINVAL;
    s->prof_mask = kinds;
    return GG_OK;
}

int gg_profile_reset(gg_solver *s)
{
    if (!s) return GG_EINVAL;
    for (int k = 0; k < GG_PROF_NKINDS; k++) {
        s->prof_ms[k] = 0;
        s->prof_cnt[k] = 0;
    }
    return GG_OK;
}

int gg_profile_get(gg_solver *s, int kind, int *launches, double *total_ms)
{
    if (!s || kind < 0 || kind >= GG_PROF_NKINDS) return GG_EINVAL;
    if (launches) *launches = (int)s->prof_cnt[kind];
    if (total_ms) *total_ms = s->prof_ms[kind];
    return GG_OK;
}

double gg_bytes_spmv(gg_solver *s)
{
    if (!s || !s->have_A) return 0.0;
    const double n = s->A.n, nnz = s->A.nnz();
    return 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;   // SURVEY.md 8(d) B_spmv
}

double gg_bytes_precond(gg_solver *s)
{
    if (!s || s->pkind < 0) return 0.0;
    s->L.fast = s->U.fast = s->div_mode;
    return s->L.alg_bytes() + s->U.alg_bytes();
}

double gg_bytes_trsv(gg_solver *s, int which)
{
    if (!s || s->pkind < 0 || (which != 0 && which != 1)) return 0.0;
    s->L.fast = s->U.fast = s->div_mode;
    return which == 0 ? s->L.alg_bytes() : s->U.alg_bytes();
}

double gg_bytes_trsv_stream(gg_solver *s, int which)
{
    if (!s || s->pkind < 0 || (which != 0 && which != 1)) return 0.0;
    s->L.fast = s->U.fast = s->div_mode;
    return which == 0 ? s->L.stream_alg_bytes() : s->U.stream_alg_bytes();
}

}  // extern "C"
