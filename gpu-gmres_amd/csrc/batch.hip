// batch.hip -- the many-RHS solve: nrhs independent right-hand sides on ONE
// matrix and preconditioner, carried through one set of launches.
//
// "many-RHS" = independent source scenarios solved as a
// batch.  The reference runs its step driver once per scenario
// (src/mna_solve_gpu_gmres.cpp:564-647 around GMRES_GPU_tran,
// src/gmres.cu:2736-2827).  Here scenario q keeps its own Krylov basis, H,
// Givens rotations, residual history and control block -- one arena per
// scenario, q * zs bytes after scenario 0's -- and every launch of a GMRES
// phase serves all scenarios at once:
//   * the SpMV reads A's sliced-ELL entries once for up to 8 scenarios
//     (k_spmv_sell_b);
//   * the 2D wavefront triangular solves run every scenario's bands side by
//     side in one launch (k_trsv_wave2d_batch): one dependency chain of
//     nx + ny - 1 steps for all of them instead of one per scenario;
//   * the MGS kernels (k_dot, k_mgs_step, k_arnoldi_finalize) reduce nrhs
//     dot products per launch, the update and the scalar kernels likewise.
// Per scenario the arithmetic is the single-RHS solve's -- the same kernels
// with a scenario offset -- so scenario q's history, iteration count and
// solution are bit-identical to gg_solve_device on that right-hand side alone
// (whose persistent and per-step orthogonalizations are bit-identical too).
// A scenario whose gate is closed (converged, restart-converged, max_iter
// exhausted) drops out of every launch; the others go on.
//
// The restart cycle is enqueued in chunks of inner iterations (GG_BATCH_CHUNK,
// default 3) with the host one chunk ahead, instead of m gated iterations: a
// transient step converges in ~9 of m = 32 iterations, and a gated launch
// still costs its dispatch.  When every scenario's cycle is over at a chunk's
// read-back, the cycle's tail (Update, residual, its norm) is enqueued; the
// host waits for the tail's control blocks only when some scenario did not
// converge inside the cycle (restart or max_iter).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "gg_solver.h"

namespace gg {

namespace {

constexpr long long kAlign = 256;
long long align_up(long long a) { return (a + kAlign - 1) / kAlign * kAlign; }

// GG_BATCH_MGS: the orthogonalization of a batched inner iteration -- 0 the
// per-step kernels with every scenario in each launch (k_dot, k_mgs_step,
// k_arnoldi_finalize: i + 3 launches), 1 the single-scenario persistent kernel
// once per scenario (k_arnoldi_persist: w and the basis step in registers, the
// same reduction tree, so the same bits)
int batch_mgs()
{
    static const int k = [] {
        const char *e = std::getenv("GG_BATCH_MGS");
        return e ? std::atoi(e) : 1;
    }();
    return k;
}

// GG_BATCH_MGS2=0: one persistent launch per scenario instead of per pair
bool batch_mgs2()
{
    static const bool on = [] {
        const char *e = std::getenv("GG_BATCH_MGS2");
        return !(e && e[0] == '0');
    }();
    return on;
}

int batch_chunk()
{
    static const int k = [] {
        const char *e = std::getenv("GG_BATCH_CHUNK");
        const int v = e ? std::atoi(e) : 3;
        return v >= 1 ? v : 3;
    }();
    return k;
}

}  // namespace

// Per-scenario arena (offsets in bytes, each 256-B aligned) and the host side
// of the read-backs.
struct BatchWs {
    int S = 0, m = -1;
    long long Ppad = 0, hist_cap = 0, ngL = 0, ngU = 0;
    long long zs = 0;                    // bytes per scenario
    DBuf<char> arena;
    long long oV = 0, ow = 0, oww = 0, or_ = 0, orr = 0, obb = 0, ot1 = 0, oxv = 0, obv = 0, opA = 0, opB = 0,
              oH = 0, os = 0, ocs = 0, osn = 0, oy = 0, ohist = 0, ods = 0, oLg = 0, oUg = 0, ogran = 0, oxgran = 0;
    // the persistent orthogonalization (GG_BATCH_MGS 1): its all-gather granules
    // per scenario (m (m+2) G, then m (m+2) sums) and XCD slots, and the
    // solver-wide election words; persist = admitted (co-residency), cleared
    // for the solver's life when a launch was not co-resident
    bool persist = false;
    bool persist2 = false;               // two scenarios per persistent launch (k_arnoldi_persist2)
    long long ngran = 0, nxgran = 0;
    DBuf<unsigned long long> elect;
    unsigned long long seq = 0;
    // read-back slots: the scenarios' control blocks + the error word, written
    // by k_pack_states_b straight into mapped pinned memory
    static constexpr int kSlots = 4;
    DevState *h_st[kSlots] = {};
    DevState *d_st[kSlots] = {};
    hipEvent_t ev[kSlots] = {};
    std::vector<long long> hist_len;     // per scenario, of the last batched solve
    double *dp(long long off) { return reinterpret_cast<double *>(arena.p + off); }
    ~BatchWs()
    {
        for (int k = 0; k < kSlots; k++) {
            if (h_st[k]) (void)hipHostFree(h_st[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
        }
    }
};

void batch_release(gg_solver *s)
{
    delete s->batch;
    s->batch = nullptr;
}

namespace {

// one scenario's outcome (the single solve's bookkeeping, solver.hip
// solve_device_once)
struct Track {
    bool fin = false, cyc_over = false;
    int ret = 1, iters = 0, inner = 0, restarts = 0, prev_j = 1;
    long long hist_len = 1;
    double relres = 0.0;
};

bool batchable(const gg_solver *s)
{
    const bool left = s->pkind == GG_PRECOND_ILU0 || s->pkind == GG_PRECOND_ILUK || s->pkind == GG_PRECOND_LU;
    if (!left || !s->wave) return false;
    if (s->L.kind != DevTri::WAVE2D || s->U.kind != DevTri::WAVE2D) return false;
    const char *e = std::getenv("GG_BATCH_SEQ");          // A/B, tests: scenario by scenario
    if (e && e[0] == '1') return false;
    DevTri &L = const_cast<DevTri &>(s->L), &U = const_cast<DevTri &>(s->U);
    L.fast = s->div_mode;
    U.fast = s->div_mode;
    return trsv_batchable(L) && trsv_batchable(U);
}

void ensure_batch(gg_solver *s, int S, int m, long long hist_need)
{
    BatchWs *B = s->batch;
    if (B && B->S == S && B->m == m && B->Ppad == s->Ppad && B->hist_cap >= hist_need &&
        B->ngL == trsv_b_granules(s->L) && B->ngU == trsv_b_granules(s->U))
        return;
    batch_release(s);
    B = new BatchWs;
    s->batch = B;
    B->S = S;
    B->m = m;
    B->Ppad = s->Ppad;
    B->hist_cap = std::max<long long>(hist_need, 64);
    B->ngL = trsv_b_granules(s->L);
    B->ngU = trsv_b_granules(s->U);
    const long long P = s->Ppad;
    long long o = 0;
    auto take = [&](long long bytes) {
        const long long at = o;
        o = align_up(o + bytes);
        return at;
    };
    B->oV = take((long long)(m + 1) * P * 8);
    B->ow = take(P * 8);
    B->oww = take(P * 8);
    B->or_ = take(P * 8);
    B->orr = take(P * 8);
    B->obb = take(P * 8);
    B->ot1 = take(P * 8);
    B->oxv = take(P * 8);
    B->obv = take(P * 8);
    B->opA = take(1024 * 8);
    B->opB = take(1024 * 8);
    B->oH = take((long long)(m + 1) * m * 8);
    B->os = take((long long)(m + 1) * 8);
    B->ocs = take((long long)(m + 1) * 8);
    B->osn = take((long long)(m + 1) * 8);
    B->oy = take((long long)(m + 1) * 8);
    B->ohist = take(B->hist_cap * 8);
    B->ods = take((long long)sizeof(DevState));
    B->oLg = take(B->ngL * 8);
    B->oUg = take(B->ngU * 8);
    {
        const int pj = arnoldi_persist_units(s->G, s->Ppad);
        const int xr = (mgs_gather_form() == 3 && mgs_prefetch()) ? kMgsXcds : 0;
        B->persist = batch_mgs() == 1 && pj != 0 && s->G + xr <= arnoldi_persist_max_blocks(pj);
        B->persist2 = B->persist && S > 1 && xr == 0 && mgs_gather_form() == 2 && mgs_prefetch() == 1 &&
                      arnoldi_persist2_units(s->G, s->Ppad) != 0 && batch_mgs2();
        if (B->persist) {
            B->ngran = (long long)m * (m + 2) * (s->G + 1);
            B->nxgran = (long long)m * (m + 2) * kMgsXcdWords;
            B->ogran = take(B->ngran * 8);
            B->oxgran = take(B->nxgran * 8);
            B->elect.alloc(kMgsElectWords);
            GG_HIP(hipMemsetAsync(B->elect.p, 0, kMgsElectWords * sizeof(unsigned long long), s->st));
        }
    }
    B->zs = align_up(o);
    B->arena.alloc((size_t)B->zs * S);
    // every vector +0 in its padding slots, every dummy granule 0 (read as ready)
    GG_HIP(hipMemsetAsync(B->arena.p, 0, (size_t)B->zs * S, s->st));
    for (int k = 0; k < BatchWs::kSlots; k++) {
        GG_HIP(hipHostMalloc(reinterpret_cast<void **>(&B->h_st[k]), sizeof(DevState) * (S + 1), hipHostMallocMapped));
        GG_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&B->d_st[k]), B->h_st[k], 0));
        GG_HIP(hipEventCreateWithFlags(&B->ev[k], hipEventDisableTiming));
    }
    B->hist_len.assign(S, 0);
}

// the scenarios' control blocks (and the error word, in slot S's err) into
// read-back slot k, then its event
void readback(gg_solver *s, BatchWs *B, int k)
{
    launch_pack_states_b(reinterpret_cast<DevState *>(B->arena.p + B->ods), B->zs, B->S, B->d_st[k], s->err.p,
                         s->st);
    GG_HIP(hipEventRecord(B->ev[k], s->st));
}

struct BatchErr {
    int bits;
};
struct BatchAbort {};     // a persistent orthogonalization grid was not co-resident
// wait for slot k; the error word: bit 0 time-out (fatal), bit 1 a WD_RCP range
// miss (the caller repeats the solve with IEEE division)
const DevState *wait_slot(BatchWs *B, int k)
{
    GG_HIP(hipEventSynchronize(B->ev[k]));
    const int err = B->h_st[k][B->S].err;
    GG_REQUIRE((err & 1) == 0, GG_ETIMEOUT, "batched solve: wavefront boundary wait timed out");
    if (err & 2) throw BatchErr{err};
    return B->h_st[k];
}

struct Ctx {
    gg_solver *s;
    BatchWs *B;
    int S, m, G;
    long long P, zs;
    UnitMap um;
    DevState *ds;
    double *V, *w, *ww, *r, *rr, *bb, *t1, *xv, *bv, *pA, *pB, *H, *sv, *cs, *sn, *y, *hist;
    unsigned long long *Lg, *Ug, *gran, *xgran;
};
// scenario q's copy of a per-scenario pointer
template <class T>
T *zq(T *p, long long zs, int q)
{
    return reinterpret_cast<T *>(reinterpret_cast<char *>(const_cast<typename std::remove_const<T>::type *>(p)) +
                                 (long long)q * zs);
}

void trsv_pair(const Ctx &c, Gate g, const double *in, double *out)
{
    gg_solver *s = c.s;
    launch_trsv_b(g, s->L, in, c.t1, c.Lg, s->err.p, c.S, c.zs, s->st);
    launch_trsv_b(g, s->U, c.t1, out, c.Ug, s->err.p, c.S, c.zs, s->st);
}

void enqueue_init_b(const Ctx &c)
{
    gg_solver *s = c.s;
    Gate none;
    trsv_pair(c, none, c.bv, c.bb);                                             // bb = M b
    launch_dot_b(none, c.bb, c.bb, c.pA, c.G, c.P, c.S, c.zs, s->st);
    launch_set_normb_b(c.pA, c.G, c.ds, c.S, c.zs, s->st);
    launch_spmv_b(none, s->dA, c.xv, c.bv, c.rr, true, c.S, c.zs, s->st);        // rr = b - A x
    trsv_pair(c, none, c.rr, c.r);                                              // r = M rr
    launch_dot_b(none, c.r, c.r, c.pA, c.G, c.P, c.S, c.zs, s->st);
    launch_init_beta_b(c.pA, c.G, c.ds, c.hist, c.S, c.zs, s->st);
}

// inner iterations [i0, i1) of the cycle (src/gmres.cu:566-717's loop body:
// w = M^-1 A v_i, MGS, Givens, residual check), every one gated per scenario
void enqueue_iters_b(const Ctx &c, int i0, int i1)
{
    gg_solver *s = c.s;
    for (int i = i0; i < i1; i++) {
        Gate gi;
        gi.done = &c.ds->done;
        gi.mask = ~0;
        gi.nit = &c.ds->nit;
        gi.i = i;
        const double *vi = c.V + (long long)i * c.P;
        launch_spmv_b(gi, s->dA, vi, nullptr, c.ww, false, c.S, c.zs, s->st);   // ww = A v_i
        trsv_pair(c, gi, c.ww, c.w);                                            // w = M^-1 ww
        if (c.B->persist) {
            // the persistent kernel: two scenarios per launch (k_arnoldi_persist2),
            // or one (k_arnoldi_persist) -- the same tree, the same bits
            for (int q = 0; q < c.S; q++) {
                Gate gq = gi;
                gq.done = zq(gi.done, c.zs, q);
                gq.nit = zq(gi.nit, c.zs, q);
                unsigned long long *gr = zq(c.gran, c.zs, q);
                if (c.B->persist2 && q + 1 < c.S) {
                    launch_arnoldi_persist2(gq, c.zs, i, c.m, zq(c.ds, c.zs, q), zq(c.w, c.zs, q), zq(c.V, c.zs, q), c.P,
                                            zq(c.H, c.zs, q), zq(c.cs, c.zs, q), zq(c.sn, c.zs, q),
                                            zq(c.sv, c.zs, q), zq(c.hist, c.zs, q),
                                            gr + (size_t)i * (c.m + 2) * c.G, c.G, c.P, s->err.p,
                                            zq(c.xgran, c.zs, q) + (size_t)i * (c.m + 2) * kMgsXcdWords,
                                            c.B->elect.p, ++c.B->seq, c.um, s->st);
                    q++;
                    continue;
                }
                launch_arnoldi_persist(gq, i, c.m, zq(c.ds, c.zs, q), zq(c.w, c.zs, q), zq(c.V, c.zs, q), c.P,
                                       zq(c.H, c.zs, q), zq(c.cs, c.zs, q), zq(c.sn, c.zs, q), zq(c.sv, c.zs, q),
                                       zq(c.hist, c.zs, q), gr + (size_t)i * (c.m + 2) * c.G,
                                       gr + (size_t)c.m * (c.m + 2) * c.G + (size_t)i * (c.m + 2), c.G, c.P,
                                       s->err.p, zq(c.xgran, c.zs, q) + (size_t)i * (c.m + 2) * kMgsXcdWords,
                                       c.B->elect.p, ++c.B->seq, c.um, s->st);
            }
            continue;
        }
        double *pin = c.pA, *pout = c.pB;
        launch_dot_b(gi, c.w, c.V, pin, c.G, c.P, c.S, c.zs, s->st);            // <w, v_0>
        for (int k = 0; k <= i; k++) {
            const double *vk = c.V + (long long)k * c.P;
            const double *vn = (k < i) ? c.V + (long long)(k + 1) * c.P : c.w;
            launch_mgs_step_b(gi, i, k, c.m, c.w, vk, vn, pin, pout, c.H, c.G, c.P, c.S, c.zs, s->st);
            std::swap(pin, pout);
        }
        launch_arnoldi_finalize_b(gi, i, c.m, c.ds, pin, c.G, c.w, c.V + (long long)(i + 1) * c.P, c.H, c.cs, c.sn,
                                  c.sv, c.hist, c.P, c.S, c.zs, s->st);
    }
}

// the cycle's tail: x += V y, r = M (b - A x), beta, history, j += nit
void enqueue_tail_b(const Ctx &c)
{
    gg_solver *s = c.s;
    Gate gu;
    gu.done = &c.ds->done;
    gu.mask = DONE_RESTART | DONE_INIT | DONE_ABORT | DONE_FINAL | DONE_EXH;
    launch_update_b(gu, c.m, c.ds, c.H, c.sv, c.y, c.V, c.P, c.xv, c.G, c.P, c.um, c.S, c.zs, s->st);
    Gate gr;
    gr.done = &c.ds->done;
    gr.mask = ~0;
    launch_spmv_b(gr, s->dA, c.xv, c.bv, c.rr, true, c.S, c.zs, s->st);
    trsv_pair(c, gr, c.rr, c.r);
    launch_dot_b(gr, c.r, c.r, c.pA, c.G, c.P, c.S, c.zs, s->st);
    launch_end_cycle_b(c.pA, c.G, c.ds, c.hist, c.S, c.zs, s->st);
}

int solve_batch_once(gg_solver *s, int S, const double *d_b, long long ldb, double *d_x, long long ldx,
                     const gg_options *opt, gg_result *res)
{
    const int m = opt->restart;
    const long long need = (long long)opt->max_iter + opt->max_iter / m + 4;
    ensure_batch(s, S, m, need);
    BatchWs *B = s->batch;
    if (!s->err.p) s->err.alloc(1);
    Ctx c;
    c.s = s;
    c.B = B;
    c.S = S;
    c.m = m;
    c.G = s->G;
    c.P = s->Ppad;
    c.zs = B->zs;
    c.um = solver_unit_map(s);
    c.ds = reinterpret_cast<DevState *>(B->arena.p + B->ods);
    c.V = B->dp(B->oV);
    c.w = B->dp(B->ow);
    c.ww = B->dp(B->oww);
    c.r = B->dp(B->or_);
    c.rr = B->dp(B->orr);
    c.bb = B->dp(B->obb);
    c.t1 = B->dp(B->ot1);
    c.xv = B->dp(B->oxv);
    c.bv = B->dp(B->obv);
    c.pA = B->dp(B->opA);
    c.pB = B->dp(B->opB);
    c.H = B->dp(B->oH);
    c.sv = B->dp(B->os);
    c.cs = B->dp(B->ocs);
    c.sn = B->dp(B->osn);
    c.y = B->dp(B->oy);
    c.hist = B->dp(B->ohist);
    c.Lg = reinterpret_cast<unsigned long long *>(B->arena.p + B->oLg);
    c.Ug = reinterpret_cast<unsigned long long *>(B->arena.p + B->oUg);
    c.gran = B->persist ? reinterpret_cast<unsigned long long *>(B->arena.p + B->ogran) : nullptr;
    c.xgran = B->persist ? reinterpret_cast<unsigned long long *>(B->arena.p + B->oxgran) : nullptr;
    hipStream_t st = s->st;

    // inputs into the solver's vector space; hand-off granules armed; control blocks
    launch_gather_b(d_b, ldb * 8, s->lay2nat.p, c.bv, c.zs, c.P, S, st);
    launch_gather_b(d_x, ldx * 8, s->lay2nat.p, c.xv, c.zs, c.P, S, st);
    launch_fill_u64_b(c.Lg, s->L.wl.ngran(), kSentinel, S, c.zs, st);
    launch_fill_u64_b(c.Ug, s->U.wl.ngran(), kSentinel, S, c.zs, st);
    launch_init_state_b(c.ds, c.zs, S, opt->tol, opt->max_iter, m, st);
    GG_HIP(hipMemsetAsync(s->err.p, 0, sizeof(int), st));
    GG_HIP(hipEventRecord(s->ev0, st));
    enqueue_init_b(c);

    std::vector<Track> tr(S);
    const int K = batch_chunk();
    int slot = 0;
    auto next_slot = [&]() {
        const int k = slot;
        slot = (slot + 1) % BatchWs::kSlots;
        return k;
    };
    if (opt->max_iter < 1) {
        // no cycle: converged at the start or max_iter exhausted (j = 1 > max_iter)
        const int k = next_slot();
        readback(s, B, k);
        const DevState *h = wait_slot(B, k);
        for (int q = 0; q < S; q++) {
            tr[q].fin = true;
            tr[q].relres = h[q].resid;
            tr[q].ret = (h[q].done & DONE_INIT) ? 0 : 1;
            tr[q].iters = (h[q].done & DONE_INIT) ? 0 : opt->max_iter;
        }
    }
    int left = 0;
    for (const Track &t : tr) left += !t.fin;
    while (left > 0) {
        // ---- one restart cycle, in chunks of K inner iterations
        launch_init_cycle_b(c.ds, c.r, c.V, c.sv, c.G, c.P, S, c.zs, st);
        if (B->persist) {
            launch_fill_u64_b(c.gran, B->ngran, kSentinel, S, c.zs, st);
            launch_fill_u64_b(c.xgran, B->nxgran, kSentinel, S, c.zs, st);
        }
        for (Track &t : tr) t.cyc_over = t.fin;
        std::deque<std::pair<int, int>> pend;              // (read-back slot, iterations enqueued)
        int issued = 0;
        auto chunk = [&]() {
            const int i1 = std::min(issued + K, m);
            enqueue_iters_b(c, issued, i1);
            issued = i1;
            const int k = next_slot();
            readback(s, B, k);
            pend.emplace_back(k, issued);
        };
        chunk();
        if (issued < m) chunk();
        const DevState *h = nullptr;
        while (true) {
            const auto [k, iend] = pend.front();
            pend.pop_front();
            h = wait_slot(B, k);
            for (int q = 0; q < S; q++)
                if (h[q].done & DONE_ABORT) throw BatchAbort{};
            bool over = true;
            for (int q = 0; q < S; q++) {
                Track &t = tr[q];
                if (t.cyc_over) continue;
                const int d = h[q].done;
                if ((d & (DONE_INIT | DONE_EXH | DONE_INNER | DONE_RESTART)) || iend >= h[q].nit) t.cyc_over = true;
                else over = false;
            }
            if (over) break;
            if (issued < m) chunk();
            GG_REQUIRE(!pend.empty(), GG_EHIP, "batched solve: cycle did not end after m iterations");
        }
        // the scenarios' outcomes as far as the last read-back decides them
        std::vector<DevState> hs(h, h + S);
        enqueue_tail_b(c);
        bool need_tail = false;
        for (int q = 0; q < S; q++) {
            Track &t = tr[q];
            if (t.fin) continue;
            const DevState &hq = hs[q];
            if (hq.done & DONE_INIT) {                      // converged at the start
                t.fin = true;
                t.ret = 0;
                t.iters = 0;
                t.hist_len = 1;
                t.relres = hq.resid;
            } else if (hq.done & DONE_INNER) {              // converged inside the cycle
                t.fin = true;
                t.ret = 0;
                t.restarts++;
                t.iters = t.prev_j + hq.conv_i;
                t.inner += hq.conv_i + 1;
                t.hist_len = hq.hist_len + hq.conv_i + 1;
                t.relres = hq.resid;
            } else {
                need_tail = true;
            }
        }
        if (need_tail) {
            const int k = next_slot();
            readback(s, B, k);
            const DevState *ht = wait_slot(B, k);
            for (int q = 0; q < S; q++) {
                Track &t = tr[q];
                if (t.fin) continue;
                const DevState &hq = ht[q];
                t.restarts++;
                t.inner += hq.nit;
                t.hist_len = hq.hist_len;
                t.relres = hq.resid;
                if (hq.done & DONE_RESTART) {
                    t.fin = true;
                    t.ret = 0;
                    t.iters = hq.j;
                } else if (hq.j > opt->max_iter) {          // while (j <= *max_iter) exhausted
                    t.fin = true;
                    t.ret = 1;
                    t.iters = opt->max_iter;                // the reference leaves *max_iter untouched
                } else {
                    t.prev_j = hq.j;
                }
            }
        }
        left = 0;
        for (const Track &t : tr) left += !t.fin;
    }
    GG_HIP(hipEventRecord(s->ev1, st));
    launch_gather_b(c.xv, c.zs, s->nat2lay.p, d_x, ldx * 8, s->A.n, S, st);
    {
        const int k = next_slot();
        readback(s, B, k);                      // the error word after every launch
        (void)wait_slot(B, k);
    }
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    int rc = GG_OK;
    for (int q = 0; q < S; q++) {
        const Track &t = tr[q];
        B->hist_len[q] = t.hist_len;
        if (t.ret) rc = 1;
        if (res) {
            res[q].status = t.ret;
            res[q].iters = t.iters;
            res[q].inner_iters = t.inner;
            res[q].restarts = t.restarts;
            res[q].relres = t.relres;
            res[q].solve_ms = ms;
        }
    }
    return rc;
}

// the solver object's own scenario-by-scenario engine (non-batchable
// configurations, GG_BATCH_SEQ=1)
int solve_batch_seq(gg_solver *s, int S, const double *d_b, long long ldb, double *d_x, long long ldx,
                    const gg_options *opt, gg_result *res)
{
    int rc = GG_OK;
    if (s->batch) s->batch->hist_len.assign(S, 0);
    for (int q = 0; q < S; q++) {
        gg_result r{};
        const int e = solve_one(s, d_b + (long long)q * ldb, d_x + (long long)q * ldx, opt, &r);
        if (e < 0) return e;
        if (e) rc = e;
        if (res) res[q] = r;
    }
    return rc;
}

}  // namespace

// the engine behind gg_solve_batch_device (also the transient batch's step)
int solve_batch(gg_solver *s, int S, const double *d_b, long long ldb, double *d_x, long long ldx,
                const gg_options *opt, gg_result *res)
{
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_solve_batch: no matrix (call gg_set_matrix)");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "gg_solve_batch: no preconditioner (call gg_set_precond_*)");
    GG_REQUIRE(opt, GG_EINVAL, "gg_solve_batch: null options");
    GG_REQUIRE(S >= 1, GG_EINVAL, "gg_solve_batch: nrhs must be >= 1");
    GG_REQUIRE(opt->restart >= 1 && opt->restart <= 512, GG_EINVAL, "gg_solve_batch: restart must be in [1, 512]");
    GG_REQUIRE(opt->max_iter >= 0, GG_EINVAL, "gg_solve_batch: negative max_iter");
    GG_REQUIRE(opt->flags == 0, GG_EINVAL, "gg_solve_batch: no flags are defined for the batch");
    GG_REQUIRE(ldb >= s->A.n && ldx >= s->A.n, GG_EINVAL, "gg_solve_batch: leading dimension below n");
    GG_HIP(hipSetDevice(s->device));
    if (!batchable(s)) return solve_batch_seq(s, S, d_b, ldb, d_x, ldx, opt, res);
    for (int attempt = 0;; attempt++) {
        try {
            return solve_batch_once(s, S, d_b, ldb, d_x, ldx, opt, res);
        } catch (BatchAbort &) {
            // not co-resident: the per-step kernels for the solver's life, repeat
            GG_HIP(hipStreamSynchronize(s->st));
            if (attempt >= 2) throw Error{GG_EHIP, "gg_solve_batch: fallbacks exhausted"};
            s->batch->persist = false;
            s->batch->persist2 = false;
        } catch (BatchErr &e) {
            // a WD_RCP range miss: IEEE division for the solver's life, repeat
            // (d_x is written only at the end)
            GG_HIP(hipStreamSynchronize(s->st));
            if (attempt >= 2) throw Error{GG_EHIP, "gg_solve_batch: fallbacks exhausted"};
            for (DevTri *T : {&s->L, &s->U})
                if (T->kind == DevTri::WAVE2D && T->div == WD_RCP) T->div = WD_HW;
        }
    }
}

bool batch_engine_on(gg_solver *s) { return batchable(s); }

long long batch_history(gg_solver *s, int q, double *out, long long cap)
{
    BatchWs *B = s->batch;
    GG_REQUIRE(B && q >= 0 && q < B->S && B->hist_len[q] > 0, GG_ESTATE,
               "gg_batch_history: no batched solve holds that scenario");
    const long long n = B->hist_len[q];
    if (out && cap > 0)
        GG_HIP(hipMemcpy(out, B->arena.p + (long long)q * B->zs + B->ohist, std::min(n, cap) * sizeof(double),
                         hipMemcpyDeviceToHost));
    return n;
}

}  // namespace gg

// ======================================================================= C ABI
namespace {
int fail_b(const gg::Error &e)
{
    gg::set_error(e.msg);
    return e.code;
}
}  // namespace
#define GG_BAPI_BEGIN try {
#define GG_BAPI_END                                                                 \
    }                                                                               \
    catch (const gg::Error &e) { return fail_b(e); }                                \
    catch (const std::bad_alloc &) { return fail_b({GG_ENOMEM, "host allocation failed"}); } \
    catch (const std::exception &e) { return fail_b({GG_EINVAL, e.what()}); }

using namespace gg;

extern "C" {

int gg_solve_batch_device(gg_solver *s, int nrhs, const double *d_b, long long ldb, double *d_x, long long ldx,
                          const gg_options *opt, gg_result *res)
{
    GG_BAPI_BEGIN
    GG_REQUIRE(s && d_b && d_x, GG_EINVAL, "null argument");
    return solve_batch(s, nrhs, d_b, ldb, d_x, ldx, opt, res);
    GG_BAPI_END
}

int gg_solve_batch(gg_solver *s, int nrhs, const double *b, long long ldb, double *x, long long ldx,
                   const gg_options *opt, gg_result *res)
{
    GG_BAPI_BEGIN
    GG_REQUIRE(s && b && x, GG_EINVAL, "null argument");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_solve_batch: no matrix");
    GG_REQUIRE(nrhs >= 1 && ldb >= s->A.n && ldx >= s->A.n, GG_EINVAL, "gg_solve_batch: bad nrhs / leading dimension");
    GG_HIP(hipSetDevice(s->device));
    const int n = s->A.n;
    DBuf<double> db, dx;
    db.alloc((size_t)nrhs * n);
    dx.alloc((size_t)nrhs * n);
    for (int q = 0; q < nrhs; q++) {
        GG_HIP(hipMemcpyAsync(db.p + (size_t)q * n, b + (size_t)q * ldb, n * sizeof(double), hipMemcpyHostToDevice, s->st));
        GG_HIP(hipMemcpyAsync(dx.p + (size_t)q * n, x + (size_t)q * ldx, n * sizeof(double), hipMemcpyHostToDevice, s->st));
    }
    const int rc = solve_batch(s, nrhs, db.p, n, dx.p, n, opt, res);
    for (int q = 0; q < nrhs; q++)
        GG_HIP(hipMemcpyAsync(x + (size_t)q * ldx, dx.p + (size_t)q * n, n * sizeof(double), hipMemcpyDeviceToHost, s->st));
    GG_HIP(hipStreamSynchronize(s->st));
    return rc;
    GG_BAPI_END
}

long long gg_batch_history(gg_solver *s, int rhs, double *out, long long cap)
{
    GG_BAPI_BEGIN
    GG_REQUIRE(s, GG_EINVAL, "null solver");
    return batch_history(s, rhs, out, cap);
    GG_BAPI_END
}

int gg_batch_engine(gg_solver *s)
{
    GG_BAPI_BEGIN
    GG_REQUIRE(s, GG_EINVAL, "null solver");
    GG_REQUIRE(s->pkind >= 0, GG_ESTATE, "gg_batch_engine: no preconditioner");
    return batch_engine_on(s) ? 1 : 0;
    GG_BAPI_END
}

int gg_transient_batch(gg_solver *s, int nrhs, int nsteps, double h, const double *cdiag, const int *src_off,
                       const int *src_node, const int *src_kind, const int *src_ptr, const double *src_data,
                       int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                       int *iters_total)
{
    GG_BAPI_BEGIN
    GG_REQUIRE(s && opt && x && cdiag && src_off && iters_total, GG_EINVAL, "null argument");
    GG_REQUIRE(s->have_A, GG_ESTATE, "gg_transient_batch: no matrix");
    GG_REQUIRE(nrhs >= 1 && nsteps >= 0 && nport >= 0, GG_EINVAL, "gg_transient_batch: bad count");
    GG_REQUIRE(nport == 0 || (port && port_out), GG_EINVAL, "null port arrays");
    const int n = s->A.n;
    GG_REQUIRE(src_off[0] == 0, GG_EINVAL, "gg_transient_batch: src_off[0] != 0");
    for (int q = 0; q < nrhs; q++) GG_REQUIRE(src_off[q + 1] >= src_off[q], GG_EINVAL, "gg_transient_batch: src_off not monotone");
    const int ns = src_off[nrhs];
    GG_REQUIRE(ns == 0 || (src_node && src_kind && src_ptr && src_data), GG_EINVAL, "null source arrays");
    int maxsrc = 0;
    std::vector<int> kind(std::max(ns, 1), GG_SRC_DC), dptr(ns + 1, 0);
    for (int q = 0; q < nrhs; q++) maxsrc = std::max(maxsrc, src_off[q + 1] - src_off[q]);
    for (int k = 0; k < ns; k++) {
        GG_REQUIRE(src_node[k] >= 0 && src_node[k] < n, GG_EINVAL, "source node out of range");
        const int len = src_ptr[k + 1] - src_ptr[k];
        GG_REQUIRE(src_ptr[k] >= 0 && len >= 0, GG_EINVAL, "transient: bad src_ptr");
        const int need = src_kind[k] == GG_SRC_DC ? 1 : src_kind[k] == GG_SRC_PULSE ? 7 : -1;
        GG_REQUIRE(src_kind[k] == GG_SRC_DC || src_kind[k] == GG_SRC_PULSE || src_kind[k] == GG_SRC_PWL, GG_EINVAL,
                   "transient: unknown source kind");
        GG_REQUIRE(need < 0 ? (len >= 2 && len % 2 == 0) : len == need, GG_EINVAL,
                   "transient: DC takes 1 value, PULSE 7, PWL (time, value) pairs");
        kind[k] = src_kind[k];
        dptr[k + 1] = src_ptr[k + 1] - src_ptr[0];
    }
    for (int j = 0; j < nport; j++) GG_REQUIRE(port[j] >= 0 && port[j] < n, GG_EINVAL, "port out of range");
    // per scenario, B^T by row: the scenario's sources of each row in ascending
    // index (cs_dl_gaxpy's column order, as gg_transient)
    std::vector<int> sptr((size_t)nrhs * (n + 1), 0), sidx(std::max(ns, 1));
    for (int q = 0; q < nrhs; q++) {
        int *sp = sptr.data() + (size_t)q * (n + 1);
        for (int k = src_off[q]; k < src_off[q + 1]; k++) sp[src_node[k] + 1]++;
        sp[0] = src_off[q];
        for (int r = 0; r < n; r++) sp[r + 1] += sp[r];
        std::vector<int> fill(sp, sp + n);
        for (int k = src_off[q]; k < src_off[q + 1]; k++) sidx[fill[src_node[k]]++] = k;
    }
    GG_HIP(hipSetDevice(s->device));
    hipStream_t st = s->st;
    DBuf<int> d_soff, d_kind, d_dptr, d_sptr, d_sidx, d_port;
    DBuf<double> d_data, d_u, d_c, d_x, d_w, d_pv;
    d_soff.upload(src_off, nrhs + 1, st);
    d_kind.upload(kind, st);
    d_dptr.upload(dptr, st);
    d_data.upload(ns ? src_data + src_ptr[0] : cdiag, ns ? (size_t)(src_ptr[ns] - src_ptr[0]) : 1, st);
    d_sptr.upload(sptr, st);
    d_sidx.upload(sidx, st);
    d_u.alloc(std::max(ns, 1));
    d_c.upload(cdiag, n, st);
    d_x.upload(x, (size_t)nrhs * n, st);
    d_w.alloc((size_t)nrhs * n);
    d_port.upload(port, nport, st);
    const long long ldo = (long long)nport * (nsteps + 1);
    d_pv.alloc((size_t)std::max<long long>(ldo * nrhs, 1));
    launch_gather_ports_b(nport, d_port.p, d_x.p, n, d_pv.p, ldo, nrhs, st);
    std::vector<gg_result> res(nrhs);
    std::vector<long long> tot(nrhs, 0);
    int status = GG_OK;
    for (int it = 1; it <= nsteps; it++) {
        launch_transient_step_b(n, nrhs, maxsrc, d_soff.p, d_kind.p, d_dptr.p, d_data.p, it, h, d_u.p, d_sptr.p,
                                d_sidx.p, d_c.p, d_x.p, d_w.p, n, st);
        const int rc = solve_batch(s, nrhs, d_w.p, n, d_x.p, n, opt, res.data());
        if (rc < 0) return rc;
        if (rc) status = rc;
        for (int q = 0; q < nrhs; q++) tot[q] += res[q].iters;
        launch_gather_ports_b(nport, d_port.p, d_x.p, n, d_pv.p + (long long)it * nport, ldo, nrhs, st);
    }
    if (nport) {
        std::vector<double> pv((size_t)ldo * nrhs);
        GG_HIP(hipMemcpyAsync(pv.data(), d_pv.p, pv.size() * sizeof(double), hipMemcpyDeviceToHost, st));
        GG_HIP(hipStreamSynchronize(st));
        for (int q = 0; q < nrhs; q++)
            for (int it = 0; it <= nsteps; it++)
                for (int j = 0; j < nport; j++)
                    port_out[((size_t)q * nport + j) * (nsteps + 1) + it] = pv[(size_t)q * ldo + (size_t)it * nport + j];
    }
    GG_HIP(hipMemcpyAsync(x, d_x.p, (size_t)nrhs * n * sizeof(double), hipMemcpyDeviceToHost, st));
    GG_HIP(hipStreamSynchronize(st));
    for (int q = 0; q < nrhs; q++) iters_total[q] = (int)std::min<long long>(tot[q], INT32_MAX);
    return status;
    GG_BAPI_END
}

}  // extern "C"
