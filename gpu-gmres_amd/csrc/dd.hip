// dd.hip -- sharded GMRES(m) + ILU(0) over P GPUs (include/ggmres_dd.h).
//
// Shard p's vector space (identical offsets on every shard):
//   [0, S0)        interior p rows in its own layout (3D/2D wavefront when the
//                  interior triangles are grid-shaped, else natural), zero padded
//   [S0, H0)       separator replica, in its own layout
//   [H0, Pl)       halo: P slots of maxI interface values (slot q = shard q's)
// Ops run over [0, H0); the dot range is [0, H0) on shard 0 (which counts the
// separator replica) and [0, S0) on the others, so the all-gathered block
// partials sum to the global dot, in one fixed order on every shard.
//
// Per Arnoldi iteration: pack+all-gather of v_i's interface (SpMV), of the
// forward solve's interface, and one 8*G-byte all-gather per MGS dot.
// The SpMV's exchange runs on a second stream beside the interior rows' SpMV
// (interior rows reference only their interior and the separator replica);
// the separator rows wait for it.  Everything else, RCCL collectives included,
// is enqueued on the main stream between the (gated) kernels, so a whole
// restart cycle is enqueued with one host read of the control block per
// cycle, as solver.hip.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>

#include "ggmres_dd.h"
#include "kernels.h"

using namespace gg;

#define GG_NCCL(call)                                                                       \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess)                                                              \
            throw ::gg::Error{GG_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)}; \
    } while (0)

namespace {

struct Shard {
    int p = 0, nI = 0, nS = 0;
    Wave2D wI, wS;
    std::vector<long long> slotI, slotS;    // region-local row -> region slot (host)
    long long PIr = 0, PSr = 0;             // region slot counts (multiples of 512)
    DevCsr AI, AS, LSH, UIS;                // A's interior rows [0, S0) and separator rows [S0, H0)
    DevTri LI, LS, UI, US;
    DBuf<long long> iface_slot;             // maxI: own interface slots (-1 pad)
    DBuf<long long> slot2nat;               // H0: natural row of each slot (-1 pad)
    DBuf<long long> own_slot, own_nat;      // rows this process writes back
    long long nown = 0;
    // workspace
    DBuf<double> V, w, ww, r, rr, bb, t1, t2, xv, bv, partA, partB, H, s, cs, sn, ysm, hist;
    DBuf<double> partC, hcgs;               // CGS2: P x (m+1) x G dot partials, the m+1 coefficients
    long long hist_cap = 0;
    DBuf<DevState> ds;
    DBuf<int> err;                          // P words (slot p is this shard's)
    double bytes_spmv = 0, bytes_trsv = 0;
    std::vector<long long> slot2perm;       // host: slot -> permuted global row (-1 pad), H0
    // the separator step as one k_sep_flow launch (LEVEL separator triangles):
    // tasks {first, count, phase} over rows = [L rows | U rows | interface rows]
    bool sepflow = false;
    int sf_ntask = 0;
    DBuf<int4> sf_tasks;
    DBuf<int> sf_rows;
};

using Get = std::function<double *(Shard &)>;

}  // namespace

struct gg_dd {
    int device = 0, P = 1, kind = GG_DD_LOCAL, rank = 0;
    ncclComm_t comm = nullptr;
    // GG_DD_IPC: this rank's exchange area (uncached device memory), every
    // rank's area as mapped here (hipIpcOpenMemHandle; own = ipc_area), the
    // per-exchange sequence number (identical on every rank: every rank
    // enqueues the same exchanges in the same order) and the error word
    void *ipc_area = nullptr;
    long long ipc_capd = 0;
    IpcPeers ipc{};
    bool ipc_connected = false;
    unsigned long long ipc_seq = 0;
    DBuf<int> xerr;
    // a peer timed out (xerr bit 4): the ranks' sequence numbers may now
    // differ, so the communicator is unusable -- every later exchange is
    // refused with GG_ESTATE (create a new gg_dd to recover)
    bool ipc_broken = false;
    // CGS2 / MGS with the exchanges inside the kernels (GG_DD_IPC /
    // GG_DD_LOOPBACK, P > 1, GG_DD_XK=1): the areas above (loopback: this
    // rank's own standing in for every peer's) and the reducers' hand-off
    // words (uncached)
    bool xk = false;
    bool xk_shared = false;                 // IPC peers on this rank's own GPU (tests)
    void *xk_local = nullptr;
    Xch xch{};
    hipStream_t st = nullptr;
    hipStream_t st2 = nullptr;              // the SpMV's interface exchange, beside the interior rows
    bool halo_inline = true;                // GG_DD_HALO_INLINE=0: the exchange on st2 beside the interior rows
    // GG_DD_IPC / LOOPBACK: the exchange and both row sets in one launch
    // (k_dd_spmv_x; GG_DD_HALO_FUSED=0: the exchange, then the rows, in line)
    bool halo_fused = true;
    DBuf<unsigned long long> arrived;       // k_dd_spmv_x's exchange blocks, counted over its launches
    unsigned long long fused_epoch = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evx = nullptr, evh = nullptr;
    bool have = false;
    int n = 0, nsep = 0, maxI = 0;
    std::vector<int> pinv, q;
    long long S0 = 0, H0 = 0, Pl = 0;
    int G = 1;
    std::vector<std::unique_ptr<Shard>> sh;
    int m_alloc = -1;
    bool cgs2 = false;                      // GG_SOLVE_CGS2 for the solve in progress
    int div_mode = GG_DIV_EXACT;            // gg_dd_set_division (the shards' wavefront solves)
    std::vector<double> last_hist;
    DBuf<double> nat_a, nat_b;
    DBuf<long long> dtmp;
    // in-solve timing (gg_dd_profile_*): hipEvent pairs on the solver's stream
    // around each family of an inner iteration, accounted for the iterations
    // that really ran (as the single solver's gg_profile_*)
    int prof_mask = 0;
    std::vector<hipEvent_t> prof_pool;
    size_t prof_used = 0;
    struct Mark { int kind, i, e0, e1; };
    std::vector<Mark> marks;
    double prof_ms[GG_DD_PROF_NKINDS] = {};
    long long prof_cnt[GG_DD_PROF_NKINDS] = {};
};

namespace {

int fail(const Error &e)
{
    set_error(e.msg);
    return e.code;
}
#define GG_API_BEGIN try {
#define GG_API_END                                                                          \
    }                                                                                       \
    catch (const gg::Error &e) { return fail(e); }                                          \
    catch (const std::bad_alloc &) { return fail({GG_ENOMEM, "host allocation failed"}); } \
    catch (const std::exception &e) { return fail({GG_EINVAL, e.what()}); }

void set_dev(gg_dd *d) { GG_HIP(hipSetDevice(d->device)); }

Gate gate_i(Shard &s, int i)
{
    Gate g;
    g.done = &s.ds.p->done;
    g.mask = ~0;
    g.nit = &s.ds.p->nit;
    g.i = i;
    return g;
}
Gate gate_mask(Shard &s, int mask)
{
    Gate g;
    g.done = &s.ds.p->done;
    g.mask = mask;
    return g;
}

// GG_DD_IPC: enqueue one all-gather of cnt doubles (slot q at buf + q*cnt)
void ipc_allgather(gg_dd *d, double *buf, long long cnt, hipStream_t st)
{
    GG_REQUIRE(d->ipc_connected, GG_ESTATE, "dd: IPC exchange used before gg_dd_ipc_connect");
    GG_REQUIRE(!d->ipc_broken, GG_ESTATE,
               "dd: IPC communicator unusable after a peer timeout (create a new gg_dd)");
    GG_REQUIRE(cnt <= d->ipc_capd, GG_EINVAL,
               "dd: IPC exchange of " + std::to_string(cnt) + " doubles exceeds the area's " +
                   std::to_string(d->ipc_capd) + " per rank (GG_DD_IPC_CAP)");
    launch_ipc_allgather(d->ipc, d->rank, d->P, buf, cnt, ++d->ipc_seq, d->ipc_capd, d->xerr.p, st);
}
void ipc_check(gg_dd *d)
{
    int e = 0;
    GG_HIP(hipMemcpyAsync(&e, d->xerr.p, sizeof(int), hipMemcpyDeviceToHost, d->st));
    GG_HIP(hipStreamSynchronize(d->st));
    if (e & 4) {
        d->ipc_broken = true;
        throw Error{GG_ETIMEOUT, "dd: IPC exchange: a peer did not arrive within 30 s "
                                 "(the communicator is unusable from here on)"};
    }
}
// GG_DD_IPC, host-synchronous (setup, error checks): every rank's value
std::vector<long long> ipc_allgather_host(gg_dd *d, long long v)
{
    DBuf<double> b;
    b.alloc(d->P);
    GG_HIP(hipMemsetAsync(b.p, 0, d->P * sizeof(double), d->st));
    GG_HIP(hipMemcpyAsync(b.p + d->rank, &v, sizeof(v), hipMemcpyHostToDevice, d->st));
    ipc_allgather(d, b.p, 1, d->st);
    std::vector<long long> out(d->P);
    GG_HIP(hipMemcpyAsync(out.data(), b.p, d->P * sizeof(long long), hipMemcpyDeviceToHost, d->st));
    ipc_check(d);
    return out;
}

// max over all shards of all processes (setup only: host-synchronous)
long long agree_max(gg_dd *d, long long v)
{
    if (d->kind == GG_DD_IPC && d->P > 1) {
        for (long long w : ipc_allgather_host(d, v)) v = std::max(v, w);
        return v;
    }
    if (d->kind != GG_DD_RCCL || d->P == 1) return v;
    DBuf<long long> b;
    b.alloc(1);
    GG_HIP(hipMemcpyAsync(b.p, &v, sizeof(v), hipMemcpyHostToDevice, d->st));
    GG_NCCL(ncclAllReduce(b.p, b.p, 1, ncclInt64, ncclMax, d->comm, d->st));
    GG_HIP(hipMemcpyAsync(&v, b.p, sizeof(v), hipMemcpyDeviceToHost, d->st));
    GG_HIP(hipStreamSynchronize(d->st));
    return v;
}

// all-gather of the slot each shard owns in buf(s) + off: slot q at off + q*cnt
void exchange(gg_dd *d, const Get &buf, long long off, long long cnt, hipStream_t st)
{
    if (d->P == 1 || cnt == 0) return;
    if (d->kind == GG_DD_RCCL) {
        Shard &s = *d->sh[0];
        double *b = buf(s) + off;
        GG_NCCL(ncclAllGather(b + (long long)s.p * cnt, b, (size_t)cnt, ncclDouble, d->comm, st));
    } else if (d->kind == GG_DD_IPC) {
        ipc_allgather(d, buf(*d->sh[0]) + off, cnt, st);
    } else if (d->kind == GG_DD_LOOPBACK) {
        // the one shard's buffer as every shard's: the all-gather kernel's
        // traffic and launch, no peer values (timing only)
        ShardPtrs ptr{};
        for (int q = 0; q < d->P; q++) ptr.p[q] = buf(*d->sh[0]);
        launch_allgather_local(ptr, d->P, off, cnt, st);
    } else {
        ShardPtrs ptr{};
        for (int q = 0; q < d->P; q++) ptr.p[q] = buf(*d->sh[q]);
        launch_allgather_local(ptr, d->P, off, cnt, st);
    }
}
void exchange(gg_dd *d, const Get &buf, long long off, long long cnt) { exchange(d, buf, off, cnt, d->st); }
// every shard's interface values of vector x -> every shard's halo slots
// (x + H0 + q*maxI), and (f0 / f1, nf > 0) nf words of two vectors of every
// shard set to the sentinel: the gather in the exchange's launch where the
// exchange is a kernel of ours (GG_DD_LOCAL / LOOPBACK / IPC: one launch instead
// of a gather per shard plus the all-gather), RCCL: gathers + ncclAllGather
void gather_exchange(gg_dd *d, const Get &x, hipStream_t st, const Get &f0 = Get{}, const Get &f1 = Get{},
                     long long nf = 0)
{
    const long long H0 = d->H0, mI = d->maxI;
    if (d->kind == GG_DD_RCCL) {
        for (auto &sp : d->sh) {
            Shard &s = *sp;
            double *v = x(s);
            launch_gather(v, s.iface_slot.p, v + H0 + (long long)s.p * mI, mI, st, f0 ? f0(s) : nullptr,
                          f1 ? f1(s) : nullptr, nf);
        }
        exchange(d, x, H0, mI, st);
        return;
    }
    if (d->kind == GG_DD_IPC) {
        Shard &s = *d->sh[0];
        launch_ipc_gather_allgather(d->ipc, d->rank, d->P, x(s), s.iface_slot.p, x(s) + H0, mI, ++d->ipc_seq,
                                    d->ipc_capd, d->xerr.p, f0 ? f0(s) : nullptr, f1 ? f1(s) : nullptr, nf, st);
        return;
    }
    ShardPtrs b{};
    IdxPtrs gi{};
    FillPtrs fl{};
    if (d->kind == GG_DD_LOOPBACK) {
        Shard &s = *d->sh[0];
        for (int q = 0; q < d->P; q++) {
            b.p[q] = x(s);
            gi.p[q] = s.iface_slot.p;
        }
        fl.f0[0] = f0 ? f0(s) : nullptr;
        fl.f1[0] = f1 ? f1(s) : nullptr;
    } else {
        for (auto &sp : d->sh) {
            Shard &s = *sp;
            b.p[s.p] = x(s);
            gi.p[s.p] = s.iface_slot.p;
            fl.f0[s.p] = f0 ? f0(s) : nullptr;
            fl.f1[s.p] = f1 ? f1(s) : nullptr;
        }
    }
    launch_gather_allgather_local(b, gi, d->P, H0, mI, fl, nf, st);
}
// own interface values of vector x -> halo slot p, then the all-gather
void halo(gg_dd *d, const Get &x, hipStream_t st)
{
    if (d->maxI == 0 || d->P == 1) return;
    gather_exchange(d, x, st);
}

Get vec(DBuf<double> Shard::*m) { return [m](Shard &s) { return (s.*m).p; }; }

// ---- in-solve profiling ------------------------------------------------------
int prof_event(gg_dd *d)
{
    if (d->prof_used == d->prof_pool.size()) {
        hipEvent_t e;
        GG_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));   // timing only
        d->prof_pool.push_back(e);
    }
    GG_HIP(hipEventRecord(d->prof_pool[d->prof_used], d->st));
    return (int)d->prof_used++;
}
int prof_begin(gg_dd *d, int kind, int i)
{
    if (i < 0 || !((d->prof_mask >> kind) & 1)) return -1;
    d->marks.push_back({kind, i, prof_event(d), -1});
    return (int)d->marks.size() - 1;
}
void prof_end(gg_dd *d, int mark)
{
    if (mark >= 0) d->marks[mark].e1 = prof_event(d);
}
void prof_collect(gg_dd *d, int executed)
{
    if (!d->prof_mask) return;
    for (const auto &mk : d->marks) {
        if (mk.i >= executed || mk.e1 < 0) continue;
        float ms = 0.f;
        GG_HIP(hipEventElapsedTime(&ms, d->prof_pool[mk.e0], d->prof_pool[mk.e1]));
        d->prof_ms[mk.kind] += ms;
        d->prof_cnt[mk.kind]++;
    }
    d->marks.clear();
    d->prof_used = 0;
}

// gate of a phase: inner iteration gi (>= 0), else the done-mask (0 = ungated)
Gate gate_of(Shard &s, int gi, int mask)
{
    return gi >= 0 ? gate_i(s, gi) : (mask ? gate_mask(s, mask) : Gate{});
}

// z = (LU)^-1 y of the arrow-ordered ILU(0), per shard (module comment of host/dd_setup.cpp)
void apply_minv(gg_dd *d, int gi, int mask, const Get &in, const Get &out)
{
    const long long S0 = d->S0;
    auto gate = [&](Shard &s) { return gate_of(s, gi, mask); };
    int mk = prof_begin(d, GG_DD_PROF_TRSV_L, gi);
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        for (DevTri *T : {&s.LI, &s.LS, &s.UI, &s.US}) T->fast = d->div_mode;
        launch_trsv(gate(s), s.LI, in(s), s.t1.p, s.err.p + s.p, d->st);          // y_I
    }
    prof_end(d, mk);
    mk = prof_begin(d, GG_DD_PROF_SEP, gi);
    // interface y (halo); the fused separator step's sentinel fills ride on the gathers
    const bool xch = d->maxI > 0 && d->P > 1;
    if (xch) {
        // (the separator is replicated: nS is the same on every shard)
        const Shard &s0 = *d->sh[0];
        gather_exchange(d, vec(&Shard::t1), d->st, [S0](Shard &s) { return s.sepflow ? s.t1.p + S0 : nullptr; },
                        [S0, &out](Shard &s) { return s.sepflow ? out(s) + S0 : nullptr; },
                        s0.sepflow ? s0.nS : 0);
    } else {
        for (auto &sp : d->sh) {
            Shard &s = *sp;
            if (s.sepflow) launch_gather(s.t1.p, s.iface_slot.p, s.t1.p, 0, d->st, s.t1.p + S0, out(s) + S0, s.nS);
        }
    }
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        Gate g = gate(s);
        if (s.sepflow) {
            // b_S - L_SI y_I and the separator L solve, the separator U solve,
            // y_I - U_IS x_S (in place in t1): one launch, the same bits
            SepFlow f;
            f.ph[0] = SepPhase{s.LS.off.rp.p, s.LS.off.ci.p, s.LS.off.v.p, s.t1.p + S0, s.LSH.rp.p, s.LSH.ci.p,
                               s.LSH.v.p, s.t1.p, in(s) + S0, s.LS.d.p, s.t1.p + S0, false};
            f.ph[1] = SepPhase{s.US.off.rp.p, s.US.off.ci.p, s.US.off.v.p, out(s) + S0, nullptr, nullptr,
                               nullptr, nullptr, s.t1.p + S0, s.US.d.p, out(s) + S0, true};
            f.ph[2] = SepPhase{s.UIS.rp.p, s.UIS.ci.p, s.UIS.v.p, out(s), nullptr, nullptr,
                               nullptr, nullptr, s.t1.p, nullptr, s.t1.p, false};
            launch_sep_flow(g, s.sf_ntask, s.sf_tasks.p, s.sf_rows.p, f, s.err.p + s.p, d->st);
            continue;
        }
        // the separator solves' sentinel fills ride on the subtraction's launch
        const bool pre = s.LS.kind == DevTri::LEVEL && s.US.kind == DevTri::LEVEL && s.LS.n == s.US.n;
        launch_sub_seq(g, s.LSH, s.t1.p, in(s) + S0, s.t2.p + S0, d->st,                // b_S - L_SI y_I
                       pre ? s.t1.p + S0 : nullptr, pre ? out(s) + S0 : nullptr, pre ? s.LS.n : 0);
        s.LS.prefilled = s.US.prefilled = pre;
        launch_trsv(g, s.LS, s.t2.p + S0, s.t1.p + S0, s.err.p + s.p, d->st);     // y_S
        launch_trsv(g, s.US, s.t1.p + S0, out(s) + S0, s.err.p + s.p, d->st);     // x_S
        s.LS.prefilled = s.US.prefilled = false;
        launch_sub_seq(g, s.UIS, out(s), s.t1.p, s.t2.p, d->st);                  // y_I - U_IS x_S
    }
    prof_end(d, mk);
    mk = prof_begin(d, GG_DD_PROF_TRSV_U, gi);
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        launch_trsv(gate(s), s.UI, s.sepflow ? s.t1.p : s.t2.p, out(s), s.err.p + s.p, d->st);   // x_I
    }
    prof_end(d, mk);
}

// y = A x (b = null) or y = b - A x: the interior rows reference only their
// own interior and the separator replica, so they run on the main stream while
// the interface exchange runs on the second; the separator rows follow it
void spmv_rows(gg_dd *d, const Get &x, const Get &b, const Get &y, bool resid,
               const std::function<Gate(Shard &)> &gate)
{
    const long long S0 = d->S0;
    const bool xch = d->maxI > 0 && d->P > 1;
    if (xch && d->halo_inline && d->halo_fused && d->sh.size() == 1 &&
        (d->kind == GG_DD_IPC || d->kind == GG_DD_LOOPBACK)) {
        // exchange, interior rows and separator rows in one launch (k_dd_spmv_x)
        Shard &s = *d->sh[0];
        if (!d->arrived.p) {
            d->arrived.alloc(1);
            GG_HIP(hipMemsetAsync(d->arrived.p, 0, sizeof(unsigned long long), d->st));
        }
        DdSpmvCall c;
        c.me = d->rank;
        c.P = d->P;
        c.loop = d->kind == GG_DD_LOOPBACK;
        c.resid = resid;
        c.halo = x(s) + d->H0;
        c.cnt = d->maxI;
        c.gidx = s.iface_slot.p;
        c.arrived = d->arrived.p;
        c.AI = &s.AI;
        c.AS = &s.AS;
        c.x = x(s);
        c.b = resid ? b(s) : nullptr;
        c.y = y(s);
        c.S0 = S0;
        if (!c.loop) {
            GG_REQUIRE(d->ipc_connected, GG_ESTATE, "dd: IPC exchange used before gg_dd_ipc_connect");
            GG_REQUIRE(!d->ipc_broken, GG_ESTATE,
                       "dd: IPC communicator unusable after a peer timeout (create a new gg_dd)");
            GG_REQUIRE(c.cnt <= d->ipc_capd, GG_EINVAL, "dd: IPC halo exceeds the exchange area (GG_DD_IPC_CAP)");
            c.pp = d->ipc;
            c.capd = d->ipc_capd;
            c.err = d->xerr.p;
            c.seq = d->ipc_seq + 1;
        } else {
            c.err = d->xerr.p;
        }
        c.epoch = d->fused_epoch + 1;
        if (launch_dd_spmv_x(gate(s), c, d->st)) {
            if (!c.loop) d->ipc_seq++;
            d->fused_epoch++;
            return;
        }
    }
    if (xch && d->halo_inline) {
        // the exchange in line on the solver's stream: no cross-stream event
        // wait pair per SpMV (GG_DD_HALO_INLINE)
        halo(d, x, d->st);
        for (auto &sp : d->sh) {
            Shard &s = *sp;
            launch_spmv(gate(s), s.AI, x(s), resid ? b(s) : nullptr, y(s), resid, d->st);
            launch_spmv(gate(s), s.AS, x(s), resid ? b(s) + S0 : nullptr, y(s) + S0, resid, d->st);
        }
        return;
    }
    if (xch) {
        GG_HIP(hipEventRecord(d->evx, d->st));              // x complete
        GG_HIP(hipStreamWaitEvent(d->st2, d->evx, 0));
        halo(d, x, d->st2);
        GG_HIP(hipEventRecord(d->evh, d->st2));
    }
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        launch_spmv(gate(s), s.AI, x(s), resid ? b(s) : nullptr, y(s), resid, d->st);
    }
    if (xch) GG_HIP(hipStreamWaitEvent(d->st, d->evh, 0));
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        launch_spmv(gate(s), s.AS, x(s), resid ? b(s) + S0 : nullptr, y(s) + S0, resid, d->st);
    }
}
void spmv(gg_dd *d, int gi, const Get &x, const Get &y)   // y = A x
{
    spmv_rows(d, x, Get{}, y, false, [&](Shard &s) { return gate_of(s, gi, 0); });
}
void resid(gg_dd *d, int mask)   // rr = b - A x
{
    spmv_rows(d, vec(&Shard::xv), vec(&Shard::bv), vec(&Shard::rr), true,
              [&](Shard &s) { return gate_of(s, -1, mask); });
}
long long dot_len(gg_dd *d, const Shard &s) { return s.p == 0 ? d->H0 : d->S0; }

// block partials of <a, b> into part slot p, then the all-gather
void dot(gg_dd *d, int gi, int mask, const Get &a, const Get &b, DBuf<double> Shard::*part)
{
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        launch_dot(gate_of(s, gi, mask), a(s), b(s), (s.*part).p + (long long)s.p * d->G, d->G, dot_len(d, s), d->st);
    }
    exchange(d, vec(part), 0, d->G);
}

void ensure_workspace(gg_dd *d, int m)
{
    if (d->m_alloc == m) return;
    const long long Pl = d->Pl;
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        s.V.alloc((size_t)(m + 1) * Pl);
        GG_HIP(hipMemsetAsync(s.V.p, 0, (size_t)(m + 1) * Pl * sizeof(double), d->st));
        for (DBuf<double> *b : {&s.w, &s.ww, &s.r, &s.rr, &s.bb, &s.t1, &s.t2, &s.xv, &s.bv}) {
            b->alloc(Pl);
            GG_HIP(hipMemsetAsync(b->p, 0, Pl * sizeof(double), d->st));
        }
        for (DBuf<double> *b : {&s.partA, &s.partB}) {
            b->alloc((size_t)d->P * d->G);
            GG_HIP(hipMemsetAsync(b->p, 0, (size_t)d->P * d->G * sizeof(double), d->st));
        }
        s.H.alloc((size_t)(m + 1) * m);
        GG_HIP(hipMemsetAsync(s.H.p, 0, (size_t)(m + 1) * m * sizeof(double), d->st));
        // two halves: the first and the second pass's partials (in-kernel
        // exchanges: a launch reads one while it writes the other)
        s.partC.alloc((size_t)2 * d->P * (m + 1) * d->G);
        GG_HIP(hipMemsetAsync(s.partC.p, 0, (size_t)2 * d->P * (m + 1) * d->G * sizeof(double), d->st));
        s.hcgs.alloc(m + 1);
        s.s.alloc(m + 1);
        s.cs.alloc(m + 1);
        s.sn.alloc(m + 1);
        s.ysm.alloc(m + 1);
        if (!s.ds.p) s.ds.alloc(1);
        if (!s.err.p) s.err.alloc(d->P);
    }
    d->m_alloc = m;
}

// the in-kernel CGS2 exchanges apply (one shard per process, the dots of
// inner iteration nk - 1 within the kernels' and the area's range)
bool use_xk(gg_dd *d, int nk)
{
    // several ranks on one GPU: a rank's waiting blocks must not starve a
    // peer's producer of CUs -- only when every rank's grid fits one block per CU
    if (d->xk_shared && (long long)d->P * d->G > 256) return false;
    return d->xk && d->sh.size() == 1 && nk <= kCgsXMax &&
           (long long)d->G * ((kCgsXMax + kCgsKC - 1) / kCgsKC) <= kIpcXF && (long long)nk * d->G <= d->ipc_capd &&
           (long long)d->G <= d->ipc_capd;
}

void enqueue_init(gg_dd *d)
{
    apply_minv(d, -1, 0, vec(&Shard::bv), vec(&Shard::bb));                    // bb = M b
    dot(d, -1, 0, vec(&Shard::bb), vec(&Shard::bb), &Shard::partA);
    for (auto &sp : d->sh) launch_set_normb(sp->partA.p, d->P * d->G, sp->ds.p, d->st);
    resid(d, 0);                                                                // rr = b - A x
    apply_minv(d, -1, 0, vec(&Shard::rr), vec(&Shard::r));                     // r = M rr
    dot(d, -1, 0, vec(&Shard::r), vec(&Shard::r), &Shard::partA);
    for (auto &sp : d->sh) launch_init_beta(sp->partA.p, d->P * d->G, sp->ds.p, sp->hist.p, d->st);
}

void enqueue_cycle(gg_dd *d, int m)
{
    const long long Pl = d->Pl, H0 = d->H0;
    const int NP = d->P * d->G;
    for (auto &sp : d->sh) launch_init_cycle(sp->ds.p, sp->r.p, sp->V.p, sp->s.p, d->G, H0, d->st);
    for (int i = 0; i < m; i++) {
        const Get vi = [i, Pl](Shard &s) { return s.V.p + (long long)i * Pl; };
        int mk = prof_begin(d, GG_DD_PROF_SPMV, i);
        spmv(d, i, vi, vec(&Shard::ww));                                        // ww = A v_i
        prof_end(d, mk);
        apply_minv(d, i, 0, vec(&Shard::ww), vec(&Shard::w));                   // w = M^-1 ww
        mk = prof_begin(d, GG_DD_PROF_ORTH, i);
        if (d->cgs2 && use_xk(d, i + 1)) {
            // CGS2 with the exchanges inside four launches (Xch): the same
            // values as below, exchange sequence numbers shared with ipc_allgather
            Shard &s = *d->sh[0];
            const int nk = i + 1;
            const long long cnt = (long long)nk * d->G;
            const long long half = (long long)d->P * (m + 1) * d->G;
            double *p1 = s.partC.p + (long long)s.p * cnt, *p2 = s.partC.p + half + (long long)s.p * cnt;
            double *pn = s.partA.p + (long long)s.p * d->G;
            const unsigned long long q1 = ++d->ipc_seq, q2 = ++d->ipc_seq, q3 = ++d->ipc_seq;
            const Gate gt = gate_i(s, i);
            launch_multidot_x(gt, s.w.p, s.V.p, Pl, nk, p1, d->G, dot_len(d, s), d->xch, q1, d->st);
            launch_cgs_update_x(gt, s.w.p, s.V.p, Pl, nk, d->G, H0, dot_len(d, s), p1, q1, s.H.p, i, m, false, p2,
                                nullptr, d->xch, q2, d->st);
            launch_cgs_update_x(gt, s.w.p, s.V.p, Pl, nk, d->G, H0, dot_len(d, s), p2, q2, s.H.p, i, m, true,
                                nullptr, pn, d->xch, q3, d->st);
            launch_arnoldi_finalize_x(gt, i, m, s.ds.p, pn, q3, d->G, s.w.p, s.V.p + (long long)(i + 1) * Pl, s.H.p,
                                      s.cs.p, s.sn.p, s.s.p, s.hist.p, H0, d->xch, d->st);
            prof_end(d, mk);
            continue;
        }
        if (d->cgs2) {
            // CGS2: h = V^T w, w -= V h, h2 = V^T w, w -= V h2 (+ the norm's
            // partials), H[:, i] = h + h2 -- three all-gathers
            // (the first update and the second pass's partials in one sweep,
            // k_cgs_update_dot, while i + 1 <= 32)
            const long long cnt = (long long)(i + 1) * d->G;
            bool have_partials = false;
            for (int pass = 0; pass < 2; pass++) {
                if (!have_partials) {
                    for (auto &sp : d->sh) {
                        Shard &s = *sp;
                        launch_multidot(gate_i(s, i), s.w.p, s.V.p, Pl, i + 1, s.partC.p + (long long)s.p * cnt,
                                        d->G, dot_len(d, s), d->st);
                    }
                }
                exchange(d, vec(&Shard::partC), 0, cnt);
                have_partials = false;
                for (auto &sp : d->sh) {
                    Shard &s = *sp;
                    launch_cgs_reduce(gate_i(s, i), s.partC.p, d->P, d->G, cnt, i + 1, s.hcgs.p, s.H.p, i, m,
                                      pass == 1, d->st);
                    if (pass == 0 && launch_cgs_update_dot(gate_i(s, i), s.w.p, s.V.p, Pl, s.hcgs.p, i + 1, d->G,
                                                           H0, dot_len(d, s),
                                                           s.partC.p + (long long)s.p * cnt, d->st)) {
                        have_partials = true;
                        continue;
                    }
                    launch_cgs_update(gate_i(s, i), s.w.p, s.V.p, Pl, s.hcgs.p, i + 1, d->G, H0, dot_len(d, s),
                                      pass == 1 ? s.partA.p + (long long)s.p * d->G : nullptr, d->st);
                }
            }
            exchange(d, vec(&Shard::partA), 0, d->G);
            for (auto &sp : d->sh) {
                Shard &s = *sp;
                launch_arnoldi_finalize_r(gate_i(s, i), i, m, s.ds.p, s.partA.p, NP, d->G, s.w.p,
                                          s.V.p + (long long)(i + 1) * Pl, s.H.p, s.cs.p, s.sn.p, s.s.p,
                                          s.hist.p, H0, d->st);
            }
            prof_end(d, mk);
            continue;
        }
        if (use_xk(d, 1)) {
            // MGS on the in-kernel exchanges: i + 3 launches
            Shard &s = *d->sh[0];
            const Gate gt = gate_i(s, i);
            double *pa = s.partA.p + (long long)s.p * d->G, *pb = s.partB.p + (long long)s.p * d->G;
            unsigned long long q = ++d->ipc_seq;
            launch_dot_x(gt, s.w.p, s.V.p, pa, d->G, dot_len(d, s), d->xch, q, d->st);
            for (int k = 0; k <= i; k++) {
                const double *vk = s.V.p + (long long)k * Pl;
                const double *vn = (k < i) ? s.V.p + (long long)(k + 1) * Pl : nullptr;
                const unsigned long long qn = ++d->ipc_seq;
                launch_mgs_step_x(gt, i, k, m, s.w.p, vk, vn, pa, q, pb, s.H.p, d->G, H0, dot_len(d, s), d->xch, qn,
                                  d->st);
                std::swap(pa, pb);
                q = qn;
            }
            launch_arnoldi_finalize_x(gt, i, m, s.ds.p, pa, q, d->G, s.w.p, s.V.p + (long long)(i + 1) * Pl, s.H.p,
                                      s.cs.p, s.sn.p, s.s.p, s.hist.p, H0, d->xch, d->st);
            prof_end(d, mk);
            continue;
        }
        dot(d, i, 0, vec(&Shard::w), [](Shard &s) { return s.V.p; }, &Shard::partA);
        DBuf<double> Shard::*pin = &Shard::partA, Shard::*pout = &Shard::partB;
        for (int k = 0; k <= i; k++) {
            for (auto &sp : d->sh) {
                Shard &s = *sp;
                const double *vk = s.V.p + (long long)k * Pl;
                const double *vn = (k < i) ? s.V.p + (long long)(k + 1) * Pl : s.w.p;
                launch_mgs_step_r(gate_i(s, i), i, k, m, s.w.p, vk, vn, (s.*pin).p, NP,
                                  (s.*pout).p + (long long)s.p * d->G, s.H.p, d->G, H0,
                                  dot_len(d, s), d->st);
            }
            exchange(d, vec(pout), 0, d->G);
            std::swap(pin, pout);
        }
        for (auto &sp : d->sh) {
            Shard &s = *sp;
            launch_arnoldi_finalize_r(gate_i(s, i), i, m, s.ds.p, (s.*pin).p, NP, d->G, s.w.p,
                                      s.V.p + (long long)(i + 1) * Pl, s.H.p, s.cs.p, s.sn.p, s.s.p,
                                      s.hist.p, H0, d->st);
        }
        prof_end(d, mk);
    }
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        launch_update(gate_mask(s, DONE_RESTART | DONE_INIT), m, s.ds.p, s.H.p, s.s.p, s.ysm.p, s.V.p,
                      Pl, s.xv.p, d->G, H0, d->st);
    }
    resid(d, ~0);                                                               // rr = b - A x
    apply_minv(d, -1, ~0, vec(&Shard::rr), vec(&Shard::r));
    dot(d, -1, ~0, vec(&Shard::r), vec(&Shard::r), &Shard::partA);
    for (auto &sp : d->sh) launch_end_cycle(sp->partA.p, NP, sp->ds.p, sp->hist.p, d->st);
}

DevState read_state(gg_dd *d)
{
    std::vector<DevState> h(d->sh.size());
    for (size_t k = 0; k < d->sh.size(); k++)
        GG_HIP(hipMemcpyAsync(&h[k], d->sh[k]->ds.p, sizeof(DevState), hipMemcpyDeviceToHost, d->st));
    GG_HIP(hipStreamSynchronize(d->st));
    for (size_t k = 1; k < h.size(); k++)     // the replicas must agree bit for bit
        GG_REQUIRE(std::memcmp(&h[k].resid, &h[0].resid, sizeof(double)) == 0 &&
                       h[k].done == h[0].done && h[k].j == h[0].j,
                   GG_EINVAL, "dd: shard control blocks diverged");
    return h[0];
}

// err bit 1: WD_RCP range (divide instead), bit 3: a static tile grid was not
// co-resident (claim tiles from the queue) -- apply_fallback, then repeat
struct Fallback {
    int bits;
};
void check_err(gg_dd *d)
{
    int any = 0;
    if (d->kind == GG_DD_RCCL && d->P > 1) {
        Shard &s = *d->sh[0];
        GG_NCCL(ncclAllGather(s.err.p + s.p, s.err.p, 1, ncclInt32, d->comm, d->st));
    }
    if (d->kind == GG_DD_LOOPBACK && d->xk) ipc_check(d);
    if (d->kind == GG_DD_IPC) {
        ipc_check(d);
        if (d->P > 1) {
            // the shards' error words (this rank's own slot), OR-ed over the ranks
            Shard &s = *d->sh[0];
            int mine = 0;
            GG_HIP(hipMemcpyAsync(&mine, s.err.p + s.p, sizeof(int), hipMemcpyDeviceToHost, d->st));
            GG_HIP(hipStreamSynchronize(d->st));
            for (long long w : ipc_allgather_host(d, mine)) any |= (int)w;
        }
    }
    for (auto &sp : d->sh) {
        std::vector<int> e(d->P, 0);
        GG_HIP(hipMemcpyAsync(e.data(), sp->err.p, d->P * sizeof(int), hipMemcpyDeviceToHost, d->st));
        GG_HIP(hipStreamSynchronize(d->st));
        for (int v : e) any |= v;
    }
    if (any & 8) throw Fallback{any};
    GG_REQUIRE((any & 1) == 0, GG_ETIMEOUT, "dd: wavefront triangular solve: boundary wait timed out");
    if (any & 2) throw Fallback{any};
}
void apply_fallback(gg_dd *d, const Fallback &f)
{
    for (auto &sp : d->sh)
        for (DevTri *T : {&sp->LI, &sp->LS, &sp->UI, &sp->US}) {
            if ((f.bits & 2) && T->kind == DevTri::WAVE2D && T->div == WD_RCP) T->div = WD_HW;
            if ((f.bits & 8) && T->kind == DevTri::WAVE2D && T->wl.tile) T->tile_queue = true;
        }
}
void reset_waves(gg_dd *d)
{
    for (auto &sp : d->sh) {
        for (DevTri *T : {&sp->LI, &sp->LS, &sp->UI, &sp->US}) {
            if (T->kind != DevTri::WAVE2D) continue;
            launch_fill_u64(T->bnd.p, T->wl.ngran(), kSentinel, d->st);
            if (T->wl.tile)     // the tile kernel's task queue
                GG_HIP(hipMemsetAsync(T->bnd.p + T->wl.ngran() + 128LL * kTileDummyBlocks, 0,
                                      64 * sizeof(unsigned long long), d->st));
            if (T->prog.p) GG_HIP(hipMemsetAsync(T->prog.p, 0, T->prog.n * sizeof(unsigned long long), d->st));
        }
        GG_HIP(hipMemsetAsync(sp->err.p, 0, d->P * sizeof(int), d->st));
    }
}

// natural global vector (device, length n) -> every shard's slots of `dst`
void gather_in(gg_dd *d, const double *nat, DBuf<double> Shard::*dst)
{
    for (auto &sp : d->sh) launch_gather(nat, sp->slot2nat.p, (sp.get()->*dst).p, d->H0, d->st);
}
void scatter_out(gg_dd *d, DBuf<double> Shard::*src, double *nat)
{
    for (auto &sp : d->sh) launch_scatter_idx((sp.get()->*src).p, sp->own_slot.p, sp->own_nat.p, nat, sp->nown, d->st);
}

int solve_once(gg_dd *d, const double *d_b, double *d_x, const gg_options *opt, gg_result *res)
{
    GG_REQUIRE(d->have, GG_ESTATE, "gg_dd_solve: no system (call gg_dd_set_system)");
    GG_REQUIRE(opt, GG_EINVAL, "gg_dd_solve: null options");
    const int m = opt->restart;
    GG_REQUIRE(m >= 1 && m <= 512, GG_EINVAL, "gg_dd_solve: restart must be in [1, 512]");
    GG_REQUIRE(opt->max_iter >= 0, GG_EINVAL, "gg_dd_solve: negative max_iter");
    GG_REQUIRE((opt->flags & ~GG_SOLVE_CGS2) == 0, GG_EINVAL, "gg_dd_solve: unknown flags");
    d->cgs2 = (opt->flags & GG_SOLVE_CGS2) != 0;
    set_dev(d);
    ensure_workspace(d, m);
    const long long need = (long long)opt->max_iter + opt->max_iter / m + 4;
    for (auto &sp : d->sh)
        if (need > sp->hist_cap) {
            sp->hist.alloc(need);
            sp->hist_cap = need;
        }
    gather_in(d, d_b, &Shard::bv);
    gather_in(d, d_x, &Shard::xv);
    reset_waves(d);
    DevState h{};
    h.tol = opt->tol;
    h.max_iter = opt->max_iter;
    h.m = m;
    h.j = 1;
    for (auto &sp : d->sh)
        GG_HIP(hipMemcpyAsync(sp->ds.p, &h, sizeof(DevState), hipMemcpyHostToDevice, d->st));
    GG_HIP(hipEventRecord(d->ev0, d->st));
    enqueue_init(d);
    h = read_state(d);
    int ret = 1, iters = 0, inner = 0, restarts = 0;
    long long hist_len = 1;
    double relres = h.resid;
    if (h.done & DONE_INIT) {
        ret = 0;
    } else {
        while (true) {
            if (h.j > opt->max_iter) {
                ret = 1;
                relres = h.resid;
                iters = opt->max_iter;
                hist_len = h.hist_len;
                break;
            }
            restarts++;
            enqueue_cycle(d, m);
            DevState prev = h;
            h = read_state(d);
            check_err(d);
            prof_collect(d, (h.done & DONE_INNER) ? h.conv_i + 1 : h.nit);
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
    GG_HIP(hipEventRecord(d->ev1, d->st));
    check_err(d);
    scatter_out(d, &Shard::xv, d_x);
    GG_HIP(hipStreamSynchronize(d->st));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, d->ev0, d->ev1));
    d->last_hist.resize(hist_len);
    if (hist_len)
        GG_HIP(hipMemcpy(d->last_hist.data(), d->sh[0]->hist.p, hist_len * sizeof(double),
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

int solve_dev(gg_dd *d, const double *d_b, double *d_x, const gg_options *opt, gg_result *res)
{
    for (int attempt = 0;; attempt++) {
        try {
            return solve_once(d, d_b, d_x, opt, res);
        } catch (Fallback &f) {
            if (attempt >= 2) throw Error{GG_EHIP, "gg_dd_solve: fallbacks exhausted"};
            apply_fallback(d, f);
        }
    }
}

// ---------------------------------------------------------------- setup
Wave2D region_wave(const CanonTri &L, const CanonTri &U)
{
    Wave2D wl;
    const char *env = std::getenv("GG_NO_WAVEFRONT");
    if (env && env[0] == '1') return wl;
    wl = detect_wave2d(L, U);
    if (wl.ok && wl.nbands > 512) wl.ok = false;
    const char *e3 = std::getenv("GG_NO_WAVE3D");
    if (!wl.ok && !(e3 && e3[0] == '1')) wl = detect_wave3d(L, U);
    return wl;
}

// rows of a region CSR (region-local row -> slot), columns mapped by `col`
template <class F>
Csr slot_csr(const Csr &C, const std::vector<long long> &slot, long long nslots, F col)
{
    std::vector<long long> row_of(nslots, -1);
    for (size_t r = 0; r < slot.size(); r++) row_of[slot[r]] = (long long)r;
    Csr O;
    O.n = (int)nslots;
    O.rp.assign(nslots + 1, 0);
    O.ci.reserve(C.nnz());
    O.v.reserve(C.nnz());
    for (long long t = 0; t < nslots; t++) {
        const long long r = row_of[t];
        if (r >= 0)
            for (int k = C.rp[r]; k < C.rp[r + 1]; k++) {
                O.ci.push_back((int)col(C.ci[k]));
                O.v.push_back(C.v[k]);
            }
        O.rp[t + 1] = (int)O.ci.size();
    }
    return O;
}

// the fused separator step (k_sep_flow) when both separator triangles are
// level-scheduled with short rows: rows of the three phases in their launch
// order (L and U in level order, then the interior rows with U_IS terms),
// cut into runs of up to 64 (GG_DD_SEPFLOW=0 keeps the four launches)
void build_sepflow(Shard &s, const DDShardHost &H, const Csr &uis, hipStream_t st)
{
    s.sepflow = false;
    const char *e = std::getenv("GG_DD_SEPFLOW");
    if ((e && e[0] == '0') || s.nS == 0 || s.LS.kind != DevTri::LEVEL || s.US.kind != DevTri::LEVEL ||
        s.LS.n != s.US.n)
        return;
    for (const CanonTri *C : {&H.LS, &H.US})
        for (int r = 0; r < C->off.n; r++)
            if (C->off.rp[r + 1] - C->off.rp[r] > kFlowLong) return;
    std::vector<int> rows;
    std::vector<int4> tasks;
    auto add_phase = [&](const std::vector<int> &pr, int phase) {
        for (size_t q = 0; q < pr.size(); q += 64) {
            const int cnt = (int)std::min<size_t>(64, pr.size() - q);
            tasks.push_back(make_int4((int)(rows.size() + q), cnt, phase, 0));
        }
        rows.insert(rows.end(), pr.begin(), pr.end());
    };
    add_phase(level_sets(H.LS).rows, 0);
    add_phase(level_sets(H.US).rows, 1);
    std::vector<int> ifr;
    for (int r = 0; r < uis.n; r++)
        if (uis.rp[r + 1] > uis.rp[r]) ifr.push_back(r);
    add_phase(ifr, 2);
    s.sf_ntask = (int)tasks.size();
    s.sf_tasks.upload(tasks, st);
    s.sf_rows.upload(rows, st);
    GG_HIP(hipStreamSynchronize(st));           // the host vectors end here
    s.sepflow = true;
}

void set_system(gg_dd *d, const Csr &A, int method)
{
    DDPlan plan = dd_plan(A, d->P, method);
    d->n = plan.n;
    d->nsep = plan.part_size[d->P];
    d->maxI = plan.maxI;
    d->pinv = plan.pinv;
    d->q = plan.q;
    // pass 1: host pieces and region layouts of this process's shards
    std::vector<int> mine;
    if (d->kind != GG_DD_LOCAL) mine.push_back(d->rank);
    else for (int p = 0; p < d->P; p++) mine.push_back(p);
    std::vector<DDShardHost> hs;
    d->sh.clear();
    long long pi_max = 0, ps = 0;
    for (int p : mine) {
        hs.push_back(dd_shard(plan, p));
        DDShardHost &H = hs.back();
        auto s = std::make_unique<Shard>();
        s->p = p;
        s->nI = H.nI;
        s->nS = H.nS;
        s->wI = region_wave(H.LI, H.UI);
        s->wS = region_wave(H.LS, H.US);
        s->slotI.resize(H.nI);
        for (int r = 0; r < H.nI; r++) s->slotI[r] = s->wI.ok ? s->wI.slot(r) : r;
        s->slotS.resize(H.nS);
        for (int r = 0; r < H.nS; r++) s->slotS[r] = s->wS.ok ? s->wS.slot(r) : r;
        s->PIr = round_up(std::max<long long>(s->wI.ok ? s->wI.P : H.nI, 1), 512);
        s->PSr = H.nS ? round_up(s->wS.ok ? s->wS.P : H.nS, 512) : 0;
        pi_max = std::max(pi_max, s->PIr);
        ps = s->PSr;            // the separator (and its layout) is the same on every shard
        d->sh.push_back(std::move(s));
    }
    plan.B = Csr{};             // the rest of the plan is not needed any more
    d->S0 = agree_max(d, pi_max);
    d->H0 = d->S0 + ps;
    d->Pl = round_up(d->H0 + (long long)d->P * d->maxI, 512);
    // dot partials per shard: one 16-B unit per thread up to 1024 blocks (the
    // single solver's reduce_grid takes 4 per thread, and a shard's vectors are
    // P times shorter: at C2 / 8 shards 69 blocks left the shard's dot and
    // CGS2 kernels latency-bound); the sharded restatement reads G from
    // gg_dd_dot_layout
    d->G = (int)std::min<long long>(1024, std::max<long long>(1, (d->H0 / 2 + kBlock - 1) / kBlock));
    // pass 2: device structures in the shard's slot space
    for (size_t k = 0; k < d->sh.size(); k++) {
        Shard &s = *d->sh[k];
        DDShardHost &H = hs[k];
        const long long S0 = d->S0, H0 = d->H0;
        const int nI = H.nI, nS = H.nS;
        std::vector<long long> lslot(nI + nS);
        for (int r = 0; r < nI; r++) lslot[r] = s.slotI[r];
        for (int r = 0; r < nS; r++) lslot[nI + r] = S0 + s.slotS[r];
        auto lcol = [&](int c) -> long long {
            if (c < nI) return s.slotI[c];
            if (c < nI + nS) return S0 + s.slotS[c - nI];
            return H0 + (c - nI - nS);
        };
        Csr As = slot_csr(H.A, lslot, H0, lcol);
        // split at S0: interior rows, separator rows (columns stay slot indices)
        Csr AI, AS;
        AI.n = (int)S0;
        AI.rp.assign(As.rp.begin(), As.rp.begin() + S0 + 1);
        AI.ci.assign(As.ci.begin(), As.ci.begin() + As.rp[S0]);
        AI.v.assign(As.v.begin(), As.v.begin() + As.rp[S0]);
        AS.n = (int)(H0 - S0);
        AS.rp.resize(AS.n + 1);
        for (int r = 0; r <= AS.n; r++) AS.rp[r] = As.rp[S0 + r] - As.rp[S0];
        AS.ci.assign(As.ci.begin() + As.rp[S0], As.ci.end());
        AS.v.assign(As.v.begin() + As.rp[S0], As.v.end());
        s.AI.upload(AI, d->st);
        s.AS.upload(AS, d->st);
        s.bytes_spmv = 12.0 * H.A.nnz() + 4.0 * (H0 + 1) + 16.0 * (nI + nS);
        // triangles on their regions
        build_tri(s.LI, H.LI, &s.wI, &s.slotI, s.PIr, d->st);
        build_tri(s.UI, H.UI, &s.wI, &s.slotI, s.PIr, d->st);
        if (nS) {
            build_tri(s.LS, H.LS, &s.wS, &s.slotS, s.PSr, d->st);
            build_tri(s.US, H.US, &s.wS, &s.slotS, s.PSr, d->st);
        }
        s.bytes_trsv = s.LI.bytes + s.UI.bytes + s.LS.bytes + s.US.bytes;
        // coupling terms: separator L rows' interface terms, interior U rows' separator terms
        Csr lsh = slot_csr(H.LSH, s.slotS, s.PSr, [&](int h) { return H0 + h; });
        s.LSH.upload(lsh, d->st);
        Csr uis = slot_csr(H.UIS, s.slotI, s.PIr, [&](int c) { return S0 + s.slotS[c]; });
        s.UIS.upload(uis, d->st);
        build_sepflow(s, H, uis, d->st);
        // interface slots, natural rows of the slots, rows written back
        std::vector<long long> ifs(std::max(d->maxI, 1), -1);
        for (size_t t = 0; t < H.iface.size(); t++) ifs[t] = s.slotI[H.iface[t]];
        s.iface_slot.upload(ifs, d->st);
        std::vector<long long> s2n(H0, -1), os, on;
        s.slot2perm.assign(H0, -1);
        for (int r = 0; r < nI + nS; r++) {
            s2n[lslot[r]] = plan.q[H.rows[r]];
            s.slot2perm[lslot[r]] = H.rows[r];
        }
        s.slot2nat.upload(s2n, d->st);
        const bool own_sep = d->kind != GG_DD_LOCAL || s.p == 0;
        for (int r = 0; r < nI + (own_sep ? nS : 0); r++) {
            os.push_back(lslot[r]);
            on.push_back(plan.q[H.rows[r]]);
        }
        s.nown = (long long)os.size();
        s.own_slot.upload(os, d->st);
        s.own_nat.upload(on, d->st);
        GG_HIP(hipStreamSynchronize(d->st));
        H = DDShardHost{};
    }
    d->m_alloc = -1;
    d->have = true;
}

void stage_nat(gg_dd *d, DBuf<double> &buf, const double *h)
{
    if (buf.n < (size_t)std::max(d->n, 1)) buf.alloc(std::max(d->n, 1));
    GG_HIP(hipMemcpyAsync(buf.p, h, sizeof(double) * d->n, hipMemcpyHostToDevice, d->st));
}
void fetch_nat(gg_dd *d, const DBuf<double> &buf, double *h)
{
    GG_HIP(hipMemcpyAsync(h, buf.p, sizeof(double) * d->n, hipMemcpyDeviceToHost, d->st));
    GG_HIP(hipStreamSynchronize(d->st));
}

}  // namespace

extern "C" {

int gg_dd_unique_id(unsigned char *id)
{
    GG_API_BEGIN
    GG_REQUIRE(id, GG_EINVAL, "null id");
    static_assert(sizeof(ncclUniqueId) == GG_DD_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    GG_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return GG_OK;
    GG_API_END
}

int gg_dd_create(int device, int nparts, int comm, int rank, const unsigned char *id, gg_dd **out)
{
    GG_API_BEGIN
    GG_REQUIRE(out, GG_EINVAL, "null out");
    GG_REQUIRE(nparts >= 1 && nparts <= kMaxShards, GG_EINVAL, "dd: nparts must be in [1, 16]");
    GG_REQUIRE(comm == GG_DD_LOCAL || comm == GG_DD_RCCL || comm == GG_DD_IPC || comm == GG_DD_LOOPBACK,
               GG_EINVAL, "dd: unknown communicator");
    GG_REQUIRE(comm != GG_DD_LOOPBACK || (rank >= 0 && rank < nparts), GG_EINVAL,
               "dd: loopback needs 0 <= rank < nparts");
    GG_REQUIRE(comm != GG_DD_RCCL || (id && rank >= 0 && rank < nparts), GG_EINVAL,
               "dd: RCCL needs an id and 0 <= rank < nparts");
    GG_REQUIRE(comm != GG_DD_IPC || (rank >= 0 && rank < nparts), GG_EINVAL,
               "dd: IPC needs 0 <= rank < nparts");
    auto d = std::make_unique<gg_dd>();
    d->device = device;
    d->P = nparts;
    d->kind = comm;
    d->rank = comm == GG_DD_LOCAL ? 0 : rank;
    set_dev(d.get());
    GG_HIP(hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking));
    {
        // default: in line (round 5, loopback C2/8: the SpMV family 41 -> 16.5 us,
        // C4/8 58 -> 47 us -- the event pair of the overlap cost more than it hid)
        const char *hi = std::getenv("GG_DD_HALO_INLINE");
        d->halo_inline = !(hi && hi[0] == '0');
        const char *hf = std::getenv("GG_DD_HALO_FUSED");
        d->halo_fused = !(hf && hf[0] == '0');
    }
    GG_HIP(hipStreamCreateWithFlags(&d->st2, hipStreamNonBlocking));
    GG_HIP(hipEventCreate(&d->ev0));
    GG_HIP(hipEventCreate(&d->ev1));
    GG_HIP(hipEventCreateWithFlags(&d->evx, hipEventDisableTiming));
    GG_HIP(hipEventCreateWithFlags(&d->evh, hipEventDisableTiming));
    if (comm == GG_DD_RCCL) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        GG_NCCL(ncclCommInitRank(&d->comm, nparts, u, rank));
    }
    if (comm == GG_DD_IPC) {
        // [flags kMaxShards x kIpcXB u64 (zero: sequence numbers start at 1)]
        // [data 2 x nparts x capd doubles], uncached so that peers' stores and
        // this rank's polls meet in memory
        const char *cap = std::getenv("GG_DD_IPC_CAP");
        d->ipc_capd = cap ? std::max(1LL, atoll(cap)) : (1LL << 20);
        const size_t bytes = xch_area_bytes(nparts, d->ipc_capd);
        GG_HIP(hipExtMallocWithFlags(&d->ipc_area, bytes, hipDeviceMallocUncached));
        GG_HIP(hipMemset(d->ipc_area, 0, bytes));
        GG_HIP(hipDeviceSynchronize());
        d->xerr.alloc(1);
        GG_HIP(hipMemset(d->xerr.p, 0, sizeof(int)));
        d->ipc.base[rank] = d->ipc_area;
        d->ipc_connected = nparts == 1;
    }
    if (comm == GG_DD_LOOPBACK && nparts > 1) {
        // the in-kernel exchanges' area, this rank's own standing in for every peer's
        d->ipc_capd = 1LL << 16;
        const size_t bytes = xch_area_bytes(nparts, d->ipc_capd);
        GG_HIP(hipExtMallocWithFlags(&d->ipc_area, bytes, hipDeviceMallocUncached));
        GG_HIP(hipMemset(d->ipc_area, 0, bytes));
        d->xerr.alloc(1);
        GG_HIP(hipMemset(d->xerr.p, 0, sizeof(int)));
        for (int q = 0; q < nparts; q++) d->ipc.base[q] = d->ipc_area;
    }
    if ((comm == GG_DD_IPC || comm == GG_DD_LOOPBACK) && nparts > 1) {
        // off by default: measured slower than the launch-per-exchange path
        // (loopback C2/8, one box: CGS2 81 vs 52.5 us per iteration, C4/8 256 vs
        // 193 us; profiles/r05/xk_ab.txt) -- the uncached-memory round trips of
        // the reducers' hand-off inside a launch cost more than the launch
        // boundaries they replace.  GG_DD_XK=1 turns it on.
        const char *xk = std::getenv("GG_DD_XK");
        d->xk = xk && xk[0] == '1';
        const size_t bytes = 2 * 64 * sizeof(double);            // hx[64] | hf[64]
        GG_HIP(hipExtMallocWithFlags(&d->xk_local, bytes, hipDeviceMallocUncached));
        GG_HIP(hipMemset(d->xk_local, 0, bytes));
        GG_HIP(hipDeviceSynchronize());
        d->xch.me = rank;
        d->xch.P = nparts;
        d->xch.loop = comm == GG_DD_LOOPBACK;
        d->xch.capd = d->ipc_capd;
        d->xch.err = d->xerr.p;
        d->xch.hx = static_cast<double *>(d->xk_local);
        d->xch.hf = reinterpret_cast<unsigned long long *>(static_cast<double *>(d->xk_local) + 64);
        // (xch.pp is filled when the areas are connected: now for loopback,
        // in gg_dd_ipc_connect for IPC)
        d->xch.pp = d->ipc;
    }
    *out = d.release();
    return GG_OK;
    GG_API_END
}

int gg_dd_destroy(gg_dd *d)
{
    if (!d) return GG_OK;
    (void)hipSetDevice(d->device);
    if (d->st) (void)hipStreamSynchronize(d->st);
    d->sh.clear();
    d->nat_a.release();
    d->nat_b.release();
    if (d->comm) (void)ncclCommDestroy(d->comm);
    if (d->ipc_area) {
        (void)hipDeviceSynchronize();
        if (d->kind == GG_DD_IPC)
            for (int q = 0; q < d->P; q++)
                if (q != d->rank && d->ipc.base[q]) (void)hipIpcCloseMemHandle(d->ipc.base[q]);
        (void)hipFree(d->ipc_area);
    }
    if (d->xk_local) (void)hipFree(d->xk_local);
    d->xerr.release();
    if (d->ev0) (void)hipEventDestroy(d->ev0);
    if (d->ev1) (void)hipEventDestroy(d->ev1);
    if (d->evx) (void)hipEventDestroy(d->evx);
    if (d->evh) (void)hipEventDestroy(d->evh);
    if (d->st2) (void)hipStreamSynchronize(d->st2);
    if (d->st2) (void)hipStreamDestroy(d->st2);
    if (d->st) (void)hipStreamDestroy(d->st);
    delete d;
    return GG_OK;
}

int gg_dd_ipc_handle(gg_dd *d, unsigned char *handle)
{
    GG_API_BEGIN
    GG_REQUIRE(d && handle, GG_EINVAL, "null argument");
    GG_REQUIRE(d->kind == GG_DD_IPC, GG_ESTATE, "dd: not an IPC communicator");
    static_assert(sizeof(hipIpcMemHandle_t) <= GG_DD_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");
    set_dev(d);
    hipIpcMemHandle_t h;
    GG_HIP(hipIpcGetMemHandle(&h, d->ipc_area));
    std::memset(handle, 0, GG_DD_IPC_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    return GG_OK;
    GG_API_END
}

int gg_dd_ipc_connect(gg_dd *d, const unsigned char *handles)
{
    GG_API_BEGIN
    GG_REQUIRE(d && handles, GG_EINVAL, "null argument");
    GG_REQUIRE(d->kind == GG_DD_IPC, GG_ESTATE, "dd: not an IPC communicator");
    GG_REQUIRE(!d->ipc_connected || d->P == 1, GG_ESTATE, "dd: IPC areas already connected");
    set_dev(d);
    for (int q = 0; q < d->P; q++) {
        if (q == d->rank) continue;
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)q * GG_DD_IPC_HANDLE_BYTES, sizeof(h));
        void *p = nullptr;
        GG_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        d->ipc.base[q] = p;
    }
    d->ipc_connected = true;
    d->xch.pp = d->ipc;
    // a first exchange: every rank has mapped every area before anyone moves
    // on; it carries a hash of each rank's PCI bus id (ranks sharing a GPU)
    char bus[64] = {};
    GG_HIP(hipDeviceGetPCIBusId(bus, sizeof bus, d->device));
    // FNV-1a in unsigned arithmetic (wraps by definition), sent as its bits
    unsigned long long hu = 1469598103934665603ULL;
    for (const char *c = bus; *c; c++) hu = (hu ^ (unsigned char)*c) * 1099511628211ULL;
    long long hb;
    std::memcpy(&hb, &hu, sizeof hb);
    int same = 0;
    for (long long v : ipc_allgather_host(d, hb)) same += v == hb;
    d->xk_shared = same > 1;
    return GG_OK;
    GG_API_END
}

int gg_dd_comm_ranks(gg_dd *d, int *ranks, int *rank)
{
    GG_API_BEGIN
    GG_REQUIRE(d && ranks, GG_EINVAL, "null argument");
    int c = 1;
    if (d->kind == GG_DD_RCCL) GG_NCCL(ncclCommCount(d->comm, &c));
    if (d->kind == GG_DD_IPC) {
        c = 0;
        for (int q = 0; q < d->P; q++) c += d->ipc.base[q] != nullptr;
        if (d->P > 1) {
            // every rank reports its own rank: the ranks are distinct and complete
            const std::vector<long long> r = ipc_allgather_host(d, d->rank);
            for (int q = 0; q < d->P; q++) GG_REQUIRE(r[q] == q, GG_ECOMM, "dd: IPC rank mismatch");
        }
    }
    *ranks = c;
    if (rank) *rank = d->rank;
    return GG_OK;
    GG_API_END
}

int gg_dd_set_system(gg_dd *d, int n, const int *rp, const int *ci, const double *val, int method)
{
    GG_API_BEGIN
    GG_REQUIRE(d && rp && (n == 0 || (ci && val)), GG_EINVAL, "null argument");
    GG_REQUIRE(n >= 1 && rp[0] == 0, GG_EINVAL, "dd: bad CSR");
    GG_REQUIRE((method & ~(GG_PART_COLOR_SEP | 3)) == 0 && (method & 3) != 3, GG_EINVAL,
               "dd: method must be GG_PART_BISECT, GG_PART_BLOCKS or GG_PART_GRID (| GG_PART_COLOR_SEP)");
    for (int r = 0; r < n; r++) {
        GG_REQUIRE(rp[r + 1] >= rp[r], GG_EINVAL, "dd: row_ptr not monotone");
        for (int k = rp[r]; k < rp[r + 1]; k++)
            GG_REQUIRE(ci[k] >= 0 && ci[k] < n, GG_EINVAL, "dd: column index out of range");
    }
    set_dev(d);
    Csr A;
    A.n = n;
    A.rp.assign(rp, rp + n + 1);
    A.ci.assign(ci, ci + rp[n]);
    A.v.assign(val, val + rp[n]);
    d->have = false;
    set_system(d, A, method);
    return GG_OK;
    GG_API_END
}

int gg_dd_info(gg_dd *d, int *info)
{
    GG_API_BEGIN
    GG_REQUIRE(d && info, GG_EINVAL, "null argument");
    GG_REQUIRE(d->have, GG_ESTATE, "dd: no system");
    const Shard &s = *d->sh[0];
    info[0] = d->n;
    info[1] = d->P;
    info[2] = d->nsep;
    info[3] = d->maxI;
    info[4] = s.nI;
    info[5] = s.wI.ok ? (s.wI.nz > 1 ? 3 : 2) : 0;
    info[6] = s.wS.ok ? (s.wS.nz > 1 ? 3 : 2) : s.sepflow ? 1 : 0;
    info[7] = (int)d->Pl;
    info[8] = (int)d->sh.size();
    info[9] = d->P * d->maxI;
    return GG_OK;
    GG_API_END
}

int gg_dd_xk_active(gg_dd *d, int *on)
{
    GG_API_BEGIN
    GG_REQUIRE(d && on, GG_EINVAL, "null argument");
    GG_REQUIRE(d->have, GG_ESTATE, "dd: no system");
    *on = use_xk(d, 1) ? 1 : 0;
    return GG_OK;
    GG_API_END
}

int gg_dd_perm(gg_dd *d, int *pinv, int *q)
{
    GG_API_BEGIN
    GG_REQUIRE(d && d->have, GG_ESTATE, "dd: no system");
    if (pinv) std::memcpy(pinv, d->pinv.data(), sizeof(int) * d->n);
    if (q) std::memcpy(q, d->q.data(), sizeof(int) * d->n);
    return GG_OK;
    GG_API_END
}

int gg_dd_dot_layout(gg_dd *d, int part, long long *out, long long cap, int *G)
{
    GG_API_BEGIN
    GG_REQUIRE(d && d->have, GG_ESTATE, "dd: no system");
    for (auto &sp : d->sh) {
        if (sp->p != part) continue;
        const long long len = dot_len(d, *sp);
        if (out) std::memcpy(out, sp->slot2perm.data(), sizeof(long long) * std::min(len, cap));
        if (G) *G = d->G;
        return (int)len;
    }
    GG_REQUIRE(false, GG_EINVAL, "dd: part not held by this process");
    return GG_EINVAL;
    GG_API_END
}

int gg_dd_solve_device(gg_dd *d, const double *d_b, double *d_x, const gg_options *opt, gg_result *res)
{
    GG_API_BEGIN
    GG_REQUIRE(d && d_b && d_x, GG_EINVAL, "null argument");
    return solve_dev(d, d_b, d_x, opt, res);
    GG_API_END
}

int gg_dd_solve(gg_dd *d, const double *b, double *x, const gg_options *opt, gg_result *res)
{
    GG_API_BEGIN
    GG_REQUIRE(d && b && x, GG_EINVAL, "null argument");
    GG_REQUIRE(d->have, GG_ESTATE, "gg_dd_solve: no system");
    set_dev(d);
    stage_nat(d, d->nat_a, b);
    stage_nat(d, d->nat_b, x);
    int rc = solve_dev(d, d->nat_a.p, d->nat_b.p, opt, res);
    if (rc >= 0) fetch_nat(d, d->nat_b, x);
    return rc;
    GG_API_END
}

int gg_dd_get_history(gg_dd *d, double *out, int cap)
{
    if (!d) return GG_EINVAL;
    const int len = (int)d->last_hist.size();
    if (out && cap > 0) std::memcpy(out, d->last_hist.data(), sizeof(double) * std::min(len, cap));
    return len;
}

int gg_dd_spmv(gg_dd *d, const double *x, double *y)
{
    GG_API_BEGIN
    GG_REQUIRE(d && x && y, GG_EINVAL, "null argument");
    GG_REQUIRE(d->have, GG_ESTATE, "dd: no system");
    set_dev(d);
    ensure_workspace(d, std::max(d->m_alloc, 1));
    stage_nat(d, d->nat_a, x);
    stage_nat(d, d->nat_b, y);
    gather_in(d, d->nat_a.p, &Shard::xv);
    spmv(d, -1, vec(&Shard::xv), vec(&Shard::ww));
    scatter_out(d, &Shard::ww, d->nat_b.p);
    fetch_nat(d, d->nat_b, y);
    return GG_OK;
    GG_API_END
}

int gg_dd_set_division(gg_dd *d, int mode)
{
    GG_API_BEGIN
    GG_REQUIRE(d, GG_EINVAL, "null argument");
    GG_REQUIRE(mode == GG_DIV_EXACT || mode == GG_DIV_RCP || mode == GG_DIV_FMA, GG_EINVAL,
               "gg_dd_set_division: mode must be GG_DIV_EXACT, GG_DIV_RCP or GG_DIV_FMA");
    d->div_mode = mode;
    return GG_OK;
    GG_API_END
}

int gg_dd_time_exchange(gg_dd *d, long long cnt, int reps, double *avg_us)
{
    GG_API_BEGIN
    GG_REQUIRE(d && avg_us && cnt > 0 && reps > 0, GG_EINVAL, "bad argument");
    GG_REQUIRE(d->have, GG_ESTATE, "dd: no system");
    set_dev(d);
    ensure_workspace(d, std::max(d->m_alloc, 1));
    // the CGS2 partials buffer holds P slots of (m+1) G doubles per shard
    GG_REQUIRE(cnt <= (long long)(d->m_alloc + 1) * d->G, GG_EINVAL,
               "gg_dd_time_exchange: cnt above the exchange buffer ((m+1) * G doubles)");
    hipEvent_t e0, e1;
    GG_HIP(hipEventCreate(&e0));
    GG_HIP(hipEventCreate(&e1));
    exchange(d, vec(&Shard::partC), 0, cnt);                  // warm-up (and a rendezvous)
    GG_HIP(hipStreamSynchronize(d->st));
    GG_HIP(hipEventRecord(e0, d->st));
    for (int r = 0; r < reps; r++) exchange(d, vec(&Shard::partC), 0, cnt);
    GG_HIP(hipEventRecord(e1, d->st));
    GG_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (d->kind == GG_DD_IPC) ipc_check(d);
    *avg_us = 1e3 * ms / reps;
    return GG_OK;
    GG_API_END
}

int gg_dd_profile_enable(gg_dd *d, int kinds)
{
    if (!d) return GG_EINVAL;
    d->prof_mask = kinds & ((1 << GG_DD_PROF_NKINDS) - 1);
    return GG_OK;
}
int gg_dd_profile_reset(gg_dd *d)
{
    if (!d) return GG_EINVAL;
    for (int k = 0; k < GG_DD_PROF_NKINDS; k++) {
        d->prof_ms[k] = 0;
        d->prof_cnt[k] = 0;
    }
    return GG_OK;
}
int gg_dd_profile_get(gg_dd *d, int kind, int *launches, double *total_ms)
{
    if (!d || kind < 0 || kind >= GG_DD_PROF_NKINDS || !launches || !total_ms) return GG_EINVAL;
    *launches = (int)d->prof_cnt[kind];
    *total_ms = d->prof_ms[kind];
    return GG_OK;
}
int gg_dd_bytes(gg_dd *d, int kind, double *bytes)
{
    if (!d || !bytes || !d->have) return GG_EINVAL;
    // algorithmic bytes of one family launch for the shards of this process
    // (each operand once, each result once)
    double b = 0;
    for (auto &sp : d->sh) {
        Shard &s = *sp;
        if (kind == GG_DD_PROF_SPMV) {
            for (const DevCsr *A : {&s.AI, &s.AS})
                b += 12.0 * A->nnz + 4.0 * (A->n + 1) + 16.0 * A->n;
        } else if (kind == GG_DD_PROF_TRSV_L) {
            b += s.LI.alg_bytes();
        } else if (kind == GG_DD_PROF_TRSV_U) {
            b += s.UI.alg_bytes();
        } else {
            return GG_EINVAL;
        }
    }
    *bytes = b;
    return GG_OK;
}

int gg_dd_precond_apply(gg_dd *d, const double *in, double *out)
{
    GG_API_BEGIN
    GG_REQUIRE(d && in && out, GG_EINVAL, "null argument");
    GG_REQUIRE(d->have, GG_ESTATE, "dd: no system");
    set_dev(d);
    ensure_workspace(d, std::max(d->m_alloc, 1));
    stage_nat(d, d->nat_a, in);
    stage_nat(d, d->nat_b, out);
    gather_in(d, d->nat_a.p, &Shard::xv);
    auto run = [&]() {
        reset_waves(d);
        apply_minv(d, -1, 0, vec(&Shard::xv), vec(&Shard::ww));
        check_err(d);
    };
    for (int attempt = 0;; attempt++) {
        try {
            run();
            break;
        } catch (Fallback &f) {
            if (attempt >= 2) throw Error{GG_EHIP, "gg_dd_precond_apply: fallbacks exhausted"};
            apply_fallback(d, f);
        }
    }
    scatter_out(d, &Shard::ww, d->nat_b.p);
    fetch_nat(d, d->nat_b, out);
    return GG_OK;
    GG_API_END
}

}  // extern "C"
