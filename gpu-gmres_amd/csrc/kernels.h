// kernels.h -- launchers for the hand-written gfx950 kernels of the GMRES path.
#pragma once

#include "gg_internal.h"

namespace gg {

// Device-side GMRES control block (one per solver, lives in HBM).  Kernels of
// a restart cycle read it to skip work once converged, so a whole cycle can be
// enqueued with a single host sync per cycle.
struct DevState {
    double normb, beta, resid, tol;
    int done;       // bit flags: 1 inner-converged, 2 restart-converged, 4 converged at start,
                    // 8 cycle aborted (a persistent grid was not co-resident: rerun)
    int conv_i;     // inner index of convergence
    int j;          // reference iteration counter at the start of the cycle
    int max_iter;
    int nit;        // inner iterations allowed in this cycle = min(m, max_iter - j + 1)
    int hist_len;   // history entries recorded before this cycle
    int m;
    int upd_k;      // column count - 1 used by the last Update
    int err;        // device-side error (1 = wavefront wait timed out)
    int pad;
};
constexpr int DONE_INNER = 1, DONE_RESTART = 2, DONE_INIT = 4, DONE_ABORT = 8;
// a cycle enqueued behind the one that ends the solve (the host's pipelined
// cycle loop) must do nothing: DONE_FINAL = the converged cycle's update has
// been applied (set by k_end_cycle), DONE_EXH = max_iter exhausted before the
// cycle (set by k_init_cycle)
constexpr int DONE_FINAL = 16, DONE_EXH = 32;

// A kernel is skipped when (*done & mask) != 0, or (nit && i >= *nit).
struct Gate {
    const int *done = nullptr;
    int mask = 0;
    const int *nit = nullptr;
    int i = 0;
};

// Which 16-B units (slot pairs) of a solver's vector space hold at least one
// real row: the wavefront layouts pad every line to T steps (C2: 10 %, C4:
// 11 % of the slots), and every vector is +0 there, so the orthogonalization
// and the update skip those units -- the same sums, bit for bit (a +0 term
// never changes a partial that starts at +0), fewer bytes
struct UnitMap {
    int kind = -1;        // -1 every unit, 0 natural order (n rows), 1 2D band wavefront, 2 3D tiles
    int nx = 0, ny = 0, nz = 1, T = 0, skew = 1, NJ = 0, nbands = 0;
    long long n = 0;
    // bordered grid (Wave2D::bnt): units [0, tbase) hold the tail (real while
    // slot < tn), the wavefront layout starts at unit tbase
    long long tbase = 0, tn = 0;
};

constexpr int kBlock = 256;
constexpr unsigned long long kSentinel = 0x7FF4DEAD0000BEEFull;  // sNaN payload: "not ready"

int reduce_grid(long long units);  // blocks for the vector kernels (units = Ppad/2)

// ---- vector ops (lengths are Ppad, a multiple of 512) --------------------
void launch_fill_u64(unsigned long long *p, long long n, unsigned long long v, hipStream_t st);
// transient step: u = sources(it*h) (DC / PULSE / PWL); w = B u + (C/h) x   (natural order, n rows)
void launch_transient_step(int n, int nsrc, const int *kind, const int *dptr, const double *data, int it,
                           double h, double *u, const int *src_ptr, const int *src_idx, const double *cdiag,
                           const double *x, double *w, hipStream_t st);
// the same with general B (n x nsrc) and R = C/h (n x n) in CSR: w = B u + R x
void launch_transient_step_csr(int n, int nsrc, const int *kind, const int *dptr, const double *data, int it,
                               double h, double *u, const int *bp, const int *bi, const double *bv,
                               const int *rp, const int *ri, const double *rv, const double *x, double *w,
                               hipStream_t st);
void launch_gather_ports(int nport, const int *port, const double *x, double *out, hipStream_t st);
// tap statistics: mode 0 seed (max = min = sum = x[tap]), 1 update, 2 finish (sum /= npts)
void launch_taps(int ntap, const int *tap, const double *x, double *mx, double *mn, double *sm, int mode,
                 double npts, hipStream_t st);
// device ILU(0) column elimination (co-resident grid of at most ilu0_columns_max_blocks())
int ilu0_columns_max_blocks();
void launch_ilu0_columns(int n, const int *cp, const int *ri, const double *cv0, double *cv, int *level,
                         int *done, int *err, int blocks, hipStream_t st);
// device ILU(k) numeric factorization on the flat ILU(k) pattern (k_iluk_wave; co-resident grid)
int iluk_wave_max_blocks();   // co-resident blocks of k_iluk_wave
int iluk_wave_cap();          // row length above which k_iluk_wave takes the long-row path
void launch_iluk_scatter(int n, const int *arp, const int *aci, const double *av, const long long *prow,
                         const int *pcol, double *val, hipStream_t st);
void launch_iluk_wave(int n, const long long *prow, const int *nl, const int *pcol, double *val, double *dinv,
                      int *done, const int *rows_short, int nshort, const int *rows_long, int nlong,
                      int long_blocks, int *scratch, int *err, int blocks, hipStream_t st);
// out[i] = idx[i]<0 ? 0 : in[idx[i]]  (+ fill0/fill1[0, nfill) = the sentinel)
void launch_gather(const double *in, const long long *idx, double *out, long long n, hipStream_t st,
                   double *fill0 = nullptr, double *fill1 = nullptr, long long nfill = 0);
void launch_copy(const double *in, double *out, long long n, hipStream_t st);
void launch_dot(Gate g, const double *a, const double *b, double *part, int G, long long Ppad, hipStream_t st);

// ---- sharded solve (dd.hip) --------------------------------------------------
// out[r] = in[r] - sum_k C.v[k] * x[C.ci[k]] (sequential, listed order), r < C.n
void launch_sub_seq(Gate g, const DevCsr &C, const double *x, const double *in, double *out,
                    hipStream_t st, double *fill0 = nullptr, double *fill1 = nullptr, int nfill = 0);
// the sharded solve's fused separator step (kernels.hip k_sep_flow): per phase,
// row r: acc = b[r] (polled when bpoll) - prefix terms (plain loads of px) -
// own terms (polled sources src[ci]); x[r] = d ? acc / d[r] : acc
struct SepPhase {
    const int *rp = nullptr, *ci = nullptr;
    const double *v = nullptr, *src = nullptr;
    const int *prp = nullptr, *pci = nullptr;
    const double *pv = nullptr, *px = nullptr;
    const double *b = nullptr, *d = nullptr;
    double *x = nullptr;
    bool bpoll = false;
};
struct SepFlow { SepPhase ph[3]; };
void launch_sep_flow(Gate g, int ntask, const int4 *tasks, const int *rows, const SepFlow &f, int *err, hipStream_t st);
struct ShardPtrs { double *p[kMaxShards]; };
// every shard's slot (b.p[s] + off + s*cnt, cnt doubles) copied to every other shard
void launch_allgather_local(const ShardPtrs &b, int P, long long off, long long cnt, hipStream_t st);
// The interface exchange with its gather in the same launch (the SpMV halo and
// the separator step's interface values): shard s's slot is formed from its
// own vector, b.p[s][gi.p[s][e]] (-1: 0), and stored into every shard's slot s
// (own included); f0 / f1: nf words of each shard set to the sentinel (the
// fills k_gather carried).  Loopback: every pointer is the one shard's.
struct IdxPtrs { const long long *p[kMaxShards]; };
struct FillPtrs { double *f0[kMaxShards], *f1[kMaxShards]; };
void launch_gather_allgather_local(const ShardPtrs &b, const IdxPtrs &gi, int P, long long off, long long cnt,
                                   const FillPtrs &fl, long long nf, hipStream_t st);
void launch_scatter_idx(const double *in, const long long *src, const long long *dst, double *out,
                        long long n, hipStream_t st);   // out[dst[i]] = in[src[i]]
// GG_DD_IPC: the exchange areas of all ranks as mapped in this process
constexpr int kIpcXB = 64;             // blocks (flag words per source rank) of one exchange
struct IpcPeers { void *base[kMaxShards]; };
// all-gather of cnt doubles per rank: slot q at buf + q*cnt (this rank's slot
// me already in place); err |= 4 when a peer did not arrive in time
void launch_ipc_allgather(const IpcPeers &pp, int me, int P, double *buf, long long cnt,
                          unsigned long long seq, long long capd, int *err, hipStream_t st);
// the same with this rank's slot gathered in the launch: buf[me*cnt + e] =
// x[gidx[e]] (-1: 0) first, and nf words of f0 / f1 set to the sentinel
// the sharded SpMV and its halo exchange in one launch (kernels.hip
// k_dd_spmv_x): y = A x (resid: b - A x) over the interior rows (AI, rows
// [0, S0)) and the separator rows (AS, rows S0..), the halo at x + H0 (slot q at
// halo + q * cnt) exchanged in the launch -- GG_DD_IPC (peers pp, sequence seq)
// or loopback (loop); arrived: a device word of this shard's, target epoch *
// (the launch's exchange blocks), epoch counting these launches from 1.  false:
// not applicable (panelled matrices), nothing launched
struct DdSpmvX {
    IpcPeers pp;
    int me, P, loop;
    double *halo;
    long long cnt, capd;
    unsigned long long seq;
    int *err;
    const long long *gidx;
    unsigned long long *arrived;
    unsigned long long target;
    int nbx, nbi, nbs;
    int i_sell, i_n, i_nb, s_sell, s_n, s_nb;
    const int *i_ptr, *i_rp, *i_ci, *s_ptr, *s_rp, *s_ci;
    const double *i_v, *s_v;
    const double *x, *b;
    double *y;
    long long S0;
};
struct DdSpmvCall {
    IpcPeers pp;
    int me = 0, P = 1;
    bool loop = false, resid = false;
    double *halo = nullptr;
    long long cnt = 0, capd = 0;
    unsigned long long seq = 0, epoch = 0;
    int *err = nullptr;
    const long long *gidx = nullptr;
    unsigned long long *arrived = nullptr;
    const DevCsr *AI = nullptr, *AS = nullptr;
    const double *x = nullptr, *b = nullptr;
    double *y = nullptr;
    long long S0 = 0;
};
bool launch_dd_spmv_x(Gate g, const DdSpmvCall &c, hipStream_t st);
void launch_ipc_gather_allgather(const IpcPeers &pp, int me, int P, const double *x, const long long *gidx,
                                 double *buf, long long cnt, unsigned long long seq, long long capd, int *err,
                                 double *f0, double *f1, long long nf, hipStream_t st);

// The CGS2 exchanges inside the kernels (GG_DD_IPC / GG_DD_LOOPBACK, one shard
// per process, inner iterations with i + 1 <= kCgsXMax): a producer kernel
// stores each block's partials into its own slot (part + me*cnt) and straight
// into every peer's area (data[seq & 1][me], as k_ipc_allgather), then raises
// the block's flag xflag[me][b] = seq there; the consumer kernel's reducer
// blocks wait for the P*G flags of their dot, sum the partials in
// k_cgs_reduce's order (the same bits) and hand the value to every block of
// the launch through `hx` / `hf` (this rank's uncached scratch).  Area of rank
// q: [flags kMaxShards x kIpcXB][data 2 x P x capd][xflags kMaxShards x kIpcXF].
constexpr int kIpcXF = 4096;           // in-kernel exchange flag words per source rank (>= 4 x the dot grid)
constexpr int kCgsXMax = 32;           // dots per inner iteration the in-kernel path takes
constexpr int kCgsKC = 8;              // dots per block of the multidot kernels (grid G x ceil(nk / 8))
struct Xch {
    IpcPeers pp;                       // areas (loopback: this rank's own for every q)
    int me = 0, P = 1, loop = 0;       // loop: the peers' slots are this rank's own (timing only)
    long long capd = 0;
    int *err = nullptr;                // |= 4: a flag did not arrive within ~30 s
    double *hx = nullptr;              // reduced values (kCgsXMax + 1)
    unsigned long long *hf = nullptr;  // their flags (sequence numbers)
};
size_t xch_area_bytes(int P, long long capd);
// <w, v_k>, k < nk: block partials published as exchange seq (part: this rank's slot)
void launch_multidot_x(Gate g, const double *w, const double *V, long long ldv, int nk, double *part, int G,
                       long long Pdot, const Xch &x, unsigned long long seq, hipStream_t st);
// h = the reduced exchange sin (H[k, i] = h[k], or += when add), w -= V h, and
// (part_out != null) the next pass's dot partials, or (norm_out) the norm's,
// published as exchange sout
void launch_cgs_update_x(Gate g, double *w, const double *V, long long ldv, int nk, int G, long long Ppad,
                         long long Pdot, const double *part_in, unsigned long long sin, double *H, int i, int m,
                         bool add, double *part_out, double *norm_out, const Xch &x, unsigned long long sout,
                         hipStream_t st);
// MGS on the same exchanges: <a, b> published as exchange seq; one MGS step
// with h reduced from exchange sin, its next partials published as sout
// (vnext null: the norm's)
void launch_dot_x(Gate g, const double *a, const double *b, double *part, int G, long long Pdot, const Xch &x,
                  unsigned long long seq, hipStream_t st);
void launch_mgs_step_x(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, unsigned long long sin, double *part_out, double *H, int G,
                       long long Ppad, long long Pdot, const Xch &x, unsigned long long sout, hipStream_t st);
// k_arnoldi_finalize with the norm reduced from exchange sin
void launch_arnoldi_finalize_x(Gate g, int i, int m, DevState *ds, const double *part_in, unsigned long long sin,
                               int G, const double *w, double *vnext, double *H, double *cs, double *sn,
                               double *s, double *hist, long long Ppad, const Xch &x, hipStream_t st);

// ---- split (PG) elementwise maps -------------------------------------------
void launch_f64_to_f32(Gate g, const double *in, float *out, int n, hipStream_t st);   // out = RN_f32(in)
// *out += sum over the nw 32-bit words w_k of p of w_k * (2k + 1) (mod 2^64)
void launch_fingerprint(const void *p, long long nw, unsigned long long *out, hipStream_t st);
void launch_f32_to_f64(Gate g, const float *in, double *out, int n, hipStream_t st);   // out = (double)in
void launch_mul(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st);            // out = in*s
void launch_div(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st);            // out = in/s

// ---- SpMV ------------------------------------------------------------------
// y = A x  (resid=false)  or  y = b - A x  (resid=true)
// y = A x (resid: y = b - A x); ydiv: y[r] /= ydiv[r] (the split engine's folded row scaling)
void launch_spmv(Gate g, const DevCsr &A, const double *x, const double *b, double *y, bool resid,
                 hipStream_t st, const double *ydiv = nullptr);
// y[r] = (sum_k a_k RN(x[c_k] / xdiv[c_k])) / ydiv[r] on the sliced copy (false, nothing
// launched, when A has none): the split engine's D_r^-1 in the SpMV's gathers
bool launch_spmv_xdiv(Gate g, const DevCsr &A, const double *x, const double *xdiv, double *y, hipStream_t st,
                      const double *ydiv, double *fill = nullptr,
                      int nfill = 0);   // + fill[< nfill] = sentinel (the next flow solve's x)

// ---- triangular solves ---------------------------------------------------------
void launch_trsv(Gate g, DevTri &T, const double *b, double *x, int *err, hipStream_t st);
// forward solve of w = A v on the 2D wavefront, the SpMV fused into the launch
// (GG_FUSE_SPMV): fused_spmv_ok says whether triangle T and A admit it
bool fused_spmv_ok(const DevTri &T, const DevCsr &A);
void launch_trsv_spmv(Gate g, DevTri &T, const DevCsr &A, const double *v, double *w, double *x, int *err,
                      hipStream_t st, const double *ydiv = nullptr,
                      const double *xdiv = nullptr);   // v[c] / xdiv[c] per gathered term
int wave_batch_steps(int div, bool d3 = false, int skew = 1);   // steps per batch of the wavefront kernel
int tile_batch_steps();                                          // steps per batch of the 3D tile kernel

// ---- GMRES scalar / MGS kernels ----------------------------------------------
void launch_set_normb(const double *part, int G, DevState *ds, hipStream_t st);
void launch_init_beta(const double *part, int G, DevState *ds, double *hist, hipStream_t st);
void launch_init_cycle(DevState *ds, const double *r, double *v0, double *s, int G, long long Ppad,
                       hipStream_t st);
void launch_mgs_step(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                     const double *part_in, double *part_out, double *H, int G, long long Ppad,
                     hipStream_t st);
// the same with a separate dot range [0, Pdot) and nparts_in input partials
// (the sharded solve: every shard's block partials after the all-gather)
void launch_mgs_step_r(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, int nparts_in, double *part_out, double *H, int G,
                       long long Ppad, long long Pdot, hipStream_t st);
// CGS2 (sharded solve, GG_SOLVE_CGS2): block partials of <w, v_k>, k < nk, at
// part[k*G + b]; every shard's partials of dot k summed into h[k] (shard q's
// slot at part + q*cnt) and into H[k, i] (add: +=); w -= sum_k h[k] v_k with
// the norm's block partials when part_norm is given
void launch_multidot(Gate g, const double *w, const double *V, long long ldv, int nk, double *part, int G,
                     long long Pdot, hipStream_t st);
void launch_cgs_reduce(Gate g, const double *part, int P, int G, long long cnt, int nk, double *h, double *H,
                       int i, int m, bool add, hipStream_t st);
void launch_cgs_update(Gate g, double *w, const double *V, long long ldv, const double *h, int nk, int G,
                       long long Ppad, long long Pdot, double *part_norm, hipStream_t st);
// the first CGS2 update and the second pass's dot partials in one launch
// (bit-identical to launch_cgs_update + launch_multidot); false: nk too large,
// nothing launched
bool launch_cgs_update_dot(Gate g, double *w, const double *V, long long ldv, const double *h, int nk, int G,
                           long long Ppad, long long Pdot, double *part, hipStream_t st);
void launch_arnoldi_finalize_r(Gate g, int i, int m, DevState *ds, const double *part, int nparts_in,
                               int G, const double *w, double *vnext, double *H, double *cs,
                               double *sn, double *s, double *hist, long long Ppad, hipStream_t st);
void launch_arnoldi_finalize(Gate g, int i, int m, DevState *ds, const double *part, int G,
                             const double *w, double *vnext, double *H, double *cs, double *sn,
                             double *s, double *hist, long long Ppad, hipStream_t st);
// persistent Arnoldi orthogonalization (one launch per inner iteration):
// units per thread (1/2/4/8, 0 = too many), how many blocks can be resident
int arnoldi_persist_units(int G, long long Ppad);
int arnoldi_persist_max_blocks(int J);
// xb: per inner step kMgsXcdWords words (the XCD-local gather's slots, kernels.hip
// gather_xcd; re-armed with the granules), elect: kMgsElectWords words (zeroed
// once), seq: strictly increasing per launch
constexpr int kMgsXcdWords = 8 * 16, kMgsElectWords = 8 * 16;
constexpr int kMgsXcds = 8;          // XCDs (GG_MGS_GATHER 3: one reducer-only block each)
int mgs_gather_form();   // GG_MGS_GATHER: 0 every block gathers, 2 XCD-local reducers, 3 reducer-only blocks
int mgs_prefetch();      // GG_MGS_PREFETCH: 1 v_{k+1} streamed during the gather, 0 after it
void launch_arnoldi_persist(Gate g, int i, int m, DevState *ds, const double *w, double *V,
                            long long ldv, double *H, double *cs, double *sn, double *s,
                            double *hist, unsigned long long *gran, unsigned long long *hg, int G,
                            long long Ppad, int *err, unsigned long long *xb, unsigned long long *elect,
                            unsigned long long seq, const UnitMap &um, hipStream_t st,
                            long long *trace = nullptr,    // diagnostics: GG_MGS_TRACE (solver.hip)
                            const double *msc = nullptr, double *mout = nullptr,    // + mout = v_{i+1} * msc
                            double *fill = nullptr, long long nfill = 0);            // + fill[< nfill] = sentinel
// two scenarios of the many-RHS batch per launch (scenario 1's buffers zs bytes
// after scenario 0's, gran / xb per scenario as above): units per thread when
// the grid can be co-resident, else 0
int arnoldi_persist2_units(int G, long long Ppad);
void launch_arnoldi_persist2(Gate g, long long zs, int i, int m, DevState *ds, const double *w, double *V,
                             long long ldv, double *H, double *cs, double *sn, double *s, double *hist,
                             unsigned long long *gran, int G, long long Ppad, int *err, unsigned long long *xb,
                             unsigned long long *elect, unsigned long long seq, const UnitMap &um, hipStream_t st);
// the same for long vectors (w on chip, the basis streamed): kWideG blocks
constexpr int kWideG = 512;
bool arnoldi_wide_ok(int G, long long Ppad);
void launch_arnoldi_wide(Gate g, int i, int m, DevState *ds, const double *w, double *V, long long ldv,
                         double *H, double *cs, double *sn, double *s, double *hist,
                         unsigned long long *gran, unsigned long long *hg, int G, long long Ppad, int *err,
                         const UnitMap &um, hipStream_t st);
void launch_update(Gate g, int m, DevState *ds, const double *H, const double *s, double *ysmall,
                   const double *V, long long ldv, double *acc, int G, long long Ppad, hipStream_t st,
                   const UnitMap &um = UnitMap{});
void launch_end_cycle(const double *part, int G, DevState *ds, double *hist, hipStream_t st);

// ---- batched (many-RHS) launches, kernels.hip: nsc scenarios per launch,
// scenario q's per-scenario buffers (vectors, partials, H, Givens, history,
// control block, hand-off granules) q * zs bytes after scenario 0's; the gate's
// done / nit likewise.  Same kernels and per-scenario arithmetic as above.
constexpr int kBatchSpmv = 8;     // scenarios per batched SpMV launch (A read once for them)
void launch_fill_u64_b(unsigned long long *p, long long n, unsigned long long v, int nsc, long long zs,
                       hipStream_t st);
// out_q[i] = idx[i] < 0 ? 0 : in_q[idx[i]]  (in / out strides zin / zout bytes)
void launch_gather_b(const double *in, long long zin, const long long *idx, double *out, long long zout,
                     long long n, int nsc, hipStream_t st);
void launch_init_state_b(DevState *ds, long long zs, int nsc, double tol, int max_iter, int m, hipStream_t st);
// out[q] = scenario q's control block, q < nsc; out[nsc].err = *err
void launch_pack_states_b(const DevState *ds, long long zs, int nsc, DevState *out, const int *err, hipStream_t st);
// u = each scenario's sources at time index it (soff: nsc + 1 offsets into the
// concatenated kind / dptr tables, maxsrc the largest count); w_q = B_q u + (C/h) x_q
// with scenario q's B^T rows at sptr + q * (n + 1) (sidx: global source indices)
void launch_transient_step_b(int n, int nsc, int maxsrc, const int *soff, const int *kind, const int *dptr,
                             const double *data, int it, double h, double *u, const int *sptr, const int *sidx,
                             const double *cdiag, const double *x, double *w, long long ldx, hipStream_t st);
void launch_gather_ports_b(int nport, const int *port, const double *x, long long ldx, double *out, long long ldo,
                           int nsc, hipStream_t st);
void launch_spmv_b(Gate g, const DevCsr &A, const double *x, const double *b, double *y, bool resid, int nsc,
                   long long zs, hipStream_t st);
// the 2D wavefront solve batched over scenarios (bnd: scenario 0's granules,
// trsv_b_granules(T) words per scenario, armed); trsv_batchable: T admits it
bool trsv_batchable(const DevTri &T);
long long trsv_b_granules(const DevTri &T);
int batch_zmap();   // GG_BATCH_ZMAP: workgroup -> (scenario, band) placement (kernels.hip trsv_wave2d_body)
void launch_trsv_b(Gate g, DevTri &T, const double *b, double *x, unsigned long long *bnd, int *err, int nsc,
                   long long zs, hipStream_t st);
void launch_dot_b(Gate g, const double *a, const double *b, double *part, int G, long long Ppad, int nsc,
                  long long zs, hipStream_t st);
void launch_set_normb_b(const double *part, int G, DevState *ds, int nsc, long long zs, hipStream_t st);
void launch_init_beta_b(const double *part, int G, DevState *ds, double *hist, int nsc, long long zs, hipStream_t st);
void launch_init_cycle_b(DevState *ds, const double *r, double *v0, double *s, int G, long long Ppad, int nsc,
                         long long zs, hipStream_t st);
void launch_mgs_step_b(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, double *part_out, double *H, int G, long long Ppad, int nsc,
                       long long zs, hipStream_t st);
void launch_arnoldi_finalize_b(Gate g, int i, int m, DevState *ds, const double *part, int G, const double *w,
                               double *vnext, double *H, double *cs, double *sn, double *s, double *hist,
                               long long Ppad, int nsc, long long zs, hipStream_t st);
void launch_update_b(Gate g, int m, DevState *ds, const double *H, const double *s, double *ysmall, const double *V,
                     long long ldv, double *acc, int G, long long Ppad, const UnitMap &um, int nsc, long long zs,
                     hipStream_t st);
void launch_end_cycle_b(const double *part, int G, DevState *ds, double *hist, int nsc, long long zs, hipStream_t st);

}  // namespace gg
