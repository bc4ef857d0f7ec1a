// kernels.hip -- hand-written gfx950 (CDNA4) kernels for the GMRES hot path.
//
// Arithmetic order: every kernel that has a serial counterpart in the
// reference (SpMV row sums, triangular-solve rows, AXPY, Update) evaluates
// the same expression in the same order with contraction disabled
// (-ffp-contract=off), so it is bit-identical to the fp64 restatement.  Only
// the dot products / norms (wave-shuffle trees) round differently.
//
// Wave = 64 lanes; vector kernels use 256-thread blocks and 16-B (double2)
// loads; every reduction is a fixed tree (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace gg {

namespace {

__device__ __forceinline__ bool gated(const Gate &g)
{
    if (g.done && (*g.done & g.mask)) return true;
    if (g.nit && g.i >= *g.nit) return true;
    return false;
}

// ---- reductions -------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// 256-thread block sum, result broadcast to every thread.
__device__ __forceinline__ double block_sum(double v)
{
    __shared__ double sh[kBlock / 64];
    __shared__ double res;
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) res = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    double r = res;
    __syncthreads();
    return r;
}

// Sum of G per-block partials, identical (bit-for-bit) in every block.
__device__ __forceinline__ double sum_partials(const double *part, int G)
{
    double v = 0.0;
    for (int k = threadIdx.x; k < G; k += kBlock) v += part[k];
    return block_sum(v);
}

__device__ __forceinline__ double2 ld2(const double *p, long long u)
{
    return reinterpret_cast<const double2 *>(p)[u];
}
__device__ __forceinline__ void st2(double *p, long long u, double2 v)
{
    reinterpret_cast<double2 *>(p)[u] = v;
}

// ---- DPP lane shifts (gfx9 wave_shr:1 / wave_shl:1) -----------------------------
__device__ __forceinline__ double dpp_shr1(double v)
{
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1(double v)
{
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int l)
{
    int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ============================================================== vector ops
__global__ void k_fill_u64(unsigned long long *p, long long n, unsigned long long v)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_gather(const double *in, const long long *idx, double *out, long long n)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        long long s = idx[i];
        out[i] = s < 0 ? 0.0 : in[s];
    }
}

__global__ void k_copy(const double *in, double *out, long long units)
{
    for (long long u = blockIdx.x * (long long)blockDim.x + threadIdx.x; u < units;
         u += (long long)gridDim.x * blockDim.x)
        st2(out, u, ld2(in, u));
}

__global__ __launch_bounds__(kBlock) void k_dot(Gate g, const double *a, const double *b,
                                                double *part, long long units)
{
    if (gated(g)) return;
    double acc = 0.0;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        double2 x = ld2(a, u), y = ld2(b, u);
        acc += x.x * y.x;
        acc += x.y * y.y;
    }
    acc = block_sum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// ------------------------------------------------------- split (PG) maps
// MyILUPPfloat::DevPrecond_* elementwise steps (src/preconditioner.cu:1424-1558)
__global__ void k_mul(Gate g, const double *in, const double *s, double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] * s[i];
}
__global__ void k_div(Gate g, const double *in, const double *s, double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] / s[i];
}
__global__ void k_gather_divsrc(Gate g, const double *in, const double *s, const int *perm,
                                double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { int p = perm[i]; out[i] = in[p] / s[p]; }
}
__global__ void k_gather_divdst(Gate g, const double *in, const double *s, const int *perm,
                                double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[perm[i]] / s[i];
}
__global__ void k_scatter_mul(Gate g, const double *in, const double *s, const int *perm,
                              double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[perm[i]] = in[i] * s[i];
}

// ================================================================= SpMV
// CSR-stream: a block owns <=256 consecutive rows holding <=kSpmvCap nnz.
// Products v*x[col] are formed with coalesced loads into LDS, then each row is
// summed serially in CSR order (computeSpMV order, src/SpMV_compute.cpp:19-36).
template <bool RESID>
__global__ __launch_bounds__(kBlock) void k_spmv_stream(Gate g, const int *blk, const int *rp,
                                                        const int *ci, const double *v,
                                                        const double *x, const double *b,
                                                        double *y)
{
    if (gated(g)) return;
    __shared__ double prod[kSpmvCap];
    const int r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const int e0 = rp[r0], e1 = rp[r1];
    const int cnt = e1 - e0;
    if (cnt > kSpmvCap) {   // one long row: strided partial sums + tree
        double acc = 0.0;
        for (int e = e0 + threadIdx.x; e < e1; e += kBlock) acc += v[e] * x[ci[e]];
        acc = block_sum(acc);
        if (threadIdx.x == 0) y[r0] = RESID ? (-1.0 * acc + 1.0 * b[r0]) : acc;
        return;
    }
    for (int e = threadIdx.x; e < cnt; e += kBlock) prod[e] = v[e0 + e] * x[ci[e0 + e]];
    __syncthreads();
    const int r = r0 + threadIdx.x;
    if (r < r1) {
        double acc = 0.0;
        const int a = rp[r] - e0, z = rp[r + 1] - e0;
        for (int e = a; e < z; e++) acc += prod[e];
        y[r] = RESID ? (-1.0 * acc + 1.0 * b[r]) : acc;
    }
}

// ======================================================= triangular solves
// Level-scheduled row solve (one launch per dependency level):
//   x[r] = (b[r] - sum_k off[k] * x[col[k]]) / d[r]   in canonical order
__global__ __launch_bounds__(kBlock) void k_trsv_level(Gate g, int cnt, const int *rows,
                                                       const int *rp, const int *ci,
                                                       const double *v, const double *d,
                                                       const double *b, double *x)
{
    if (gated(g)) return;
    int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= cnt) return;
    int r = rows[t];
    double acc = b[r];
    for (int k = rp[r]; k < rp[r + 1]; k++) acc = acc - v[k] * x[ci[k]];
    x[r] = acc / d[r];
}

// 2D structured-grid wavefront solve.  Layout (gg_internal.h Wave2D): band =
// 64 grid lines = one wave, lane l = line 64*band+l, step t = column i + l.
// Each step a lane needs its own previous value (same line, column i-+1) and
// the neighbour line's value from the previous step, moved in-register with
// DPP wave_shr/wave_shl.  The band boundary (lane 0 / lane 63) is exchanged
// between bands (workgroups on different CUs) through 8-byte granules whose
// payload is the flag (sentinel = not ready): relaxed agent-scope (sc1) store
// by the producer lane, relaxed agent-scope polling loads by the consumer,
// which resets the slot for the next launch.
constexpr int kWaveBatch = 16;
constexpr int kSpinLimit = 1 << 20;

template <bool FWD, bool UNIT>
__global__ __launch_bounds__(64) void k_trsv_wave2d(Gate g, int nx, int T, int nbands,
                                                    const double *__restrict__ b,
                                                    const double *__restrict__ c1,
                                                    const double *__restrict__ c2,
                                                    const double *__restrict__ dv,
                                                    double *__restrict__ x,
                                                    unsigned long long *bnd, int *err)
{
    if (gated(g)) return;
    const int band = FWD ? blockIdx.x : (nbands - 1 - blockIdx.x);
    const int lane = threadIdx.x;
    const long long base = (long long)band * T * 64 + lane;
    const bool has_src = FWD ? (band > 0) : (band < nbands - 1);
    const bool is_prod = FWD ? (band < nbands - 1) : (band > 0);
    const int edge = FWD ? 0 : 63;          // lane that consumes the boundary
    unsigned long long *src = bnd + (long long)(FWD ? band - 1 : band + 1) * nx;
    unsigned long long *dst = bnd + (long long)band * nx;

    double xp = 0.0;                        // this lane's previous step value
    const int nbatch = T / kWaveBatch;      // T is a multiple of kWaveBatch
    bool dead = false;                      // gave up waiting once: never wait again
    for (int bi = 0; bi < nbatch; bi++) {
        // ---- boundary batch: lane k holds the value the edge lane needs at
        //      batch step k (FWD: column t; BWD: column t-63)
        double bv = 0.0;
        if (has_src && !dead) {
            const int tk = FWD ? bi * kWaveBatch + lane : (T - 1) - (bi * kWaveBatch + lane);
            const int col = FWD ? tk : tk - 63;
            const bool need = lane < kWaveBatch && col >= 0 && col < nx &&
                              (FWD ? tk < T : tk >= 0);
            unsigned long long bits = kSentinel;
            int spins = 0;
            while (true) {
                if (need) bits = ld_agent(src + col);
                const bool ok = !need || bits != kSentinel;
                if (__all(ok)) break;
                if (++spins > kSpinLimit) {
                    if (lane == 0) atomicOr(err, 1);
                    dead = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (need) {
                bv = __longlong_as_double((long long)bits);
                src[col] = kSentinel;   // re-arm for the next launch
            }
        }
#pragma unroll
        for (int tt = 0; tt < kWaveBatch; tt++) {
            const int t = FWD ? bi * kWaveBatch + tt : (T - 1) - (bi * kWaveBatch + tt);
            const long long idx = base + (long long)t * 64;
            const double bb = b[idx], a1 = c1[idx], a2 = c2[idx];
            double xs = FWD ? dpp_shr1(xp) : dpp_shl1(xp);
            const double bval = readlane_d(bv, tt);
            if (lane == edge) xs = has_src ? bval : 0.0;
            double acc = bb - a1 * xs;      // line neighbour first (|offset| = nx)
            acc = acc - a2 * xp;            // then the in-line neighbour (|offset| = 1)
            if (!UNIT) acc = acc / dv[idx];
            xp = acc;
            x[idx] = acc;
            if (is_prod) {
                if (FWD) {
                    if (lane == 63 && t - 63 >= 0 && t - 63 < nx)
                        st_agent(dst + (t - 63), (unsigned long long)__double_as_longlong(acc));
                } else {
                    if (lane == 0 && t < nx)
                        st_agent(dst + t, (unsigned long long)__double_as_longlong(acc));
                }
            }
        }
    }
}

// ============================================================ GMRES kernels
__global__ void k_set_normb(const double *part, int G, DevState *ds)
{
    double s = sum_partials(part, G);
    if (threadIdx.x == 0) {
        double nb = sqrt(s);
        ds->normb = (nb == 0.0) ? 1.0 : nb;     // src/gmres.cu:604
    }
}

__global__ void k_init_beta(const double *part, int G, DevState *ds, double *hist)
{
    double s = sum_partials(part, G);
    if (threadIdx.x == 0) {
        double beta = sqrt(s);
        double resid = beta / ds->normb;
        ds->beta = beta;
        ds->resid = resid;
        hist[0] = resid;
        ds->hist_len = 1;
        ds->j = 1;
        if (resid <= ds->tol) ds->done = DONE_INIT;   // "<=" (src/gmres.cu:608)
    }
}

// v0 = r * (1/beta); s = 0; s[0] = beta; nit = min(m, max_iter - j + 1)
__global__ __launch_bounds__(kBlock) void k_init_cycle(DevState *ds, const double *r, double *v0,
                                                       double *s, long long units)
{
    if (ds->done) return;
    const double beta = ds->beta;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int nit = ds->max_iter - ds->j + 1;
        if (nit > ds->m) nit = ds->m;
        ds->nit = nit;
        for (int k = 0; k <= ds->m; k++) s[k] = 0.0;
        s[0] = beta;
    }
    const double inv = 1.0 / beta;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        double2 a = ld2(r, u);
        a.x = inv * a.x;
        a.y = inv * a.y;
        st2(v0, u, a);
    }
}

// One MGS step k of inner iteration i (src/gmres.cu:638-641):
//   h = <w, v_k> (from the previous kernel's partials); H[k,i] = h;
//   w = (-h) v_k + w;  partials of <w, vnext>  (vnext = v_{k+1}, or w for the norm)
__global__ __launch_bounds__(kBlock) void k_mgs_step(Gate g, int i, int k, int m, double *w,
                                                     const double *vk, const double *vnext,
                                                     const double *part_in, double *part_out,
                                                     double *H, int G, long long units)
{
    if (gated(g)) return;
    const double h = sum_partials(part_in, G);
    if (blockIdx.x == 0 && threadIdx.x == 0) H[k + i * (m + 1)] = h;
    const double a = -h;
    double acc = 0.0;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        double2 wv = ld2(w, u), vv = ld2(vk, u);
        wv.x = a * vv.x + wv.x;
        wv.y = a * vv.y + wv.y;
        st2(w, u, wv);
        double2 nv = (vnext == w) ? wv : ld2(vnext, u);
        acc += wv.x * nv.x;
        acc += wv.y * nv.y;
    }
    acc = block_sum(acc);
    if (threadIdx.x == 0) part_out[blockIdx.x] = acc;
}

__device__ __forceinline__ void apply_rot(double &dx, double &dy, double cs, double sn)
{
    double temp = cs * dx + sn * dy;     // ApplyPlaneRotation (src/gmres.cu:192-197)
    dy = -sn * dx + cs * dy;
    dx = temp;
}
__device__ __forceinline__ void gen_rot(double dx, double dy, double &cs, double &sn)
{
    if (dy == 0.0) { cs = 1.0; sn = 0.0; }   // GeneratePlaneRotation (:200-216)
    else if (fabs(dy) > fabs(dx)) {
        double temp = dx / dy;
        sn = 1.0 / sqrt(1.0 + temp * temp);
        cs = temp * sn;
    } else {
        double temp = dy / dx;
        cs = 1.0 / sqrt(1.0 + temp * temp);
        sn = temp * cs;
    }
}

// H[i+1,i] = ||w||; Givens on column i; residual check; v_{i+1} = w * (1/H[i+1,i])
__global__ __launch_bounds__(kBlock) void k_arnoldi_finalize(Gate g, int i, int m, DevState *ds,
                                                             const double *part, int G,
                                                             const double *w, double *vnext,
                                                             double *H, double *cs, double *sn,
                                                             double *s, double *hist,
                                                             long long units)
{
    if (gated(g)) return;
    const double hn = sqrt(sum_partials(part, G));
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int ld = m + 1;
        double *Hc = H + i * ld;
        Hc[i + 1] = hn;
        for (int k = 0; k < i; k++) apply_rot(Hc[k], Hc[k + 1], cs[k], sn[k]);
        double c, sv;
        gen_rot(Hc[i], Hc[i + 1], c, sv);
        cs[i] = c;
        sn[i] = sv;
        apply_rot(Hc[i], Hc[i + 1], c, sv);
        apply_rot(s[i], s[i + 1], c, sv);
        const double resid = fabs(s[i + 1]) / ds->normb;
        hist[ds->hist_len + i] = resid;
        ds->resid = resid;
        if (resid < ds->tol) {               // "<" (src/gmres.cu:654)
            ds->conv_i = i;
            ds->done = DONE_INNER;
        }
    }
    // lucky breakdown (hn == 0): the reference divides by zero; v_{i+1} := 0
    const double inv = (hn != 0.0) ? 1.0 / hn : 0.0;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        double2 a = ld2(w, u);
        a.x = inv * a.x;
        a.y = inv * a.y;
        st2(vnext, u, a);
    }
}

// y = H(0:k,0:k)^-1 s(0:k)  (Update, src/gmres.cu:93-116); k = conv_i or nit-1
__global__ void k_update_y(Gate g, int m, DevState *ds, const double *H, const double *s,
                           double *y)
{
    if (gated(g)) return;
    if (threadIdx.x != 0) return;
    const int k = (ds->done & DONE_INNER) ? ds->conv_i : ds->nit - 1;
    ds->upd_k = k;
    const int ld = m + 1;
    for (int i = 0; i <= k; i++) y[i] = s[i];
    for (int i = k; i >= 0; i--) {
        y[i] /= H[i + i * ld];
        for (int j = i - 1; j >= 0; j--) y[j] -= H[j + i * ld] * y[i];
    }
}

// acc += sum_{j<=k} V_j y_j   (ascending j, as the reference's x[i] += v*y loop)
__global__ __launch_bounds__(kBlock) void k_update_x(Gate g, const DevState *ds, const double *y,
                                                     const double *V, long long ldv, double *acc,
                                                     long long units)
{
    if (gated(g)) return;
    const int k = ds->upd_k;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        double2 a = ld2(acc, u);
        for (int j = 0; j <= k; j++) {
            const double yj = y[j];
            double2 vv = ld2(V + j * ldv, u);
            a.x = a.x + vv.x * yj;
            a.y = a.y + vv.y * yj;
        }
        st2(acc, u, a);
    }
}

// beta = ||r|| after a restart; history; j += nit
__global__ void k_end_cycle(const double *part, int G, DevState *ds, double *hist)
{
    if (ds->done) return;
    double s = sum_partials(part, G);
    if (threadIdx.x == 0) {
        double beta = sqrt(s);
        double resid = beta / ds->normb;
        ds->beta = beta;
        ds->resid = resid;
        hist[ds->hist_len + ds->nit] = resid;
        ds->hist_len += ds->nit + 1;
        ds->j += ds->nit;
        if (resid < ds->tol) ds->done = DONE_RESTART;   // "<" (src/gmres.cu:686)
    }
}

inline int blocks_for(long long n, int bs = kBlock, int cap = 65535)
{
    long long b = (n + bs - 1) / bs;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

}  // namespace

// ======================================================= host launchers
int reduce_grid(long long units)
{
    long long g = (units + kBlock * 4 - 1) / (kBlock * 4);   // >= 8 elements / thread
    if (g < 1) g = 1;
    if (g > 1024) g = 1024;
    return (int)g;
}

void launch_fill_u64(unsigned long long *p, long long n, unsigned long long v, hipStream_t st)
{
    k_fill_u64<<<blocks_for(n, kBlock, 4096), kBlock, 0, st>>>(p, n, v);
}
void launch_gather(const double *in, const long long *idx, double *out, long long n, hipStream_t st)
{
    k_gather<<<blocks_for(n, kBlock, 8192), kBlock, 0, st>>>(in, idx, out, n);
}
void launch_copy(const double *in, double *out, long long n, hipStream_t st)
{
    k_copy<<<blocks_for(n / 2, kBlock, 8192), kBlock, 0, st>>>(in, out, n / 2);
}
void launch_dot(Gate g, const double *a, const double *b, double *part, int G, long long Ppad,
                hipStream_t st)
{
    k_dot<<<G, kBlock, 0, st>>>(g, a, b, part, Ppad / 2);
}

void launch_mul(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st)
{
    k_mul<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, out, n);
}
void launch_div(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st)
{
    k_div<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, out, n);
}
void launch_gather_divsrc(Gate g, const double *in, const double *s, const int *perm, double *out,
                          int n, hipStream_t st)
{
    k_gather_divsrc<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, perm, out, n);
}
void launch_gather_divdst(Gate g, const double *in, const double *s, const int *perm, double *out,
                          int n, hipStream_t st)
{
    k_gather_divdst<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, perm, out, n);
}
void launch_scatter_mul(Gate g, const double *in, const double *s, const int *perm, double *out,
                        int n, hipStream_t st)
{
    k_scatter_mul<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, perm, out, n);
}

void launch_spmv(Gate g, const DevCsr &A, const double *x, const double *b, double *y, bool resid,
                 hipStream_t st)
{
    if (A.nblk == 0) return;
    if (resid)
        k_spmv_stream<true><<<A.nblk, kBlock, 0, st>>>(g, A.blk.p, A.rp.p, A.ci.p, A.v.p, x, b, y);
    else
        k_spmv_stream<false><<<A.nblk, kBlock, 0, st>>>(g, A.blk.p, A.rp.p, A.ci.p, A.v.p, x, b, y);
}

void launch_trsv(Gate g, DevTri &T, const double *b, double *x, int *err, hipStream_t st)
{
    if (T.kind == DevTri::LEVEL) {
        const int nlev = (int)T.lev_ptr.size() - 1;
        for (int l = 0; l < nlev; l++) {
            const int cnt = T.lev_ptr[l + 1] - T.lev_ptr[l];
            if (cnt == 0) continue;
            k_trsv_level<<<(cnt + kBlock - 1) / kBlock, kBlock, 0, st>>>(
                g, cnt, T.lev_rows.p + T.lev_ptr[l], T.off.rp.p, T.off.ci.p, T.off.v.p, T.d.p, b, x);
        }
    } else if (T.kind == DevTri::WAVE2D) {
        const Wave2D &w = T.wl;
        dim3 grid(w.nbands), blk(64);
        if (T.lower) {
            if (T.unit)
                k_trsv_wave2d<true, true><<<grid, blk, 0, st>>>(g, w.nx, w.T, w.nbands, b, T.c1.p,
                                                                T.c2.p, nullptr, x, T.bnd.p, err);
            else
                k_trsv_wave2d<true, false><<<grid, blk, 0, st>>>(g, w.nx, w.T, w.nbands, b, T.c1.p,
                                                                 T.c2.p, T.dw.p, x, T.bnd.p, err);
        } else {
            if (T.unit)
                k_trsv_wave2d<false, true><<<grid, blk, 0, st>>>(g, w.nx, w.T, w.nbands, b, T.c1.p,
                                                                 T.c2.p, nullptr, x, T.bnd.p, err);
            else
                k_trsv_wave2d<false, false><<<grid, blk, 0, st>>>(g, w.nx, w.T, w.nbands, b, T.c1.p,
                                                                  T.c2.p, T.dw.p, x, T.bnd.p, err);
        }
    }
}

void launch_set_normb(const double *part, int G, DevState *ds, hipStream_t st)
{
    k_set_normb<<<1, kBlock, 0, st>>>(part, G, ds);
}
void launch_init_beta(const double *part, int G, DevState *ds, double *hist, hipStream_t st)
{
    k_init_beta<<<1, kBlock, 0, st>>>(part, G, ds, hist);
}
void launch_init_cycle(DevState *ds, const double *r, double *v0, double *s, int G, long long Ppad,
                       hipStream_t st)
{
    k_init_cycle<<<G, kBlock, 0, st>>>(ds, r, v0, s, Ppad / 2);
}
void launch_mgs_step(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                     const double *part_in, double *part_out, double *H, int G, long long Ppad,
                     hipStream_t st)
{
    k_mgs_step<<<G, kBlock, 0, st>>>(g, i, k, m, w, vk, vnext, part_in, part_out, H, G, Ppad / 2);
}
void launch_arnoldi_finalize(Gate g, int i, int m, DevState *ds, const double *part, int G,
                             const double *w, double *vnext, double *H, double *cs, double *sn,
                             double *s, double *hist, long long Ppad, hipStream_t st)
{
    k_arnoldi_finalize<<<G, kBlock, 0, st>>>(g, i, m, ds, part, G, w, vnext, H, cs, sn, s, hist,
                                              Ppad / 2);
}
void launch_update(Gate g, int m, DevState *ds, const double *H, const double *s, double *ysmall,
                   const double *V, long long ldv, double *acc, int G, long long Ppad, hipStream_t st)
{
    k_update_y<<<1, 64, 0, st>>>(g, m, ds, H, s, ysmall);
    k_update_x<<<G, kBlock, 0, st>>>(g, ds, ysmall, V, ldv, acc, Ppad / 2);
}
void launch_end_cycle(const double *part, int G, DevState *ds, double *hist, hipStream_t st)
{
    k_end_cycle<<<1, kBlock, 0, st>>>(part, G, ds, hist);
}

}  // namespace gg
