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
// 64 grid lines, lane l = line 64*band+l, step t = column i + l; a lane's two
// consecutive steps are adjacent in memory (16 B per array per step pair, 1 KiB
// per wave instruction).
//
// One workgroup per band, four waves, one per SIMD:
//  * wave 0 (compute) runs the recurrence: each step a lane needs its own
//    previous value (same line, column i-+1) and the neighbour line's value
//    from the previous step, moved in-register with DPP wave_shr/wave_shl.  It
//    reads right-hand side and coefficients from LDS only, so its vector-memory
//    queue holds nothing but fire-and-forget stores;
//  * waves 2-3 (loaders) stream b / coefficients HBM -> LDS with LDS-DMA
//    (global_load_lds_dwordx4) into a kWaveR-slot ring, kWaveR-1 batches ahead,
//    each retiring a batch with its own counted vmcnt before the barrier;
//  * wave 1 (boundary) polls the neighbouring band's edge-lane values one batch
//    ahead and hands them over through LDS.
// The four waves meet at one raw s_barrier per 16-step batch (no fence, no
// drain).  Band-to-band hand-off (workgroups on different CUs): 8-byte granules
// whose payload is the flag (sentinel = not ready): the producing compute wave
// stores one 16-lane batch per 16 steps with relaxed agent-scope (sc1) stores;
// the boundary wave polls with relaxed agent-scope loads and re-arms each slot
// (sc1 sentinel store) for the next launch.  Every spin is bounded.
constexpr int kWaveBatch = 16;             // steps per batch
constexpr int kWavePB = kWaveBatch / 2;    // step pairs per batch
constexpr int kWaveR = 4;                  // LDS ring slots (batches)
constexpr int kSpinLimit = 1 << 20;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// s_waitcnt immediate: wait until <= n vector-memory ops are outstanding (gfx9)
__host__ __device__ constexpr int vm_wait(int n)
{
    return (n & 15) | (7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14);
}

__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// loader wave: NA arrays starting at a0, batch j -> ring slot j % kWaveR
template <bool FWD, int A, int NA>
__device__ __forceinline__ void wave_loader(const double2 *const *src, int a0, double2 *lds, int np,
                                            int nbatch)
{
    constexpr int SLOT = A * kWavePB * 64;      // double2 per ring slot
    constexpr int NPER = NA * kWavePB;          // DMA instructions per batch
    auto issue = [&](int j) {
        double2 *slot = lds + (j % kWaveR) * SLOT;
#pragma unroll
        for (int ai = 0; ai < NA; ai++)
#pragma unroll
            for (int kk = 0; kk < kWavePB; kk++) {
                const int p = j * kWavePB + kk;
                const long long q = (long long)(FWD ? p : np - 1 - p) * 64;
                __builtin_amdgcn_global_load_lds((gbl_void_t *)(src[a0 + ai] + q),
                                                 (lds_void_t *)(slot + (a0 + ai) * kWavePB * 64 + kk * 64),
                                                 16, 0, 0);
            }
    };
    for (int j = 0; j < kWaveR - 1 && j < nbatch; j++) issue(j);
    for (int j = 0; j < nbatch; j++) {
        // batch j has landed when at most the batches issued after it are in flight
        const int after = (j + kWaveR - 1 < nbatch ? j + kWaveR - 1 : nbatch) - j - 1;
        if (after >= 2) __builtin_amdgcn_s_waitcnt(vm_wait(2 * NPER));
        else if (after == 1) __builtin_amdgcn_s_waitcnt(vm_wait(NPER));
        else __builtin_amdgcn_s_waitcnt(vm_wait(0));
        raw_barrier();                          // batch j visible; slot (j-1) % R free
        if (j + kWaveR - 1 < nbatch) issue(j + kWaveR - 1);
    }
}

template <bool FWD, bool UNIT>
__global__ __launch_bounds__(256) void k_trsv_wave2d(Gate g, int nx, int T, int nbands,
                                                     const double *__restrict__ b,
                                                     const double *__restrict__ c1,
                                                     const double *__restrict__ c2,
                                                     const double *__restrict__ dv,
                                                     double *__restrict__ x,
                                                     unsigned long long *bnd, int *err)
{
    static_assert(kWaveR == 4, "loader waits are written for a 4-slot ring");
    if (gated(g)) return;
    constexpr int A = UNIT ? 3 : 4;             // streamed arrays: b, c1, c2 (, d)
    constexpr int SLOT = A * kWavePB * 64;      // double2 per ring slot
    // one LDS object: data ring, then the 2 x 16 boundary values
    __shared__ double2 lds[kWaveR * SLOT + kWaveBatch];
    double *bring = reinterpret_cast<double *>(lds + kWaveR * SLOT);
    const int band = FWD ? blockIdx.x : (nbands - 1 - blockIdx.x);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int np = T / 2;                       // step pairs per band
    const int nbatch = T / kWaveBatch;          // T is a multiple of kWaveBatch
    const bool has_src = FWD ? (band > 0) : (band < nbands - 1);
    const bool is_prod = FWD ? (band < nbands - 1) : (band > 0);
    const long long boff = (long long)band * np * 64 + lane;    // double2 units

    if (wave >= 2) {
        // ------------------------------------------------ loader waves
        const double2 *src[4] = {reinterpret_cast<const double2 *>(b) + boff,
                                 reinterpret_cast<const double2 *>(c1) + boff,
                                 reinterpret_cast<const double2 *>(c2) + boff,
                                 UNIT ? nullptr : reinterpret_cast<const double2 *>(dv) + boff};
        if (wave == 2) wave_loader<FWD, A, 2>(src, 0, lds, np, nbatch);
        else wave_loader<FWD, A, A - 2>(src, 2, lds, np, nbatch);
        return;
    }
    if (wave == 1) {
        // ------------------------------------------------ boundary wave
        // before barrier j it has placed batch j's values in bring[j & 1];
        // between barriers j and j+1 it fetches batch j+1
        unsigned long long *src = bnd + (long long)(FWD ? band - 1 : band + 1) * nx;
        bool dead = false;
        for (int bi = 0; bi < nbatch; bi++) {
            if (has_src) {
                // column the compute wave's edge lane needs at step `lane` of batch bi
                const int t = FWD ? bi * kWaveBatch + lane : (T - 1) - (bi * kWaveBatch + lane);
                const int c = FWD ? t : t - 63;
                const int col = (lane < kWaveBatch && c >= 0 && c < nx) ? c : -1;
                unsigned long long v = (col >= 0 && !dead) ? ld_agent(src + col) : 0ull;
                int spins = 0;
                while (!dead && !__all(col < 0 || v != kSentinel)) {
                    __builtin_amdgcn_s_sleep(1);
                    if (col >= 0 && v == kSentinel) v = ld_agent(src + col);
                    if (++spins > kSpinLimit) {
                        dead = true;
                        if (lane == 0) atomicOr(err, 1);
                    }
                }
                if (col >= 0) st_agent(src + col, kSentinel);   // re-arm for the next launch
                if (lane < kWaveBatch)
                    bring[(bi & 1) * kWaveBatch + lane] =
                        (col >= 0) ? __longlong_as_double((long long)v) : 0.0;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            raw_barrier();
        }
        return;
    }

    // ---------------------------------------------------- compute wave
    double2 *X2 = reinterpret_cast<double2 *>(x) + boff;
    constexpr int edge = FWD ? 0 : 63;      // lane that consumes the boundary
    constexpr int plane = FWD ? 63 : 0;     // lane whose values the next band needs
    unsigned long long *dst = bnd + (long long)band * nx;
    double xp = 0.0;                        // this lane's previous step value
    double bacc = 0.0;                      // producer-lane values of this batch (lane k = step k)
    for (int bi = 0; bi < nbatch; bi++) {
        raw_barrier();                      // batch bi's data and boundary values are in LDS
        const double2 *sl = lds + (bi % kWaveR) * SLOT + lane;
        const double bv = (has_src && lane < kWaveBatch) ? bring[(bi & 1) * kWaveBatch + lane] : 0.0;
#pragma unroll
        for (int kk = 0; kk < kWavePB; kk++) {
            const int p = bi * kWavePB + kk;
            const double2 cb = sl[0 * kWavePB * 64 + kk * 64];
            const double2 a1 = sl[1 * kWavePB * 64 + kk * 64];
            const double2 a2 = sl[2 * kWavePB * 64 + kk * 64];
            double2 dd = make_double2(1.0, 1.0);
            if (!UNIT) dd = sl[3 * kWavePB * 64 + kk * 64];
            double xo0 = 0.0, xo1 = 0.0;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int tt = 2 * kk + h;                       // step within the batch
                const bool sx = FWD ? (h == 0) : (h == 1);       // even step <-> .x
                const double bb = sx ? cb.x : cb.y, e1 = sx ? a1.x : a1.y, e2 = sx ? a2.x : a2.y;
                double xs = FWD ? dpp_shr1(xp) : dpp_shl1(xp);
                const double bval = readlane_d(bv, tt);
                if (lane == edge) xs = has_src ? bval : 0.0;
                double acc = bb - e1 * xs;      // line neighbour first (|offset| = nx)
                acc = acc - e2 * xp;            // then the in-line neighbour (|offset| = 1)
                if (!UNIT) acc = acc / (sx ? dd.x : dd.y);
                xp = acc;
                if (sx) xo0 = acc; else xo1 = acc;
                const double pv = readlane_d(acc, plane);
                if (lane == tt) bacc = pv;
            }
            X2[(long long)(FWD ? p : np - 1 - p) * 64] = make_double2(xo0, xo1);
        }
        // ---- publish this batch's producer-lane values (lanes 0..15), issued by
        //      every lane (lanes with nothing to publish write a dummy slot)
        {
            const int t = FWD ? bi * kWaveBatch + lane : (T - 1) - (bi * kWaveBatch + lane);
            const int c = FWD ? t - 63 : t;
            const bool real = is_prod && lane < kWaveBatch && c >= 0 && c < nx;
            st_agent(real ? dst + c : bnd + (long long)nbands * nx + lane,
                     (unsigned long long)__double_as_longlong(bacc));
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
        dim3 grid(w.nbands), blk(256);
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
