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
#include <type_traits>

#include "kernels.h"

namespace gg {

namespace {

__device__ __forceinline__ bool gated(const Gate &g)
{
    if (g.done && (*g.done & g.mask)) return true;
    if (g.nit && g.i >= *g.nit) return true;
    return false;
}

// Batched launches (kernels.h, the many-RHS solve): scenario sc's copy of a
// per-scenario buffer (vectors, partials, H, the control block, hand-off
// granules -- one arena per scenario) lies sc * zs bytes after scenario 0's.
// zs = 0: the single-scenario launch, every pointer as given.
// (char-pointer arithmetic, not an integer round trip: the compiler keeps the
// global address space -- global_* instead of flat_* accesses, which the
// wavefront kernel's writer could not afford)
template <class T>
__device__ __forceinline__ T *zp(T *p, long long zs, int sc)
{
    using C = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return reinterpret_cast<T *>(reinterpret_cast<C *>(p) + (long long)sc * zs);
}
__device__ __forceinline__ bool gated_z(const Gate &g, long long zs, int sc)
{
    Gate h = g;
    if (g.done) h.done = zp(g.done, zs, sc);
    if (g.nit) h.nit = zp(g.nit, zs, sc);
    return gated(h);
}

// ---- reductions -------------------------------------------------------------
// The xor butterfly v += v[lane ^ o], o = 32, 16, .., 1 (every lane ends with
// the same sum).  After the steps above o, v depends only on the lane bits
// below 2o, so any lane that agrees with lane ^ o on the bits below o and
// differs in bit o holds v[lane ^ o]: in-place v_permlane32 / 16 swaps (o =
// 32, 16) and DPP row_ror:o within rows of 16 (o = 8 .. 1; adding o mod 16
// flips bit o and keeps the lower bits).  The same operands in the same order
// as the ds_bpermute form (__shfl_xor), so the same bits, at VALU latency
// instead of six LDS round trips.  GG_WAVE_SUM_SHFL=1 keeps __shfl_xor.
#ifndef GG_WAVE_SUM_SHFL
#define GG_WAVE_SUM_SHFL 0
#endif
__device__ __forceinline__ unsigned perm32_self(unsigned v)
{
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0" : "+v"(v));
    return v;
}
__device__ __forceinline__ unsigned perm16_self(unsigned v)
{
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0" : "+v"(v));
    return v;
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double v)
{
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum(double v)
{
    if constexpr (GG_WAVE_SUM_SHFL) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        return v;
    } else {
        v += __hiloint2double((int)perm32_self((unsigned)__double2hiint(v)),
                              (int)perm32_self((unsigned)__double2loint(v)));
        v += __hiloint2double((int)perm16_self((unsigned)__double2hiint(v)),
                              (int)perm16_self((unsigned)__double2loint(v)));
        v += dpp64<0x128>(v);       // row_ror:8
        v += dpp64<0x124>(v);       // row_ror:4
        v += dpp64<0x122>(v);       // row_ror:2
        v += dpp64<0x121>(v);       // row_ror:1
        return v;
    }
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

// block_sum with one barrier instead of three, the same bits (the same
// wave_sum per wave and (0 + 1) + (2 + 3)), every thread forming the sum from
// the four wave sums itself: the wave sums alternate between two LDS rows
// (`par`, uniform, flipped per call), so a call's writes never meet the
// previous call's reads -- between a call and the one after next there is
// always the barrier of the call in between.
__device__ __forceinline__ double block_sum_pp(double v, int &par)
{
    __shared__ double sh[2][kBlock / 64];
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[par][w] = v;
    __syncthreads();
    const double r = (sh[par][0] + sh[par][1]) + (sh[par][2] + sh[par][3]);
    par ^= 1;
    return r;
}

// block_sum of acc[k] for every k < nk at once, stored by thread k at
// part[k * kstride]: the same wave_sum per wave and (0 + 1) + (2 + 3) as
// block_sum, so the same bits, with one barrier instead of three per value.
// Once per kernel (its LDS is not re-armed).
template <int NK>
__device__ __forceinline__ void block_sum_store(const double (&acc)[NK], int nk, double *part, long long kstride)
{
    __shared__ double sh[kBlock / 64][NK];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NK; k++) {
        if (k < nk) {
            const double v = wave_sum(acc[k]);
            if (lane == 0) sh[w][k] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < nk) {
        const int k = threadIdx.x;
        part[k * kstride] = (sh[0][k] + sh[1][k]) + (sh[2][k] + sh[3][k]);
    }
}

// Sum of G per-block partials, identical (bit-for-bit) in every block.
__device__ __forceinline__ double sum_partials(const double *part, int G)
{
    double v = 0.0;
    for (int k = threadIdx.x; k < G; k += kBlock) v += part[k];
    return block_sum(v);
}

// UnitMap (kernels.h): does unit u (slots 2u, 2u+1) hold a real row?
__device__ __forceinline__ bool unit_real(const UnitMap &m, long long u)
{
    if (m.kind < 0) return true;
    if (m.kind == 0) return 2 * u < m.n;
    if (m.tbase) {
        if (u < m.tbase) return 2 * u < m.tn;
        u -= m.tbase;
    }
    const int lane = (int)(u & 63);
    const long long q = u >> 6;
    const int th = m.T >> 1;
    int j, k, lo;
    long long tp;
    if (m.kind == 1) {
        // 2D band layout (gg_internal.h Wave2D::slot): q = plane*nbands*T/2 + band*T/2 + t/2
        const long long per_plane = (long long)m.nbands * th;
        const long long kpl = q / per_plane;
        const long long r = q - kpl * per_plane;
        const int band = (int)(r / th);
        tp = r - (long long)band * th;
        j = band * 64 + lane;
        k = (int)kpl;
        lo = m.skew * lane + (m.skew - 1);              // the line's first real step
    } else {
        // 3D tiles: lane a + 8 g(c), t = i + a + c, band = K*NJ + J
        const long long band = q / th;
        tp = q - band * th;
        const int J = (int)(band % m.NJ), K = (int)(band / m.NJ);
        const int a = lane & 7, g = lane >> 3, c = g ^ (g >> 1) ^ (g >> 2);
        j = 8 * J + a;
        k = 8 * K + c;
        lo = a + c;
    }
    if (j >= m.ny || k >= m.nz) return false;
    const long long t0 = 2 * tp;
    return t0 + 1 >= lo && t0 < lo + m.nx;
}

__device__ __forceinline__ double2 ld2(const double *p, long long u)
{
    return reinterpret_cast<const double2 *>(p)[u];
}
// streamed once: non-temporal (does not displace re-used data from the caches)
typedef double dbl2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2_nt(const double *p, long long u)
{
    const dbl2v v = __builtin_nontemporal_load(reinterpret_cast<const dbl2v *>(p) + u);
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2(double *p, long long u, double2 v)
{
    reinterpret_cast<double2 *>(p)[u] = v;
}

// ---- relaxed agent-scope loads/stores for the band hand-off --------------------
constexpr int kSpinLimit = 1 << 20;
// a wait this long (~10 ms of polls) only happens when a workgroup it waits on
// was never dispatched: persistent grids that were sized to be co-resident
// treat it as "not resident" and fall back (gather_first, k_trsv_tile3d)
constexpr int kResidSpin = 1 << 13;
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16 bytes stored write-through (two agent-scope 8-byte stores, sc1): visible
// to other XCDs once drained.  (Not inline asm: the compiler does not guard an
// asm store's data registers against the VALU write hazard that follows it.)
__device__ __forceinline__ void st_sc1_16(double2 *p, double2 v)
{
    unsigned long long *q = reinterpret_cast<unsigned long long *>(p);
    __hip_atomic_store(q, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ============================================================== vector ops
__global__ void k_fill_u64(unsigned long long *p, long long n, unsigned long long v, long long zs = 0)
{
    p = zp(p, zs, blockIdx.y);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_gather(const double *in, const long long *idx, double *out, long long n,
                         unsigned long long *f0, unsigned long long *f1, long long nf)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        long long s = idx[i];
        out[i] = s < 0 ? 0.0 : in[s];
    }
    // (sentinel fills riding on the launch: the x arrays of a flow solve that follows)
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nf;
         i += (long long)gridDim.x * blockDim.x) {
        f0[i] = kSentinel;
        f1[i] = kSentinel;
    }
}

__global__ void k_copy(const double *in, double *out, long long units)
{
    for (long long u = blockIdx.x * (long long)blockDim.x + threadIdx.x; u < units;
         u += (long long)gridDim.x * blockDim.x)
        st2(out, u, ld2(in, u));
}

__global__ __launch_bounds__(kBlock) void k_dot(Gate g, const double *a, const double *b,
                                                double *part, long long units, long long zs = 0)
{
    // units: the dot range (a prefix of the vector space; the sharded solve
    // counts its separator replica on one shard only); zs: batched (blockIdx.y
    // = scenario, every operand per scenario)
    if (gated_z(g, zs, blockIdx.y)) return;
    a = zp(a, zs, blockIdx.y);
    b = zp(b, zs, blockIdx.y);
    part = zp(part, zs, blockIdx.y);
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u0 = blockIdx.x * (long long)kBlock + threadIdx.x; u0 < units; u0 += 4 * stride) {
        double2 x[4], y[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const long long u = u0 + j * stride;
            if (u < units) { x[j] = ld2(a, u); y[j] = ld2(b, u); }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (u0 + j * stride < units) {
                acc += x[j].x * y[j].x;
                acc += x[j].y * y[j].y;
            }
        }
    }
    acc = block_sum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// ---- sharded solve (dd.hip) helpers ---------------------------------------------
// out[r] = in[r] - v_0 x[c_0] - v_1 x[c_1] - ...  in the listed (reference) order:
// the coupling terms a triangular row subtracts before its own triangle's terms
// (separator rows' interior terms, interior rows' separator terms)
// (f0, f1: nf words each set to the sentinel -- the x arrays of the two flow
// solves that follow, whose own fill launches this saves)
__global__ void k_sub_seq(Gate g, int n, const int *rp, const int *ci, const double *v,
                          const double *x, const double *in, double *out, unsigned long long *f0,
                          unsigned long long *f1, int nf)
{
    if (gated(g)) return;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        double acc = in[r];
        for (int k = rp[r]; k < rp[r + 1]; k++) acc -= v[k] * x[ci[k]];
        out[r] = acc;
    }
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < nf; r += gridDim.x * blockDim.x) {
        if (f0) f0[r] = kSentinel;
        if (f1) f1[r] = kSentinel;
    }
}
// all shards of one process: slot s of shard s' buffer (at off + s*cnt) -> every other shard
__global__ void k_allgather_local(ShardPtrs b, int P, long long off, long long cnt)
{
    const long long tot = P * cnt;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot;
         e += (long long)gridDim.x * blockDim.x) {
        const int src = (int)(e / cnt);
        const double v = b.p[src][off + e];
        for (int q = 0; q < P; q++)
            if (q != src) b.p[q][off + e] = v;
    }
}
// k_allgather_local with each shard's slot gathered from its own vector in the
// same launch (kernels.h launch_gather_allgather_local)
__global__ void k_gather_allgather_local(ShardPtrs b, IdxPtrs gi, int P, long long off, long long cnt, FillPtrs fl,
                                         long long nf)
{
    const long long tot = P * cnt;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot;
         e += (long long)gridDim.x * blockDim.x) {
        const int src = (int)(e / cnt);
        const long long s = gi.p[src][e - src * cnt];
        const double v = s < 0 ? 0.0 : b.p[src][s];
        for (int q = 0; q < P; q++) b.p[q][off + e] = v;
    }
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nf;
         i += (long long)gridDim.x * blockDim.x) {
        for (int q = 0; q < P; q++) {
            if (fl.f0[q]) reinterpret_cast<unsigned long long *>(fl.f0[q])[i] = kSentinel;
            if (fl.f1[q]) reinterpret_cast<unsigned long long *>(fl.f1[q])[i] = kSentinel;
        }
    }
}
// GG_DD_IPC all-gather: one process per shard, every shard's exchange area
// mapped into every process (hipIpc; xGMI between GPUs).  Area of rank q:
// [flags: kMaxShards x kIpcXB u64][data: 2 parities x P slots x capd doubles].
// Block b owns chunk b of the cnt exchanged doubles: it stores the chunk of
// this rank's slot (buf + me*cnt) into every peer's data[seq & 1][me], releases
// flag[me][b] = seq at system scope in every peer's area, then waits (acquire,
// time-bounded) until every peer's flag[q][b] in this rank's area reached seq
// and copies those chunks to buf + q*cnt.  Sequence numbers only grow, so the
// flags are never re-armed; two parities suffice because a rank enters
// exchange k+1 only after every peer has entered exchange k, i.e. after it has
// finished copying out exchange k-1.  The area is uncached device memory
// (hipDeviceMallocUncached): remote stores and local polls need no cache
// maintenance beyond the system-scope release / acquire.
// gidx (k_ipc_gather_allgather's form): this rank's slot is gathered first,
// buf[me*cnt + e] = x[gidx[e]] (-1: 0), by the block that sends it
__global__ __launch_bounds__(kBlock) void k_ipc_allgather(IpcPeers pp, int me, int P, double *buf,
                                                          long long cnt, unsigned long long seq,
                                                          long long capd, int *err, const double *x,
                                                          const long long *gidx, unsigned long long *f0,
                                                          unsigned long long *f1, long long nf)
{
    const int nb = gridDim.x, b = blockIdx.x, t = threadIdx.x;
    const long long chunk = (cnt + nb - 1) / nb;
    const long long lo = (long long)b * chunk, hi = lo + chunk < cnt ? lo + chunk : cnt;
    const int par = (int)(seq & 1);
    constexpr long long kFlagWords = (long long)kMaxShards * kIpcXB;
    double *src = buf + (long long)me * cnt;
    if (gidx) {
        for (long long e = lo + t; e < hi; e += kBlock) {
            const long long s = gidx[e];
            src[e] = s < 0 ? 0.0 : x[s];
        }
    }
    for (long long i = b * (long long)kBlock + t; i < nf; i += (long long)nb * kBlock) {
        f0[i] = kSentinel;
        f1[i] = kSentinel;
    }
    for (int q = 0; q < P; q++) {
        if (q == me) continue;
        double *dst = reinterpret_cast<double *>(pp.base[q]) + kFlagWords + ((long long)par * P + me) * capd;
        for (long long e = lo + t; e < hi; e += kBlock) dst[e] = src[e];
    }
    __threadfence_system();
    __syncthreads();
    if (t < P && t != me) {
        unsigned long long *f = reinterpret_cast<unsigned long long *>(pp.base[t]) + (long long)me * kIpcXB + b;
        __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        // wait for peer t's chunk b in this rank's area (bounded: ~30 s of the 100 MHz clock)
        const unsigned long long *w = reinterpret_cast<const unsigned long long *>(pp.base[me]) +
                                      (long long)t * kIpcXB + b;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {
                atomicOr(err, 4);
                break;
            }
        }
    }
    __syncthreads();
    for (int q = 0; q < P; q++) {
        if (q == me) continue;
        const double *rcv = reinterpret_cast<const double *>(pp.base[me]) + kFlagWords + ((long long)par * P + q) * capd;
        double *dst = buf + (long long)q * cnt;
        for (long long e = lo + t; e < hi; e += kBlock) dst[e] = rcv[e];
    }
}

// out[dst[i]] = in[src[i]]
__global__ void k_scatter_idx(const double *in, const long long *src, const long long *dst,
                              double *out, long long n)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[dst[i]] = in[src[i]];
}

// ------------------------------------------------------- split (PG) maps
// MyILUPPfloat::DevPrecond_* elementwise steps (src/preconditioner.cu:1424-1558)
__global__ void k_mul(Gate g, const double *in, const double *s, double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] * s[i];
}
// the user-preconditioner boundary (fp32 arrays, src/preconditioner.h:34-84)
// order-independent fingerprint: sum of w_k * (2k + 1) over 32-bit words, mod 2^64
__global__ __launch_bounds__(kBlock) void k_fingerprint(const unsigned *p, long long nw, unsigned long long *out)
{
    unsigned long long acc = 0;
    for (long long k = blockIdx.x * (long long)kBlock + threadIdx.x; k < nw; k += (long long)gridDim.x * kBlock)
        acc += (unsigned long long)p[k] * (unsigned long long)(2 * k + 1);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);      // integer adds: any order, same sum
}

__global__ void k_f64_to_f32(Gate g, const double *in, float *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)in[i];
}
__global__ void k_f32_to_f64(Gate g, const float *in, double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (double)in[i];
}
__global__ void k_div(Gate g, const double *in, const double *s, double *out, int n)
{
    if (gated(g)) return;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] / s[i];
}

// ================================================================= SpMV
// CSR-stream: a block owns <=256 consecutive rows holding <=kSpmvCap nnz.
// Products v*x[col] are formed with coalesced loads into LDS, then each row is
// summed serially in CSR order (computeSpMV order, src/SpMV_compute.cpp:19-36).
// YDIV: y[r] = (the row's result) / ydiv[r] -- the split engine's row gather
// and D_l scaling (gather_divsrc, src/preconditioner.cu:1592-1626) folded into
// the SpMV of the row-permuted matrix: the same division of the same value.
// XA: x read with agent-scope (sc1) loads -- values handed over inside the
// launch (k_dd_spmv_x's separator rows)
template <bool XA>
__device__ __forceinline__ double ld_x(const double *p)
{
    if constexpr (XA) return __longlong_as_double((long long)ld_agent(reinterpret_cast<const unsigned long long *>(p)));
    else return *p;
}
template <bool RESID, bool YDIV, bool XA = false>
__device__ __forceinline__ void spmv_stream_block(int bid, const int *blk, const int *rp, const int *ci,
                                                  const double *v, const double *x, const double *b, double *y,
                                                  const double *ydiv)
{
    constexpr int U = kSpmvCap / kBlock;        // products per thread
    __shared__ double prod[kSpmvCap];
    __shared__ int srp[kBlock + 1];
    const int tid = threadIdx.x;
    const int r0 = blk[bid], r1 = blk[bid + 1];
    const int nr = r1 - r0;                     // <= kBlock rows
    // the block's nr + 1 row pointers (nr <= kBlock: the last one by thread 0)
    if (tid < nr) srp[tid] = rp[r0 + tid];
    if (tid == 0) srp[nr] = rp[r1];
    __syncthreads();
    const int e0 = srp[0], e1 = srp[nr];
    const int cnt = e1 - e0;
    if (cnt > kSpmvCap) {   // one long row: strided partial sums + tree
        double acc = 0.0;
        for (int e = e0 + tid; e < e1; e += kBlock) acc += v[e] * ld_x<XA>(x + ci[e]);
        acc = block_sum(acc);
        if (tid == 0) {
            const double o = RESID ? (-1.0 * acc + 1.0 * b[r0]) : acc;
            y[r0] = YDIV ? o / ydiv[r0] : o;
        }
        return;
    }
    // entries in aligned pairs (8-B index and 16-B value loads) from the even
    // entry at or below e0; all index/value loads first, then all gathers
    constexpr int U2 = U / 2 + 1;               // pairs per thread (the alignment adds one)
    const int ea = e0 & ~1;
    const int npair = (e1 - ea + 1) >> 1;
    int2 c[U2];
    double2 vv[U2], xv[U2];
#pragma unroll
    for (int u = 0; u < U2; u++) {
        const int p = tid + u * kBlock;
        if (p < npair) {
            c[u] = reinterpret_cast<const int2 *>(ci + ea)[p];
            vv[u] = reinterpret_cast<const double2 *>(v + ea)[p];
        }
    }
#pragma unroll
    for (int u = 0; u < U2; u++) {
        const int p = tid + u * kBlock;
        const int e = ea + 2 * p;
        if (p < npair) {
            if (e >= e0) xv[u].x = ld_x<XA>(x + c[u].x);
            if (e + 1 < e1) xv[u].y = ld_x<XA>(x + c[u].y);
        }
    }
#pragma unroll
    for (int u = 0; u < U2; u++) {
        const int p = tid + u * kBlock;
        const int e = ea + 2 * p;
        if (p < npair) {
            if (e >= e0) prod[e - e0] = vv[u].x * xv[u].x;
            if (e + 1 < e1) prod[e + 1 - e0] = vv[u].y * xv[u].y;
        }
    }
    __syncthreads();
    if (tid < nr) {
        // the row's products in CSR order; eight LDS reads in flight per
        // group (a read-then-add loop waits an LDS round trip per term)
        double acc = 0.0;
        const int a = srp[tid] - e0, z = srp[tid + 1] - e0;
        int e = a;
        for (; e + 8 <= z; e += 8) {
            double t[8];
#pragma unroll
            for (int q = 0; q < 8; q++) t[q] = prod[e + q];
#pragma unroll
            for (int q = 0; q < 8; q++) acc += t[q];
        }
        for (; e < z; e++) acc += prod[e];
        const int r = r0 + tid;
        const double o = RESID ? (-1.0 * acc + 1.0 * b[r]) : acc;
        y[r] = YDIV ? o / ydiv[r] : o;
    }
}
template <bool RESID, bool YDIV = false>
__global__ __launch_bounds__(kBlock) void k_spmv_stream(Gate g, const int *blk, const int *rp,
                                                        const int *ci, const double *v,
                                                        const double *x, const double *b,
                                                        double *y, const double *ydiv)
{
    if (gated(g)) return;
    spmv_stream_block<RESID, YDIV>(blockIdx.x, blk, rp, ci, v, x, b, y, ydiv);
}

// Sliced ELL: one wave per 64-row slice, lane = row; the slice's entries are
// read k-major (each load instruction is one coalesced 256-B / 512-B line per
// wave), up to 8 index/value pairs in flight before their gathers; each row is
// summed serially in CSR order from 0.0, skipping the padding (col -1): the
// same operations as k_spmv_stream (computeSpMV order).
// GG_SPMV_XCD: blocks b, b+8, ... (one XCD under round-robin dispatch, for
// speed only) take consecutive slices, so the x lines that neighbouring slices
// share are fetched into one L2 (the 3D tile layout's line and plane
// neighbours are 64 and 13,824 rows away)
#ifndef GG_SPMV_XCD
#define GG_SPMV_XCD 1
#endif
__device__ __forceinline__ int xcd_block()
{
    if (!GG_SPMV_XCD) return blockIdx.x;
    const int nb = gridDim.x, q = nb >> 3, rem = nb & 7, x = blockIdx.x & 7;
    return x * q + (x < rem ? x : rem) + (blockIdx.x >> 3);
}

// XDIV: x[c] = RN(x[c] / xdiv[c]) formed per gathered term -- the split
// engine's D_r^-1 pass (k_div) folded into the gathers, the same division
template <bool RESID, bool YDIV, bool XDIV, bool XA = false>
__device__ __forceinline__ void spmv_sell_slice(int s, int n, const int *sptr, const int *__restrict__ ci,
                                                const double *__restrict__ v, const double *x,
                                                const double *__restrict__ b, double *__restrict__ y,
                                                const double *__restrict__ ydiv, const double *__restrict__ xdiv)
{
    const int lane = threadIdx.x & 63;
    const int off = sptr[s], w = (sptr[s + 1] - off) >> 6;
    const int *cp = ci + off + lane;
    const double *vp = v + off + lane;
    double acc = 0.0;
    for (int k0 = 0; k0 < w; k0 += 8) {
        int c[8];
        double a[8], xv[8];
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k0 + k < w) {
                c[k] = __builtin_nontemporal_load(cp + (k0 + k) * 64);
                a[k] = __builtin_nontemporal_load(vp + (k0 + k) * 64);
            }
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k0 + k < w && c[k] >= 0) xv[k] = ld_x<XA>(x + c[k]);
        if constexpr (XDIV) {
            double dv[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (k0 + k < w && c[k] >= 0) dv[k] = xdiv[c[k]];
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (k0 + k < w && c[k] >= 0) xv[k] = xv[k] / dv[k];
        }
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k0 + k < w && c[k] >= 0) acc += a[k] * xv[k];
    }
    const int r = s * 64 + lane;
    if (r < n) {
        const double o = RESID ? (-1.0 * acc + 1.0 * b[r]) : acc;
        y[r] = YDIV ? o / ydiv[r] : o;
    }
}
template <bool RESID, bool YDIV = false, bool XDIV = false>
__global__ __launch_bounds__(kBlock) void k_spmv_sell(Gate g, int n, int nslice, const int *sptr,
                                                      const int *__restrict__ ci,
                                                      const double *__restrict__ v,
                                                      const double *__restrict__ x,
                                                      const double *__restrict__ b,
                                                      double *__restrict__ y,
                                                      const double *__restrict__ ydiv,
                                                      const double *__restrict__ xdiv,
                                                      unsigned long long *fill = nullptr, int nfill = 0)
{
    // (XDIV, fill: the next flow solve's x set to the sentinel, rows < nfill --
    // the k_fill_gated launch that solve would make)
    if (gated(g)) return;
    const int s = xcd_block() * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (s >= nslice) return;
    if constexpr (XDIV) {
        const int r = s * 64 + (int)(threadIdx.x & 63);
        if (fill && r < nfill) fill[r] = kSentinel;
    }
    spmv_sell_slice<RESID, YDIV, XDIV>(s, n, sptr, ci, v, x, b, y, ydiv, xdiv);
}

// Column-panel SpMV, one launch per panel p (DevCsr::panel): a block owns a
// run of <= 256 of the panel's row segments (a row's terms whose columns fall
// in the panel, in CSR order) holding <= kSpmvCap entries (pblk, host-made),
// and works like k_spmv_stream on it -- entries loaded coalesced, x gathered
// (from the panel's slice, which the XCD's L2 keeps), products into LDS, then
// each segment's products summed by its thread in order, continuing the row's
// running sum kept in y (0.0 at the row's first segment, seg_row = ~row).
// Every row is thus summed exactly as computeSpMV sums it.  Empty rows get 0
// in pass 0.  GG_PANEL_NT=1: the panel's entries and segment tables streamed
// non-temporally, so that they do not push the x slice out of the L2.
// (C3 stand-in, one box, profiles/r06/c3_panel_ab.txt: 648 -> 640 us at 4 MiB
// panels, 651 -> 626 us at 6 MiB)
#ifndef GG_PANEL_NT
#define GG_PANEL_NT 1
#endif
template <class T>
__device__ __forceinline__ T pan_ld(const T *p)
{
    if constexpr (GG_PANEL_NT) return __builtin_nontemporal_load(p);
    else return *p;
}
// one sub-block (<= 256 segments, <= kSpmvCap entries) of the panel layout;
// YA: the running sums read with agent-scope loads (k_spmv_rtile: the row's
// previous segment was stored by this block, by another of its threads)
template <bool YA>
__device__ __forceinline__ void panel_subblock(int sb, const int *__restrict__ pblk, const int *__restrict__ seg_row,
                                               const int *__restrict__ seg_ptr, const int *__restrict__ pci,
                                               const double *__restrict__ pv, const double *__restrict__ x, double *y)
{
    constexpr int U = kSpmvCap / kBlock;        // entries per thread
    __shared__ double prod[kSpmvCap];
    __shared__ int sp[kBlock + 1];
    const int tid = threadIdx.x;
    const int s0 = pblk[sb], s1 = pblk[sb + 1];
    const int ns = s1 - s0;                     // <= kBlock segments
    if (tid < ns) sp[tid] = pan_ld(seg_ptr + s0 + tid);
    if (tid == 0) sp[ns] = pan_ld(seg_ptr + s1);
    int rr = 0;
    double acc = 0.0;
    if (tid < ns) {
        rr = pan_ld(seg_row + s0 + tid);
        if (rr >= 0) acc = ld_x<YA>(y + rr);    // the row's running sum so far
    }
    __syncthreads();
    const int e0 = sp[0], cnt = sp[ns] - e0;
    int c[U];
    double a[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int q = tid + u * kBlock;
        if (q < cnt) {
            c[u] = pan_ld(pci + e0 + q);
            a[u] = pan_ld(pv + e0 + q);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
        if (tid + u * kBlock < cnt) xv[u] = x[c[u]];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int q = tid + u * kBlock;
        if (q < cnt) prod[q] = a[u] * xv[u];
    }
    __syncthreads();
    if (tid < ns) {
        const int lo = sp[tid] - e0, hi = sp[tid + 1] - e0;
        int e = lo;
        for (; e + 8 <= hi; e += 8) {
            double t[8];
#pragma unroll
            for (int q = 0; q < 8; q++) t[q] = prod[e + q];
#pragma unroll
            for (int q = 0; q < 8; q++) acc += t[q];
        }
        for (; e < hi; e++) acc += prod[e];
        y[rr < 0 ? ~rr : rr] = acc;
    }
}
__global__ __launch_bounds__(kBlock) void k_spmv_panel(Gate g, const int *__restrict__ pblk,
                                                       const int *__restrict__ seg_row,
                                                       const int *__restrict__ seg_ptr,
                                                       const int *__restrict__ pci, const double *__restrict__ pv,
                                                       const double *__restrict__ x, double *__restrict__ y,
                                                       const int *__restrict__ zero_rows, int nzero)
{
    if (gated(g)) return;
    if (nzero)
        for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nzero; i += (long long)gridDim.x * kBlock)
            y[zero_rows[i]] = 0.0;
    panel_subblock<false>(blockIdx.x, pblk, seg_row, seg_ptr, pci, pv, x, y);
}
// Row tiles (DevCsr::rtile): ONE launch, block b walking its sub-blocks
// rt_sub[b] .. rt_sub[b+1]-1 in order -- its rows' segments panel by panel, so
// a row's terms are added in column order (the CSR order: the same bits), its
// running sum in y only ever touched by this block.  Between sub-blocks the
// y stores are drained and the block synchronises; the next sub-block reads y
// with agent-scope loads (past this CU's L1).
__global__ __launch_bounds__(kBlock) void k_spmv_rtile(Gate g, const int *__restrict__ rt_sub,
                                                       const int *__restrict__ pblk,
                                                       const int *__restrict__ seg_row,
                                                       const int *__restrict__ seg_ptr,
                                                       const int *__restrict__ pci, const double *__restrict__ pv,
                                                       const double *__restrict__ x, double *y,
                                                       const int *__restrict__ zero_rows, int nzero)
{
    if (gated(g)) return;
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < nzero; i += (long long)gridDim.x * kBlock)
        y[zero_rows[i]] = 0.0;
    const int b0 = rt_sub[blockIdx.x], b1 = rt_sub[blockIdx.x + 1];
    for (int sb = b0; sb < b1; sb++) {
        panel_subblock<true>(sb, pblk, seg_row, seg_ptr, pci, pv, x, y);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this sub-block's y stores done
        __syncthreads();
    }
}

// The sharded SpMV with its interface exchange in ONE launch (dd.hip
// spmv_rows; GG_DD_IPC / GG_DD_LOOPBACK, one shard per process): north_star's
// overlap of the halo exchange with the interior rows, without a second
// stream and its cross-stream event pair.
//   blocks [0, nbx): the exchange -- k_ipc_allgather's protocol with this
//     rank's slot gathered in the launch (IPC), or the loopback all-gather over
//     this shard's own buffer (LOOPBACK, timing only: k_gather_allgather_local's
//     stores); every halo value is stored write-through (sc1), each storing wave
//     drains its stores, and after a barrier one lane adds 1 to *arrived
//   blocks [nbx, nbx + nbi): the interior rows (they read no halo value)
//   blocks after: the separator rows; one lane waits for *arrived >= target,
//     the block passes a barrier, then reads x with agent-scope loads only
//     (MI355X_MICROARCH.md's hand-off table, row 1)
// A block waits only on blocks of lower index (dispatched first).  Each row's
// operations are k_spmv_sell's / k_spmv_stream's: the same bits as the
// unfused launches.
template <bool RESID>
__global__ __launch_bounds__(kBlock) void k_dd_spmv_x(Gate g, DdSpmvX a)
{
    const int bid = blockIdx.x, t = threadIdx.x;
    if (bid < a.nbx) {
        const int nb = a.nbx;
        if (a.loop) {
            // loopback: slot q of the halo = this shard's own interface values
            const long long tot = (long long)a.P * a.cnt;
            for (long long e = bid * (long long)kBlock + t; e < tot; e += (long long)nb * kBlock) {
                const long long sq = a.gidx[e % a.cnt];
                const double v = sq < 0 ? 0.0 : a.x[sq];
                st_agent(reinterpret_cast<unsigned long long *>(a.halo + e), (unsigned long long)__double_as_longlong(v));
            }
        } else {
            const long long chunk = (a.cnt + nb - 1) / nb;
            const long long lo = (long long)bid * chunk, hi = lo + chunk < a.cnt ? lo + chunk : a.cnt;
            const int par = (int)(a.seq & 1);
            constexpr long long kFlagWords = (long long)kMaxShards * kIpcXB;
            double *src = a.halo + (long long)a.me * a.cnt;
            for (long long e = lo + t; e < hi; e += kBlock) {
                const long long sq = a.gidx[e];
                const double v = sq < 0 ? 0.0 : a.x[sq];
                st_agent(reinterpret_cast<unsigned long long *>(src + e), (unsigned long long)__double_as_longlong(v));
                for (int q = 0; q < a.P; q++) {
                    if (q == a.me) continue;
                    double *dst = reinterpret_cast<double *>(a.pp.base[q]) + kFlagWords + ((long long)par * a.P + a.me) * a.capd;
                    dst[e] = v;
                }
            }
            __threadfence_system();
            __syncthreads();
            if (t < a.P && t != a.me) {
                unsigned long long *f = reinterpret_cast<unsigned long long *>(a.pp.base[t]) + (long long)a.me * kIpcXB + bid;
                __hip_atomic_store(f, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned long long *w = reinterpret_cast<const unsigned long long *>(a.pp.base[a.me]) +
                                              (long long)t * kIpcXB + bid;
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {
                        atomicOr(a.err, 4);
                        break;
                    }
                }
            }
            __syncthreads();
            for (int q = 0; q < a.P; q++) {
                if (q == a.me) continue;
                const double *rcv =
                    reinterpret_cast<const double *>(a.pp.base[a.me]) + kFlagWords + ((long long)par * a.P + q) * a.capd;
                double *dst = a.halo + (long long)q * a.cnt;
                for (long long e = lo + t; e < hi; e += kBlock)
                    st_agent(reinterpret_cast<unsigned long long *>(dst + e),
                             (unsigned long long)__double_as_longlong(rcv[e]));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every wave's halo stores drained
        __syncthreads();
        if (t == 0) __hip_atomic_fetch_add(a.arrived, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (gated(g)) return;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    if (bid < a.nbx + a.nbi) {
        const int q = bid - a.nbx;
        if (a.i_sell) {
            const int sl = q * (kBlock / 64) + wv;
            if (sl < a.i_nb) spmv_sell_slice<RESID, false, false>(sl, a.i_n, a.i_ptr, a.i_ci, a.i_v, a.x, a.b, a.y,
                                                                  nullptr, nullptr);
        } else {
            spmv_stream_block<RESID, false>(q, a.i_ptr, a.i_rp, a.i_ci, a.i_v, a.x, a.b, a.y, nullptr);
        }
        return;
    }
    if (t == 0) {
        int spins = 0;
        while (ld_agent(a.arrived) < a.target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kSpinLimit * 16) {
                atomicOr(a.err, 4);
                break;
            }
        }
    }
    __syncthreads();
    const int q = bid - a.nbx - a.nbi;
    const double *bs = RESID ? a.b + a.S0 : nullptr;
    double *ys = a.y + a.S0;
    if (a.s_sell) {
        const int sl = q * (kBlock / 64) + wv;
        if (sl < a.s_nb) spmv_sell_slice<RESID, false, false, true>(sl, a.s_n, a.s_ptr, a.s_ci, a.s_v, a.x, bs, ys,
                                                                    nullptr, nullptr);
    } else {
        spmv_stream_block<RESID, false, true>(q, a.s_ptr, a.s_rp, a.s_ci, a.s_v, a.x, bs, ys, nullptr);
    }
}

// Batched SpMV (the many-RHS solve): y_sc = A x_sc (RESID: b_sc - A x_sc) for
// up to NS scenarios per launch (scenario sc's vectors sc * zs bytes after
// scenario 0's), A's sliced-ELL entries read ONCE per wave for all of them.
// Every row of every scenario is summed exactly as k_spmv_sell sums it (entry
// order from 0.0, no contraction): the same bits.  A scenario whose gate is
// closed (converged) is skipped.
template <bool RESID, int NS>
__global__ __launch_bounds__(kBlock) void k_spmv_sell_b(Gate g, long long zs, int nsc, int n, int nslice,
                                                        const int *sptr, const int *__restrict__ ci,
                                                        const double *__restrict__ v, const double *x,
                                                        const double *b, double *y)
{
    const int s = xcd_block() * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (s >= nslice) return;
    bool act[NS];
    bool any = false;
#pragma unroll
    for (int q = 0; q < NS; q++) {
        act[q] = q < nsc && !gated_z(g, zs, q);
        any |= act[q];
    }
    if (!any) return;
    const int lane = threadIdx.x & 63;
    const int off = sptr[s], w = (sptr[s + 1] - off) >> 6;
    const int *cp = ci + off + lane;
    const double *vp = v + off + lane;
    double acc[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) acc[q] = 0.0;
    for (int k0 = 0; k0 < w; k0 += 8) {
        int c[8];
        double a[8];
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k0 + k < w) {
                c[k] = __builtin_nontemporal_load(cp + (k0 + k) * 64);
                a[k] = __builtin_nontemporal_load(vp + (k0 + k) * 64);
            }
#pragma unroll
        for (int q = 0; q < NS; q++) {
            if (!act[q]) continue;
            const double *xq = zp(x, zs, q);
            double xv[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (k0 + k < w && c[k] >= 0) xv[k] = xq[c[k]];
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (k0 + k < w && c[k] >= 0) acc[q] += a[k] * xv[k];
        }
    }
    const int r = s * 64 + lane;
    if (r < n) {
#pragma unroll
        for (int q = 0; q < NS; q++) {
            if (!act[q]) continue;
            zp(y, zs, q)[r] = RESID ? (-1.0 * acc[q] + 1.0 * zp(b, zs, q)[r]) : acc[q];
        }
    }
}

// ======================================================= triangular solves
// Level-scheduled row solve (one launch per dependency level):
//   x[r] = (b[r] - sum_k off[k] * x[col[k]]) / d[r]   in canonical order
// y (optional): RN(1/d) -- x = RN(acc * y), WD_MUL's row (a bordered grid's
// tail under gg_set_division(GG_DIV_RCP), DevTri::tail).  fm: GG_DIV_FMA's row
// (a bordered grid's tail, DevTri::tail_fma): acc = RN(b * y) (b when y is null),
// then acc = fma(-v, x, acc) over the terms as stored -- pre-scaled by y and in
// the fused order (nearest first) -- and no division
__global__ __launch_bounds__(kBlock) void k_trsv_level(Gate g, int cnt, const int *rows,
                                                       const int *rp, const int *ci,
                                                       const double *v, const double *d,
                                                       const double *b, double *x, const double *y, int fm)
{
    if (gated(g)) return;
    int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= cnt) return;
    int r = rows[t];
    if (fm) {                       // GG_DIV_FMA's rows (the terms pre-scaled and in fused order)
        double acc = y ? b[r] * y[r] : b[r];
        for (int k = rp[r]; k < rp[r + 1]; k++) acc = __builtin_fma(-v[k], x[ci[k]], acc);
        x[r] = acc;
        return;
    }
    double acc = b[r];
    for (int k = rp[r]; k < rp[r + 1]; k++) acc = acc - v[k] * x[ci[k]];
    x[r] = y ? acc * y[r] : acc / d[r];
}

// Sync-free (dataflow) form of the same solve, one launch per triangle: x is
// pre-filled with the sentinel and a row's value is its own ready flag.  Rows
// are taken in level order (lev_rows), a wave 64 consecutive ones, the
// co-resident grid striding over the list; a lane loads all its sources with
// agent-scope loads, and if none is the sentinel finishes the row with the
// same operations as k_trsv_level (canonical order, then / d[r]) and stores it
// with an agent-scope store; otherwise it retries inside a wave-uniform loop
// (sources of one wave's rows may be other lanes of the wave).  The smallest
// unfinished row in level order always has its sources done, so the grid
// drains; spins are bounded (err bit 0).
__global__ void k_fill_gated(Gate g, unsigned long long *p, long long n, unsigned long long v)
{
    if (gated(g)) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}

// long rows: issue the next round's loads before this round's serial sum (1;
// 92 VGPRs, 5 waves per SIMD) or after it (0; 62 VGPRs, 8 waves per SIMD)
#ifndef GG_FLOW_PREFETCH
#define GG_FLOW_PREFETCH 1
#endif
// one long row (more than kFlowLong terms), the whole wave: each round 256 of
// its terms (4 per lane) are loaded and polled together, their products v*x
// formed in parallel, then lane 0 subtracts them from acc one by one in
// canonical order -- the reference's serial arithmetic
__device__ __forceinline__ void flow_long_row(int r, const int *__restrict__ rp, const int *__restrict__ ci,
                                              const double *__restrict__ v, const double *__restrict__ d,
                                              const double *__restrict__ b, unsigned long long *xu, int *err,
                                              const double *__restrict__ y, double *wprod, int lane)
{
    const int k0 = rp[r], k1 = rp[r + 1];
    double acc = b[r];
    int spins = 0;
    // round kc's columns, coefficients and x polls; the next round's
    // are issued before this round's serial sum (their latency hidden)
    int c[4];
    double vv[4];
    unsigned long long u[4];
    auto fetch = [&](int kc, int *cc, double *vc, unsigned long long *uc) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int k = kc + q * 64 + lane;
            cc[q] = k < k1 ? ci[k] : -1;
            vc[q] = k < k1 ? v[k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) uc[q] = cc[q] >= 0 ? ld_agent(xu + cc[q]) : 0ull;
    };
    fetch(k0, c, vv, u);
    for (int kc = k0; kc < k1; kc += 256) {
        if (!GG_FLOW_PREFETCH && kc > k0) fetch(kc, c, vv, u);
        while (true) {
            bool miss = false;
#pragma unroll
            for (int q = 0; q < 4; q++) miss |= c[q] >= 0 && u[q] == kSentinel;
            if (!__any(miss)) break;
            __builtin_amdgcn_s_sleep(2);
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(err, 1);
                break;
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (c[q] >= 0 && u[q] == kSentinel) u[q] = ld_agent(xu + c[q]);
        }
        double pq[4];
#pragma unroll
        for (int q = 0; q < 4; q++) pq[q] = vv[q] * __longlong_as_double((long long)u[q]);
        if (GG_FLOW_PREFETCH && kc + 256 < k1) fetch(kc + 256, c, vv, u);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            wprod[lane] = pq[q];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const int cnt = k1 - (kc + q * 64);
            if (lane == 0) {
                // the 64 products in canonical order, read 8 at a time one
                // chunk ahead (a read-then-subtract loop waits an LDS round
                // trip per term)
                const double2 *wp2 = reinterpret_cast<const double2 *>(wprod);
                double2 cur[4], nxt[4];
#pragma unroll
                for (int e = 0; e < 4; e++) cur[e] = wp2[e];
#pragma unroll
                for (int c8 = 0; c8 < 8; c8++) {
                    if (c8 + 1 < 8) {
#pragma unroll
                        for (int e = 0; e < 4; e++) nxt[e] = wp2[(c8 + 1) * 4 + e];
                    }
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const int j = c8 * 8 + 2 * e;
                        if (j < cnt) acc = acc - cur[e].x;
                        if (j + 1 < cnt) acc = acc - cur[e].y;
                    }
#pragma unroll
                    for (int e = 0; e < 4; e++) cur[e] = nxt[e];
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
    }
    if (lane == 0) st_agent(xu + r, (unsigned long long)__double_as_longlong(y ? acc * y[r] : acc / d[r]));
}

// ELL: short rows read their terms from the sliced copy (DevTri::eci / ev,
// task {.z, .w}) instead of rp / ci / v: no rp -> ci -> poll chain of dependent
// loads, one coalesced load per term index; the operations are the same (pgr:
// L 84.0 -> 62.8, U 103.0 -> 68.9 us, profiles/r04/r04y_pgr_e*.json; a software-
// pipelined task loop -- the next task's loads behind this one's polls --
// measured 67.1 / 73.1 us, r04z_pgr_e1.json, not kept).
// s_sleep between a wave's poll rounds while a lane waits on a source
#ifndef GG_FLOW_SLEEP
#define GG_FLOW_SLEEP 4
#endif
// how a short row's lane polls its sources (x pre-filled with the sentinel,
// each slot written once per launch: a value other than the sentinel is final)
//   0: every round re-loads the chunk's sources from the first unconsumed one
//   1: a source seen ready is kept in a register; only sentinel ones re-polled
//   2: as 1, and each source's first probe is a PLAIN load (L1/L2-served: a
//      stale copy can only show the sentinel, which falls back to the agent poll)
#ifndef GG_FLOW_POLL
#define GG_FLOW_POLL 1
#endif
__device__ __forceinline__ unsigned long long ld_flow_first(const unsigned long long *p)
{
    if constexpr (GG_FLOW_POLL == 2) return *reinterpret_cast<const volatile unsigned long long *>(p);
    else return ld_agent(p);
}
template <bool ELL>
__global__ __launch_bounds__(kBlock) void k_trsv_flow(Gate g, int ntask, const int4 *__restrict__ tasks,
                                                      const int *__restrict__ rows,
                                                      const int *__restrict__ rp, const int *__restrict__ ci,
                                                      const double *__restrict__ v,
                                                      const double *__restrict__ d,
                                                      const double *__restrict__ b, double *x, int *err,
                                                      const double *__restrict__ y, int fm,
                                                      const int *__restrict__ eci, const double *__restrict__ ev)
{
    if (gated(g)) return;
    __shared__ double prod[kBlock];            // a long row's products, one 64-slot area per wave
    const int lane = threadIdx.x & 63;
    double *wprod = prod + (threadIdx.x & ~63);
    const long long wid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long nw = (gridDim.x * (long long)blockDim.x) >> 6;
    unsigned long long *xu = reinterpret_cast<unsigned long long *>(x);
    for (long long t = wid; t < ntask; t += nw) {
        const int4 tk = tasks[t];
        if (tk.y < 0) {
            // (fm triangles are built without long rows: build_tri_bordered)
            flow_long_row(rows[tk.x], rp, ci, v, d, b, xu, err, y, wprod, lane);
            continue;
        }
        if constexpr (ELL) {
            // up to 64 short rows, one per lane, terms from the sliced copy four
            // at a time (cc / vv: terms kb .. kb+3; column -1 past the row's end)
            const int r = lane < tk.y ? rows[tk.x + lane] : -1;
            const int w = tk.w;
            const long long eb = (long long)tk.z * 64 + lane;
            int cc[4];
            double vv[4];
            auto chunk = [&](int kb) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    cc[j] = kb + j < w ? eci[eb + (long long)(kb + j) * 64] : -1;
                    vv[j] = kb + j < w ? ev[eb + (long long)(kb + j) * 64] : 0.0;
                }
            };
            chunk(0);
            bool pending = r >= 0;
            // y: the reciprocal (WD_MUL's row; fm: b's pre-scale, GG_DIV_FMA's row)
            double acc = pending ? ((fm && y) ? b[r] * y[r] : b[r]) : 0.0;
            const double dr = pending ? (y ? y[r] : d[r]) : 1.0;
            int kb = 0, k = 0;                  // chunk base, terms consumed
            int spins = 0;
            unsigned long long u[4];            // GG_FLOW_POLL >= 1: the chunk's sources as last seen
            bool fresh = true;                  // the chunk not probed yet
            while (__any(pending)) {
                if (pending) {
                    // consume the sources in canonical order as far as they
                    // are ready (a source once seen stays final)
                    while (true) {
                        if constexpr (GG_FLOW_POLL == 0) {
#pragma unroll
                            for (int j = 0; j < 4; j++) u[j] = (kb + j >= k && cc[j] >= 0) ? ld_agent(xu + cc[j]) : 0ull;
                        } else if (fresh) {
#pragma unroll
                            for (int j = 0; j < 4; j++) u[j] = (kb + j >= k && cc[j] >= 0) ? ld_flow_first(xu + cc[j]) : 0ull;
                            fresh = false;
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; j++)
                                if (kb + j >= k && cc[j] >= 0 && u[j] == kSentinel) u[j] = ld_agent(xu + cc[j]);
                        }
                        bool stop = false;
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            if (!stop && kb + j >= k && cc[j] >= 0) {
                                if (u[j] == kSentinel) {
                                    stop = true;
                                } else {
                                    const double xj = __longlong_as_double((long long)u[j]);
                                    acc = fm ? __builtin_fma(-vv[j], xj, acc) : acc - vv[j] * xj;
                                    k++;
                                }
                            }
                        }
                        if (stop) break;
                        if (cc[3] < 0 || kb + 4 >= w) {
                            st_agent(xu + r, (unsigned long long)__double_as_longlong(fm ? acc : y ? acc * dr : acc / dr));
                            pending = false;
                            break;
                        }
                        kb += 4;
                        chunk(kb);
                        fresh = true;
                    }
                }
                if (__any(pending)) {
                    __builtin_amdgcn_s_sleep(GG_FLOW_SLEEP);
                    if (++spins > kSpinLimit) {
                        if (pending) atomicOr(err, 1);
                        pending = false;
                    }
                }
            }
            continue;
        }
        // up to 64 short rows, one per lane
        const int r = lane < tk.y ? rows[tk.x + lane] : -1;
        bool pending = r >= 0;
        int k = pending ? rp[r] : 0;
        const int k1 = pending ? rp[r + 1] : 0;
        // y: the reciprocal (WD_MUL's row; fm: b's pre-scale, GG_DIV_FMA's row)
        double acc = pending ? ((fm && y) ? b[r] * y[r] : b[r]) : 0.0;
        const double dr = pending ? (y ? y[r] : d[r]) : 1.0;
        int spins = 0;
        unsigned long long u[4];                // GG_FLOW_POLL >= 1: sources k .. k+3 as last seen
        int ub = -1;                            // the k they were loaded for (-1: none)
        while (__any(pending)) {
            if (pending) {
                // consume the sources in canonical order as far as they are
                // ready (one outstanding poll per waiting lane); a source
                // once seen stays final, so acc is built incrementally
                bool stop = false;
                while (!stop && k < k1) {
                    // up to 4 polls in flight
                    if (GG_FLOW_POLL == 0) {
#pragma unroll
                        for (int j = 0; j < 4; j++) u[j] = k + j < k1 ? ld_agent(xu + ci[k + j]) : 0ull;
                    } else if (ub != k) {
#pragma unroll
                        for (int j = 0; j < 4; j++) u[j] = k + j < k1 ? ld_flow_first(xu + ci[k + j]) : 0ull;
                        ub = k;
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (k + j < k1 && u[j] == kSentinel) u[j] = ld_agent(xu + ci[k + j]);
                    }
                    const int k0 = k;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if (stop || k >= k1) break;
                        if (u[j] == kSentinel) { stop = true; break; }
                        const double xj = __longlong_as_double((long long)u[j]);
                        acc = fm ? __builtin_fma(-v[k], xj, acc) : acc - v[k] * xj;
                        k++;
                    }
                    if (stop && k != k0) {
                        // sources k0 .. k-1 consumed: shift the window to start at k
                        const int sh = k - k0;          // 1..3 (selects: no indexed registers)
                        const unsigned long long t1 = u[1], t2 = u[2], t3 = u[3];
                        u[0] = sh == 1 ? t1 : sh == 2 ? t2 : t3;
                        u[1] = sh == 1 ? t2 : sh == 2 ? t3 : kSentinel;
                        u[2] = sh == 1 ? t3 : kSentinel;
                        u[3] = kSentinel;
                        ub = k;
                    }
                }
                if (k == k1) {
                    st_agent(xu + r, (unsigned long long)__double_as_longlong(fm ? acc : y ? acc * dr : acc / dr));
                    pending = false;
                }
            }
            if (__any(pending)) {
                __builtin_amdgcn_s_sleep(GG_FLOW_SLEEP);
                if (++spins > kSpinLimit) {
                    if (pending) atomicOr(err, 1);
                    pending = false;
                }
            }
        }
    }
}

// Bordered grid, forward solve (DevTri::tail): a grid row's tail terms lead
// its canonical order, so b[row] - (its tail terms, in order) is exactly the
// head of the row's own sum; it is formed here, in place, once the tail is
// solved, and the wavefront continues the sum from it.  One row per thread.
__global__ void k_border_sub(Gate g, int nrow, const long long *__restrict__ slot, const int *__restrict__ rp,
                             const int *__restrict__ ci, const double *__restrict__ v,
                             const double *__restrict__ x, double *b, int fm)
{
    if (gated(g)) return;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrow) return;
    const long long p = slot[q];
    double acc = b[p];
    // fm: GG_DIV_FMA's unit L rows (the tail terms lead the fused row too)
    for (int k = rp[q]; k < rp[q + 1]; k++) acc = fm ? __builtin_fma(-v[k], x[ci[k]], acc) : acc - v[k] * x[ci[k]];
    b[p] = acc;
}

// A small bordered-grid tail (DevTri::tail_small) in ONE workgroup: its level
// sets one after the other with a barrier between (no sentinel pre-fill, no
// polls), each row with k_trsv_level's operations (fm: GG_DIV_FMA's rows, y:
// the multiply); then, for the forward solve, the mesh rows' tail terms
// (k_border_sub's operations) -- the three or four launches of the general
// path (fill, flow, coupling) in one: 4-5 us each for an 800-row tail
__global__ __launch_bounds__(1024) void k_tail_small(Gate g, int nlev, const int *__restrict__ lev_ptr,
                                                     const int *__restrict__ rows, const int *__restrict__ rp,
                                                     const int *__restrict__ ci, const double *__restrict__ v,
                                                     const double *__restrict__ d, const double *__restrict__ y,
                                                     int fm, const double *b, double *x, int ncoup,
                                                     const long long *__restrict__ cslot, const int *__restrict__ crp,
                                                     const int *__restrict__ cci, const double *__restrict__ cv,
                                                     double *bmut, int cfm)
{
    if (gated(g)) return;
    for (int l = 0; l < nlev; l++) {
        const int q1 = lev_ptr[l + 1];
        for (int q = lev_ptr[l] + (int)threadIdx.x; q < q1; q += (int)blockDim.x) {
            const int r = rows[q];
            double acc;
            if (fm) {
                acc = y ? b[r] * y[r] : b[r];
                for (int k = rp[r]; k < rp[r + 1]; k++) acc = __builtin_fma(-v[k], x[ci[k]], acc);
            } else {
                acc = b[r];
                for (int k = rp[r]; k < rp[r + 1]; k++) acc = acc - v[k] * x[ci[k]];
                acc = y ? acc * y[r] : acc / d[r];
            }
            x[r] = acc;
        }
        __syncthreads();
    }
    for (int q = threadIdx.x; q < ncoup; q += blockDim.x) {
        const long long p = cslot[q];
        double acc = bmut[p];
        for (int k = crp[q]; k < crp[q + 1]; k++)
            acc = cfm ? __builtin_fma(-cv[k], x[cci[k]], acc) : acc - cv[k] * x[cci[k]];
        bmut[p] = acc;
    }
}

// The sharded solve's separator step in ONE launch (dd.hip apply_minv): the
// three row phases of SepFlow -- separator L rows (b_S - L_SI y_I, then the
// separator triangle's terms, / d), separator U rows (y_S, then the triangle's
// terms, / d), interface rows of the interior (y_I - U_IS x_S, in place) -- as
// one dataflow task list in that order (each phase in level order), short rows
// one per lane as in k_trsv_flow.  Every row runs the operations and order of
// the launches it replaces (k_sub_seq, k_trsv_flow, k_trsv_flow, k_sub_seq),
// so the result is the same bit for bit.  Values a row polls: its own-phase
// sources (sentinel = not ready) and, in the U phase, b = y_S.
__global__ __launch_bounds__(kBlock) void k_sep_flow(Gate g, int ntask, const int4 *__restrict__ tasks,
                                                     const int *__restrict__ rows, SepFlow f, int *err)
{
    if (gated(g)) return;
    const int lane = threadIdx.x & 63;
    const long long wid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long nw = (gridDim.x * (long long)blockDim.x) >> 6;
    for (long long t = wid; t < ntask; t += nw) {
        const int4 tk = tasks[t];
        const SepPhase &P = f.ph[tk.z];
        const unsigned long long *src = reinterpret_cast<const unsigned long long *>(P.src);
        const int r = lane < tk.y ? rows[tk.x + lane] : -1;
        bool pending = r >= 0;
        int k = pending ? P.rp[r] : 0;
        const int k1 = pending ? P.rp[r + 1] : 0;
        double acc = 0.0;
        bool have_b = !pending;
        if (pending && !P.bpoll) {
            acc = P.b[r];
            if (P.prp)
                for (int q = P.prp[r]; q < P.prp[r + 1]; q++) acc -= P.pv[q] * P.px[P.pci[q]];
            have_b = true;
        }
        int spins = 0;
        while (__any(pending)) {
            if (pending && !have_b) {
                const unsigned long long u = ld_agent(reinterpret_cast<const unsigned long long *>(P.b) + r);
                if (u != kSentinel) {
                    acc = __longlong_as_double((long long)u);
                    have_b = true;
                }
            }
            if (pending && have_b) {
                bool stop = false;
                while (!stop && k < k1) {
                    unsigned long long u[4];            // up to 4 polls in flight
#pragma unroll
                    for (int j = 0; j < 4; j++) u[j] = k + j < k1 ? ld_agent(src + P.ci[k + j]) : 0ull;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if (stop || k >= k1) break;
                        if (u[j] == kSentinel) { stop = true; break; }
                        acc = acc - P.v[k] * __longlong_as_double((long long)u[j]);
                        k++;
                    }
                }
                if (k == k1) {
                    const double o = P.d ? acc / P.d[r] : acc;
                    st_agent(reinterpret_cast<unsigned long long *>(P.x) + r, (unsigned long long)__double_as_longlong(o));
                    pending = false;
                }
            }
            if (__any(pending)) {
                __builtin_amdgcn_s_sleep(4);
                if (++spins > kSpinLimit) {
                    if (pending) atomicOr(err, 1);
                    pending = false;
                }
            }
        }
    }
}

// 2D structured-grid wavefront solve.  Layout (gg_internal.h Wave2D): band =
// 64 grid lines, lane l = line 64*band+l, step t = column i + l; a lane's two
// consecutive steps are adjacent in memory (16 B per array per step pair, 1 KiB
// per wave instruction).
//
// One workgroup per band, 3 + A waves (A = streamed arrays: b, c1, c2 and, for
// a non-unit triangle, the divisor d and its reciprocal):
//  * wave 0 (compute) runs the recurrence.  Each step a lane needs its own
//    previous value (same line, column i-+1) and the neighbour line's value
//    from the previous step, moved in-register with DPP wave_shr/wave_shl; the
//    edge lane keeps the DPP "old" operand, which holds the neighbouring band's
//    value.  Its operands come from LDS a few step pairs ahead of their use,
//    so the recurrence waits on memory at most once per batch; its results go to LDS staging (a global store costs the issuing
//    wave ~50 cycles, an LDS write a few);
//  * wave 2 (writer) stores the compute wave's x from LDS staging to HBM and
//    publishes the band's edge values, one batch behind;
//  * waves 3.. (loaders, one array each) stream HBM -> LDS with LDS-DMA
//    (global_load_lds_dwordx4) into an R-slot ring, each retiring batches with
//    its own counted vmcnt before the barrier (batch j by barrier j);
//  * wave 1 (boundary) polls the neighbouring band's edge values and hands
//    them over through LDS.
// All waves meet at one raw s_barrier per batch (no fence, no drain).
// Band-to-band hand-off (workgroups on different CUs): one 8-byte granule per
// step, bnd[band*T + t], whose payload is the flag (sentinel = not ready).  The
// producing band's writer wave stores the edge values of a batch with one
// relaxed agent-scope (sc1) store; the consumer polls with relaxed agent-scope loads
// and re-arms each granule it read (sc1 sentinel store) for the next launch.
// Every spin is bounded.
//
// Division (non-unit triangles).  x = RN(acc / d) is needed bit-exactly.  The
// IEEE division sequence (div_scale/rcp/fma/div_fmas/div_fixup) is ~70 cycles
// of dependent latency per step; WD_RCP instead uses the host-computed
// reciprocal y = RN(1/d) and two FMA corrections (Markstein):
//   q0 = RN(acc*y); q1 = RN(q0 + RN(acc - d*q0)*y); q2 = RN(q1 + (acc - d*q1)*y)
// q1 is within one ulp of acc/d, so acc - d*q1 is exact and q2 = RN(acc/d)
// (Markstein's theorem; y within half an ulp of 1/d).  The remainders are
// formed as -(d*q - acc) so signed zeros come out as in acc/d.  The theorem
// needs every intermediate in the normal range: the host admits WD_RCP only for
// 2^-100 <= |d| <= 2^100, and the writer wave flags results outside rcp_safe
// (err bit 2), on which the caller repeats the work with WD_HW.
// WD_MUL (gg_set_division(GG_DIV_RCP), tolerance parity): x = RN(acc * y) with
// the streamed y = RN(1/d) in place of d -- within about one ulp of RN(acc/d)
// per row, one dependent multiply instead of five operations, four streamed
// arrays instead of five.  The oracle restates it (orc_set_div_mode) for the
// order-matched checks; the host admits it when every 1/d is finite and normal.
// Steps per batch: one barrier, one boundary hand-over and one LDS-latency
// exposure per batch, so longer is cheaper per step, as far as the LDS budget
// lets the ring hold kWaveRing of them (GG_WAVE_BATCH_UNIT for the unit
// triangle, 3 streams; the non-unit ones stream 4-5 arrays).
#ifndef GG_WAVE_BATCH_UNIT
#define GG_WAVE_BATCH_UNIT 16
#endif
#ifndef GG_WAVE_POLL
#define GG_WAVE_POLL 2
#endif
#ifndef GG_WAVE_BATCH_HW
#define GG_WAVE_BATCH_HW 16
#endif
#ifndef GG_WAVE_BATCH_RCP
#define GG_WAVE_BATCH_RCP 16
#endif
// the compute wave reads a batch's operands after that batch's barrier, kWaveLook
// step pairs ahead of their use
#ifndef GG_WAVE_LOOK
#define GG_WAVE_LOOK 3
#endif
constexpr int kWaveLook = GG_WAVE_LOOK;
// the unit forward solve with the SpMV in its launch looks further ahead
// (round 5, one box each: C2's fused L 96.2 -> 93.8 us at 4 pairs; the U solve
// lost 1.5 us at 4 and the netlist's unfused unit L 2.2 us, so they keep 3)
#ifndef GG_WAVE_LOOK_L
#define GG_WAVE_LOOK_L 4
#endif
constexpr int kWaveLookL = GG_WAVE_LOOK_L;
// the compute wave's LDS traffic is issued in the shadow of each step's DPP shift
#ifndef GG_WAVE_SHADOW
#define GG_WAVE_SHADOW 1
#endif
constexpr bool kWaveShadow = GG_WAVE_SHADOW != 0;
// Ring depth: batches j and j+1 are in LDS at barrier j and kWaveRing-3 more are
// in flight (enough to cover the HBM latency at this stream rate).
#ifndef GG_WAVE_RING
#define GG_WAVE_RING 5
#endif
constexpr int kWaveRing = GG_WAVE_RING;
// One loader wave streaming every array, or one per array.  Every wave with
// loads in flight on a CU delays that CU's hand-off polls (MI355X_MICROARCH.md
// handoff-1to1: the price sits in the consumer CU's memory queue).
#ifndef GG_WAVE_LOADERS
#define GG_WAVE_LOADERS 1
#endif
constexpr int kWaveLoaders = GG_WAVE_LOADERS;
// the writer publishes a batch when the compute wave has staged it (1) or after
// the next batch's barrier (0); the boundary wave passes the barrier before (1)
// or after (0) its re-arm store and look-ahead poll.  Measured on C2 (U solve):
// 0/0 120.4 us, early barrier 123.8, decoupled 191-194 (the writer's LDS polls
// slow the compute wave's LDS traffic) -- so 0/0 for the 2D kernel, while the
// 3D tile kernel, whose bands wait on two sources, gains from both.
#ifndef GG_WAVE_DECOUPLE
#define GG_WAVE_DECOUPLE 0
#endif
// Round 6, re-measured on the per-wave compute loop (C2, one box, alternating,
// profiles/r06/earlybar_ab.txt): the early barrier helps the forward solve (L
// 83.2 -> 81.0 us) and not the backward one (U 81.2 -> 81.7): 2 = forward only
// (0 none, 1 both); C2 4,299 -> 4,339 it/s
#ifndef GG_WAVE_EARLYBAR
#define GG_WAVE_EARLYBAR 2
#endif
// (Measured, not kept, round 5: the 2D boundary wave retrying a batch's
// granules with two polls in flight, s_sleep 0 / 1 / 10 between them: C2 U
// 99.6 -> 102.6-105.6 us, L 95.7 -> 97.8-101.5 us, profiles/r05/stage_ab.txt.)
// GG_WAVE_XCD = X workgroups dealt per band of the backward solve, one running:
// the bands land on 8 / X of the XCDs (8: all on one XCD, 4: alternating over
// two, 2: over four).  Round 5, two compute waves per band, C2 on one box:
// U 99.3 us at 8 -> 97.9 at 4, 98.7 at 2 (profiles/r05/stage_ab.txt r05ab / r05ad)
#ifndef GG_WAVE_XCD
#define GG_WAVE_XCD 4
#endif
// Redundant compute waves: GG_WAVE_NC waves (on distinct SIMDs) run the same
// recurrence on the same operands -- bit-identical values -- and wave c stages
// only the step pairs kk with kk % NC == c for the writer wave.  A single
// wave's LDS store path runs at half rate (MI355X_MICROARCH.md LDS table:
// stores from one wave), so the pair's ds_write_b128 (~26 cycles) sat on the
// recurrence: C2 trace 44 cycles per step with it, 33 with no staging at all
// (timing bound, GG_WAVE_NOSTAGE; C2 4,123 -> 4,350 it/s on one box).
// Measured on one box (round 5, profiles/r05/stage_ab.txt): NC = 1 / 2 / 3 / 4
// 3,723 / 3,787 / 3,700 / 3,689 it/s (more waves: more LDS reads and a later
// barrier), so 2.  Not kept: four ds_write_addtid_b32 per pair instead of the
// b128 (one data dword, no address): 53 cycles per step -- a single wave's
// addtid stores run at a fraction of their rate.  Nor (round 5, C2 one box,
// profiles/r05/stage_ab.txt): the compute waves storing x themselves (one
// global_store_dwordx4 per pair) and handing only the edge lane's batch to the
// writer through LDS: 3,408 / 3,440 it/s (NC 2 / 1) against 3,773 -- stores
// from one active lane cost the store path what full ones do (8 b128 at the
// batch end: 551 cycles to the barrier).
#ifndef GG_WAVE_NC
#define GG_WAVE_NC 2
#endif
constexpr int kWaveNC = GG_WAVE_NC;
// diagnostics only (timing bound, wrong results): no x staging at all
#ifndef GG_WAVE_NOSTAGE
#define GG_WAVE_NOSTAGE 0
#endif

template <int DIV, bool D3 = false, int S = 1>
struct WaveCfg {
    // streamed arrays: b, c1, c2 (, d (, RN(1/d))); a skewed 2D grid (ILU(S-1))
    // adds the fill coefficients of offsets nx-1 .. nx-S+1; a 3D grid adds the
    // plane coefficient c0 and the previous plane's x
    static constexpr int AE = (DIV == WD_UNIT || DIV == WD_UFMA) ? 3 : DIV == WD_RCP ? 5 : 4;   // first fill array (WD_MUL / WD_SFMA stream y as d)
    static constexpr int A2 = AE + (S - 1);
    static constexpr int A = A2 + (D3 ? 2 : 0);
    static constexpr int B16 = (DIV == WD_UNIT || DIV == WD_UFMA) ? GG_WAVE_BATCH_UNIT
                             : DIV == WD_RCP  ? GG_WAVE_BATCH_RCP
                                              : GG_WAVE_BATCH_HW;
    // steps per batch: 8 where 16-step slots of A arrays would not leave room for 3 slots
    static constexpr int B = (B16 == 16 && 3 * A * 8 * 64 + 64 + 2 * 8 * 64 > 150 * 1024 / 16) ? 8 : B16;
    static constexpr int PBN = B / 2;                                     // step pairs per batch
    static constexpr int SLOT = A * PBN * 64;                            // double2 per ring slot
    // loader waves: GG_WAVE_LOADERS where it divides the arrays (2D, unskewed),
    // each streaming A / LOADERS of them with its own vmcnt budget
    static constexpr int LOADERS = (!D3 && S == 1 && kWaveLoaders > 1 && A % kWaveLoaders == 0) ? kWaveLoaders : 1;
    static constexpr int NA = A / LOADERS;                              // arrays per loader wave
    static constexpr int NPER = NA * PBN;                               // DMA instructions per batch per loader
    // ring slots: kWaveRing, at most what fits 150 KiB of LDS beside the boundary
    // values and the x staging, and at most what the 6-bit vmcnt can count
    static constexpr int RFIT = (150 * 1024 / 16 - 64 - 2 * PBN * 64) / SLOT;
    static constexpr int RVM = 2 + 63 / NPER;
    static constexpr int R = kWaveRing < RFIT ? (kWaveRing < RVM ? kWaveRing : RVM) : (RFIT < RVM ? RFIT : RVM);
    static constexpr int NC = kWaveNC;                                  // redundant compute waves
    static constexpr int THREADS = (2 + NC + LOADERS) * 64;             // compute(s), boundary, writer, loaders
    static constexpr int LDS2 = R * SLOT + 64 + 2 * PBN * 64;            // ring, boundary, x staging
    static_assert(R >= 3 && (R - 2) * NPER <= 63, "ring depth vs vmcnt range");
    static_assert(B == 8 || B == 16, "batch");
    static_assert(kWaveTAlign % (B * GG_WAVE_POLL) == 0, "batches per band must be a multiple of the poll depth");
    static_assert(!D3 || LOADERS == 1, "3D grids stream every array from one loader wave");
    static_assert(S >= 1 && S <= 3 && (S == 1 || (!D3 && LOADERS == 1)), "skew: 2D, one loader");
    static_assert(kWaveLook >= 1 && kWaveLook <= PBN && kWaveLookL >= 1 && kWaveLookL <= PBN, "lookahead");
    static_assert(LDS2 * 16 <= 160 * 1024, "LDS budget");
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// s_waitcnt immediate: wait until <= n vector-memory ops are outstanding (gfx9)
__host__ __device__ constexpr int vm_wait(int n)
{
    return (n & 15) | (7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14);
}
// wait until at most max(min(after, K), 0) batches of NPER instructions are in flight
template <int K, int NPER>
__device__ __forceinline__ void vm_wait_batches(int after)
{
    if constexpr (K == 0) {
        __builtin_amdgcn_s_waitcnt(vm_wait(0));
    } else {
        static_assert(K * NPER <= 63, "vmcnt is 6 bits");
        if (after >= K) __builtin_amdgcn_s_waitcnt(vm_wait(K * NPER));
        else vm_wait_batches<K - 1, NPER>(after);
    }
}

__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// 64-bit DPP lane shift whose out-of-range lane keeps `old`
template <int CTRL>
__device__ __forceinline__ double dpp_shift_old(double v, double old)
{
    int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// WD_RCP's range condition, checked on the results x (by the writer wave, off
// the recurrence): with 2^-100 <= |d| <= 2^100, |x| in [2^-800, 2^800] keeps
// |acc| = |x d| inside [2^-900, 2^900], where every intermediate of the two
// corrections is normal.  x == 0 comes from acc == 0, or from a quotient below
// 2^-1074 that both roundings flush alike except within one subnormal ulp.
__device__ __forceinline__ bool rcp_safe(double v)
{
    const double a = __builtin_fabs(v);
    return v == 0.0 || (a >= 0x1p-800 && a <= 0x1p800);
}

// loader wave: batch j -> ring slot j % R; batch j landed by barrier j
template <bool FWD, int R, int SLOT, int NA, int PBN, int SC1 = -1>
__device__ __forceinline__ void wave_loader(const double2 *const *src, double2 *lds, int np, int nbatch,
                                            long long *tr = nullptr)
{
    // array SC1 (a 3D grid's previous-plane x, written by another workgroup in
    // this launch) is read write-through coherent (sc1: cache policy 16)
    constexpr int PB = PBN * 64;                // double2 per array per slot
    auto issue = [&](int j) {
        double2 *slot = lds + (j % R) * SLOT;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a == SC1) continue;
#pragma unroll
            for (int kk = 0; kk < PBN; kk++) {
                const int p = j * PBN + kk;
                const long long q = (long long)(FWD ? p : np - 1 - p) * 64;
                __builtin_amdgcn_global_load_lds((gbl_void_t *)(src[a] + q),
                                                 (lds_void_t *)(slot + a * PB + kk * 64), 16, 0, 0);
            }
        }
        if constexpr (SC1 >= 0) {
#pragma unroll
            for (int kk = 0; kk < PBN; kk++) {
                const int p = j * PBN + kk;
                const long long q = (long long)(FWD ? p : np - 1 - p) * 64;
                __builtin_amdgcn_global_load_lds((gbl_void_t *)(src[SC1] + q),
                                                 (lds_void_t *)(slot + SC1 * PB + kk * 64), 16, 0, 16);
            }
        }
    };
    for (int j = 0; j < R - 1 && j < nbatch; j++) issue(j);
    for (int j = 0; j < nbatch; j++) {
        // batch j must have landed; the ones after it may stay in flight
        const int issued = j + R - 1 < nbatch ? j + R - 1 : nbatch;
        vm_wait_batches<R - 2, NA * PBN>(issued - (j + 1));
        if (tr && (threadIdx.x & 63) == 0) tr[j] = (long long)__builtin_amdgcn_s_memrealtime();   // diagnostics
        raw_barrier();                          // slot (j-1) % R is free from here on
        if (j + R - 1 < nbatch) issue(j + R - 1);
    }
}

// The SpMV fused into the forward solve's launch (GG_FUSE_SPMV, k_trsv_wave2d_spmv):
// b = A v is produced by extra workgroups of the same launch (blocks >= nbands)
// while the bands run.  Slices (64 layout rows, the sliced-ELL copy of A) are
// taken kFsGroup at a time in band-major order, each row summed exactly as
// k_spmv_sell sums it (entry order, no contraction), stored write-through
// (agent scope) and counted per band once drained; a band's loader wave waits
// for its band's count before its first batch (no DMA in flight then), re-arms
// the counter and streams b with the coherent (sc1) policy.  The SpMV blocks
// never wait on anything and take the LOW block indices, so they are dispatched
// before the bands that wait on them: with more bands than resident slots the
// SpMV blocks still finish and the bands run in dispatch order, each waiting
// only on blocks dispatched before it (with the bands first, a grid
// of nbands >= resident slots would spin on never-dispatched SpMV blocks).
struct FusedSpmv {
    const int *sptr = nullptr, *sci = nullptr;
    const double *sv = nullptr, *v = nullptr;
    double *w = nullptr;                    // = the solve's b
    unsigned long long *cnt = nullptr;      // per slice group: 1 = stored (0 between launches)
    const double *ydiv = nullptr;           // split engine: row divisors (k_spmv_sell's YDIV)
    const double *xdiv = nullptr;           // split engine: v[c] / xdiv[c] per gathered term (k_spmv_sell's XDIV)
    int n = 0;                              // rows of A (layout space)
    int ns = 0;                             // SpMV blocks: blockIdx < ns, the bands after them
};
// slices per group: C2 fused L 92.5 / 87.0 / 85.8 us at 8 / 4 / 2 (a group's
// chain is shorter with fewer loads per lane; profiles/r03/r03_fs_knobs.txt)
constexpr int kFsGroup = 2;                 // (kWaveTAlign is a multiple)

template <bool XD>
__device__ __forceinline__ void fused_spmv_groups(const FusedSpmv &fs, int nbands, int T, int nwv)
{
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NW = fs.ns * nwv;
    const int gpb = T / kFsGroup;
    const int ngroups = nbands * gpb;
    for (int q = (int)blockIdx.x * nwv + wv; q < ngroups; q += NW) {
        const int s0 = q * kFsGroup;
        int off[kFsGroup], wd[kFsGroup];
        int wmax = 0;
#pragma unroll
        for (int j = 0; j < kFsGroup; j++) {
            off[j] = fs.sptr[s0 + j];
            wd[j] = (fs.sptr[s0 + j + 1] - off[j]) >> 6;
            wmax = wd[j] > wmax ? wd[j] : wmax;
        }
        double acc[kFsGroup];
#pragma unroll
        for (int j = 0; j < kFsGroup; j++) acc[j] = 0.0;
        for (int k0 = 0; k0 < wmax; k0 += 8) {
            int c[kFsGroup][8];
            double a[kFsGroup][8], xv[kFsGroup][8];
#pragma unroll
            for (int j = 0; j < kFsGroup; j++)
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k0 + k < wd[j]) {
                        c[j][k] = __builtin_nontemporal_load(fs.sci + off[j] + lane + (k0 + k) * 64);
                        a[j][k] = __builtin_nontemporal_load(fs.sv + off[j] + lane + (k0 + k) * 64);
                    }
#pragma unroll
            for (int j = 0; j < kFsGroup; j++)
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k0 + k < wd[j] && c[j][k] >= 0) xv[j][k] = fs.v[c[j][k]];
            if constexpr (XD) {
                double dv[kFsGroup][8];
#pragma unroll
                for (int j = 0; j < kFsGroup; j++)
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        if (k0 + k < wd[j] && c[j][k] >= 0) dv[j][k] = fs.xdiv[c[j][k]];
#pragma unroll
                for (int j = 0; j < kFsGroup; j++)
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        if (k0 + k < wd[j] && c[j][k] >= 0) xv[j][k] = xv[j][k] / dv[j][k];
            }
#pragma unroll
            for (int j = 0; j < kFsGroup; j++)
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k0 + k < wd[j] && c[j][k] >= 0) acc[j] += a[j][k] * xv[j][k];
        }
#pragma unroll
        for (int j = 0; j < kFsGroup; j++) {
            const int r = (s0 + j) * 64 + lane;
            if (r < fs.n) {
                const double o = fs.ydiv ? acc[j] / fs.ydiv[r] : acc[j];
                st_agent(reinterpret_cast<unsigned long long *>(fs.w) + r, (unsigned long long)__double_as_longlong(o));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the group's rows stored
        if (lane == 0) st_agent(fs.cnt + q, 1ull);          // one word per group: no contention
    }
}
// xdiv (the split engine's D_r^-1 pass folded into the gathers, as
// k_spmv_sell<.., XDIV>): one uniform branch, the loops unchanged otherwise
__device__ __forceinline__ void fused_spmv_role(const FusedSpmv &fs, int nbands, int T, int nwv)
{
    if (fs.xdiv) fused_spmv_groups<true>(fs, nbands, T, nwv);
    else fused_spmv_groups<false>(fs, nbands, T, nwv);
}

// IL: the in-line term (|offset| = 1) comes first in the row's canonical order,
// then the line term -- the split (ILU++) U factor's ascending-column rows
// (MyILUPP::HostPrecond_right, src/preconditioner.cu:1117-1137).
// FS: the SpMV fused into the launch (see FusedSpmv; forward unskewed 2D only).
// BT: a batched launch (the many-RHS solve) -- zS scenarios of nbands
// workgroups each; scenario sc's b, x and hand-off granules (with its dummies)
// lie sc * zs bytes after scenario 0's, its control block likewise (the gate).
// zmap 0: workgroup = band * zS + sc (workgroups being dealt round-robin over
// the XCDs, a scenario's bands share an XCD when zS is a multiple of 8, so its
// hand-offs stay in one L2); zmap 1: workgroup = sc * nbands + band (band b of
// every scenario on one XCD: the coefficient streams shared in its L2).
template <bool FWD, int DIV, bool TRACE, bool D3, int S, bool IL, bool FS, bool BT = false>
__device__ __forceinline__ void trsv_wave2d_body(
    Gate g, int T, int nbands, const double *__restrict__ b, const double *__restrict__ c1,
    const double *__restrict__ c2, const double *__restrict__ dv, const double *__restrict__ rv,
    double *__restrict__ x, unsigned long long *bnd, int *err, long long *trace,
    int nz, long long P2, const double *__restrict__ c0, unsigned long long *prog,
    const double *__restrict__ ce1, const double *__restrict__ ce2, const FusedSpmv &fs,
    int zS = 1, long long zs = 0, int zmap = 0)
{
    using C = WaveCfg<DIV, D3, S>;
    // LDS work in the lane shift's shadow -- not for the unit L's fused rows,
    // whose step is one FMA after the shift: there the pair's reads and staging
    // write go after the pair (C2 fused L 86.7 -> 84.5 us, netlist L 91.5 ->
    // 90.4; the other forms keep it: the exact unit L 88.9 -> 90.3 without)
    constexpr bool SH = kWaveShadow && DIV != WD_UFMA;
    static_assert(!FS || (FWD && !D3 && S == 1 && !TRACE), "fused SpMV: forward 2D");
    static_assert(!IL || (S == 1 && !D3), "in-line-first rows: unskewed 2D grids");
    constexpr bool FM = DIV == WD_UFMA || DIV == WD_SFMA;     // GG_DIV_FMA rows
    static_assert(!FM || (!D3 && !IL), "fused rows: 2D grids (one order for both IL)");
    static_assert(!(TRACE && S > 1), "no trace for skewed grids");
    constexpr int PB = C::PBN * 64;            // double2 per array per slot
    static_assert(!(D3 && TRACE), "no trace for 3D grids");
    static_assert(!BT || (!FS && !D3 && !TRACE), "batched: 2D, separate SpMV, no trace");
    if (!BT && gated(g)) return;
    int bid = (int)blockIdx.x;                  // this workgroup among the bands
    if constexpr (BT) {
        const int sc = zmap == 0 ? bid % zS : bid / nbands;
        bid = zmap == 0 ? bid / zS : bid % nbands;
        if (gated_z(g, zs, sc)) return;
        b = zp(b, zs, sc);
        x = zp(x, zs, sc);
        bnd = zp(bnd, zs, sc);
    }
    if constexpr (FS) {
        if (bid < fs.ns) {
            fused_spmv_role(fs, nbands, T, C::THREADS / 64);
            return;
        }
        bid -= fs.ns;
    }
    // one LDS object: data ring [R][A][C::PBN][64] double2, 2 x 64 boundary values
    // (lanes 0..C::B-1 of each half are used), x staging [2][C::PBN][64]
    __shared__ double2 lds[C::LDS2];
    __shared__ int xdone;                       // batches the compute wave has staged (GG_WAVE_DECOUPLE)
    double2 *ring = lds;                        // ring | boundary | x staging
    double *bring = reinterpret_cast<double *>(lds + C::R * C::SLOT);
    double2 *xbuf = lds + C::R * C::SLOT + 64;
    if (threadIdx.x == 0) xdone = 0;            // read only after the first barrier
    int seq = 0;                                // batches this workgroup has run (uniform)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int np = T / 2;                       // step pairs per band
    const int nbatch = T / C::B;          // T is a multiple of kWaveTAlign
    constexpr int plane = FWD ? 63 : 0;     // lane whose values the next band needs
    // Tasks: (plane, band) in dependency order, a workgroup takes every
    // gridDim.x-th (2D: one band per workgroup, nz = 1).  A 3D task also needs
    // the previous plane's x (same band): its writer publishes prog[] =
    // batches stored, the boundary wave polls it, the loader streams it.
    // GG_WAVE_XCD = X > 1 (2D backward solve): the launch has X workgroups per
    // band and only every X-th runs one, so that (workgroups being dealt
    // round-robin over the XCDs) the bands share one XCD and its L2 --
    // placement is for speed only, the hand-off protocol is the same.
    // Measured on C2: U 121.0 -> 117.9 us, while L (3 streamed arrays) slows
    // 88.9 -> 90.0 us (round 3, re-measured: 89.4 / 90.3 -> 89.9 / 90.4 us), so
    // the forward solve keeps one workgroup per band.
    // (the fused SpMV's launch holds one workgroup per band: no placement there)
    constexpr int XS = (D3 || FS || FWD || BT) ? 1 : GG_WAVE_XCD;
    if (XS > 1 && bid % XS) return;
    const int blk = bid / XS;
    const int ntask = nz * nbands;
    for (int task = blk; task < ntask; task += ((FS || BT) ? nbands : (int)gridDim.x / XS)) {
    const int kq = task / nbands, bq = task % nbands;
    const int band = FWD ? bq : (nbands - 1 - bq);
    const int kp = FWD ? kq : (nz - 1 - kq);    // plane
    const bool has_src = FWD ? (band > 0) : (band < nbands - 1);
    const bool is_prod = FWD ? (band < nbands - 1) : (band > 0);
    const bool has_prev = D3 && (FWD ? kp > 0 : kp < nz - 1);
    const long long boff = (long long)band * np * 64 + lane + (long long)kp * (P2 / 2);   // double2 units
    const long long prev_off = (FWD ? -1 : 1) * (P2 / 2);                                // previous plane
    unsigned long long *pub = bnd + ((long long)kp * nbands + band) * T;
    unsigned long long *prog_mine = D3 ? prog + (long long)kp * nbands + band : nullptr;
    unsigned long long *prog_prev = has_prev ? prog + (long long)(FWD ? kp - 1 : kp + 1) * nbands + band : nullptr;
    constexpr int NC = C::NC;                   // waves [0, NC) compute, NC boundary, NC + 1 writer, loaders
    static_assert(NC >= 1 && NC <= 4 && (NC == 1 || !GG_WAVE_DECOUPLE), "redundant compute waves");
    if (wave >= NC + 2) {
        // ------------------------------------------------ loader wave(s)
        const int li = wave - NC - 2;           // this loader's arrays: [li * NA, (li + 1) * NA)
        const double2 *src[7] = {reinterpret_cast<const double2 *>(b) + boff,
                                 reinterpret_cast<const double2 *>(c1) + boff,
                                 reinterpret_cast<const double2 *>(c2) + boff,
                                 reinterpret_cast<const double2 *>(dv) + boff,
                                 reinterpret_cast<const double2 *>(rv) + boff,
                                 nullptr, nullptr};
        if constexpr (S >= 2) src[C::AE] = reinterpret_cast<const double2 *>(ce1) + boff;
        if constexpr (S >= 3) src[C::AE + 1] = reinterpret_cast<const double2 *>(ce2) + boff;
        if constexpr (D3) {
            // the plane coefficient and the previous plane's x (zeros on the
            // first plane, where c0 is 0) follow the 2D arrays
            src[C::A2] = reinterpret_cast<const double2 *>(c0) + boff;
            src[C::A2 + 1] = reinterpret_cast<const double2 *>(has_prev ? x : c0) + boff + (has_prev ? prev_off : 0);
        }
        if constexpr (D3) {
            // the prologue streams batches 0..R-2 before the boundary wave has
            // checked anything: wait here for the previous plane to store them
            // (no DMA is in flight yet, so a blocking poll is free)
            if (has_prev) {
                const unsigned long long need = (unsigned long long)(C::R - 1 < nbatch ? C::R - 1 : nbatch);
                int spins = 0;
                while (ld_agent(prog_prev) < need) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) {
                        if (lane == 0) atomicOr(err, 1);
                        break;
                    }
                }
            }
        }
        if (FS && li == 0) {
            // this band's b rows all stored by the SpMV blocks (no DMA in flight
            // yet: a blocking poll is free); the counter is re-armed after the
            // stream (a store in flight would upset the loader's vmcnt count)
            // -- by the loader of b (array 0) alone
            const int gpb = T / kFsGroup;
            const unsigned long long *fl = fs.cnt + (long long)band * gpb;
            auto all_stored = [&]() {
                bool ok = true;
                for (int k = lane; k < gpb; k += 64) ok &= ld_agent(fl + k) != 0ull;
                return __all(ok);
            };
            int spins = 0;
            while (!all_stored()) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinLimit) {
                    if (lane == 0) atomicOr(err, 1);
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        if constexpr (C::LOADERS == 1) {
            wave_loader<FWD, C::R, C::SLOT, C::A, C::PBN, D3 ? C::A2 + 1 : FS ? 0 : -1>(src, ring, np, nbatch);
        } else if (li == 0) {
            wave_loader<FWD, C::R, C::SLOT, C::NA, C::PBN, FS ? 0 : -1>(src, ring, np, nbatch);
        } else {
            wave_loader<FWD, C::R, C::SLOT, C::NA, C::PBN>(src + li * C::NA, ring + li * C::NA * PB, np, nbatch);
        }
        if (FS && li == 0) {
            const int gpb = T / kFsGroup;
            for (int k = lane; k < gpb; k += 64) st_agent(fs.cnt + (long long)band * gpb + k, 0ull);   // re-arm
        }
        raw_barrier();                      // final barrier (the writer drains the last batch)
        continue;
    }
    if (wave == NC + 1) {
        // ------------------------------------------------ writer wave
        // After barrier bi+1 the compute wave's x of batch bi sits in xbuf[bi & 1]:
        // store it to HBM and publish the edge lane's values of the batch as
        // hand-off granules (lanes 0..C::B-1, one coalesced sc1 store).
        // 3D: x is stored write-through (sc1) and, once a batch's stores have
        // drained (checked one batch later, off the critical path), counted in
        // prog_mine for the next plane.
        // GG_WAVE_DECOUPLE: batch bi is published as soon as the compute wave
        // has staged it (LDS counter xdone), not after barrier bi+1, which
        // also waits for this band's boundary values of batch bi+1: a band's
        // upstream must not hold back what it hands downstream.
        double2 *X2 = reinterpret_cast<double2 *>(x) + boff;
        [[maybe_unused]] bool bad = false;  // WD_RCP range guard (see rcp_safe)
        for (int bi = 0; bi <= nbatch; bi++) {
            if (!GG_WAVE_DECOUPLE || bi == 0) raw_barrier();
            if (bi == 0) continue;
            const int pb = bi - 1;
            if constexpr (GG_WAVE_DECOUPLE) {
                while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&xdone, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)) <= seq + pb)
                    __builtin_amdgcn_s_sleep(1);
            }
            if constexpr (D3) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // batches < pb stored
                if (lane == 0 && pb > 0) st_agent(prog_mine, (unsigned long long)pb);
            }
            const double2 *xb = xbuf + (pb & 1) * PB;
            // the hand-off granules first: they are on the critical path, x is not
            const int tt = lane & (C::B - 1);
            const double e = reinterpret_cast<const double *>(xb + (tt >> 1) * 64 + plane)
                [FWD ? (tt & 1) : 1 - (tt & 1)];
            if (is_prod && lane < C::B) {
                const int t = FWD ? pb * C::B + tt : (T - 1) - (pb * C::B + tt);
                st_agent(pub + t, (unsigned long long)__double_as_longlong(e));
            }
            double2 v[C::PBN];
#pragma unroll
            for (int kk = 0; kk < C::PBN; kk++) v[kk] = xb[kk * 64 + lane];
#pragma unroll
            for (int kk = 0; kk < C::PBN; kk++) {
                const int p = pb * C::PBN + kk;
                double2 *dst = X2 + (long long)(FWD ? p : np - 1 - p) * 64;
                if constexpr (D3) {
                    st_sc1_16(dst, v[kk]);
                } else {
                    *dst = v[kk];
                }
                if constexpr (DIV == WD_RCP) bad |= !rcp_safe(v[kk].x) || !rcp_safe(v[kk].y);
            }

            if (TRACE && lane == 0)
                trace[(long long)band * (3 * nbatch + 8) + nbatch + 8 + pb] =
                    (long long)__builtin_amdgcn_s_memrealtime();
            if constexpr (GG_WAVE_DECOUPLE) raw_barrier();     // barrier bi (the last: the final one)
        }
        seq += nbatch;
        if constexpr (D3) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) st_agent(prog_mine, (unsigned long long)nbatch);
        }
        if constexpr (DIV == WD_RCP) {
            if (__any(bad) && lane == 0) atomicOr(err, 2);
        }
        continue;
    }
    if (wave == NC) {
        // ------------------------------------------------ boundary wave
        // Before barrier bi it places batch bi's values in bring[bi & 1].  Step
        // t of this band's edge lane needs the source band's step t -+ 63.  Polls
        // are pipelined kPoll batches deep (one register per ring position): the
        // load for batch bi+kPoll is issued right after batch bi is handed over,
        // so in steady state a batch's granules have arrived when it is checked.
        // Every memory op is issued by all lanes (lanes with nothing to do use
        // the dummy granules after the bands: 64 zeros to read, 64 to write),
        // which keeps the vmcnt arithmetic exact.
        constexpr int kPoll = GG_WAVE_POLL;
        // the barrier before (EB) or after the re-arm store and look-ahead poll
        constexpr bool EB = GG_WAVE_EARLYBAR == 1 || (GG_WAVE_EARLYBAR == 2 && FWD);
        // 3D: lane 32 polls the previous plane's progress instead: before
        // barrier bi it must have stored the batches the loader streams after
        // it (up to bi + R - 1); its word is never re-armed here, but reset to
        // 0 when this task is done (the producer has finished by then).
        unsigned long long *src = bnd + ((long long)kp * nbands + (FWD ? band - 1 : band + 1)) * T;
        // this workgroup's dummy granules (64 zeros to read, 64 write-only words)
        unsigned long long *dummy_ld = bnd + (long long)nz * nbands * T + (long long)blk * 128 + lane;
        unsigned long long *dummy_st = dummy_ld + 64;
        constexpr int kProgLane = 32;
        const bool prog_lane = has_prev && lane == kProgLane;
        auto gaddr = [&](int bj) {
            const int t = FWD ? bj * C::B + lane : (T - 1) - (bj * C::B + lane);
            const int gi = FWD ? t + (64 * S - 1) : t - (64 * S - 1);     // the neighbour's edge lane
            const bool need = has_src && lane < C::B && bj < nbatch && gi >= 0 && gi < T;
            return need ? src + gi : (unsigned long long *)nullptr;
        };
        auto poll_addr = [&](int bj) -> unsigned long long * {
            if (prog_lane) return prog_prev;
            unsigned long long *ga = gaddr(bj);
            return ga ? ga : dummy_ld;
        };
        auto ready = [&](unsigned long long w, int bj) {
            if (prog_lane) return w >= (unsigned long long)(bj + C::R < nbatch ? bj + C::R : nbatch);
            return w != kSentinel;
        };
        // the prologue mirrors the steady-state issue order (re-arm store, poll)
        // so the same vmcnt holds in every iteration
        unsigned long long v[kPoll];
#pragma unroll
        for (int u = 0; u < kPoll; u++) {
            if (u > 0) st_agent(dummy_st, kSentinel);
            v[u] = ld_agent(poll_addr(u));
        }
        bool dead = false;
        long long bw_spins = 0, bw_cyc = 0;     // TRACE: poll retries, cycles in retry loops
        for (int bi0 = 0; bi0 < nbatch; bi0 += kPoll) {     // nbatch is a multiple of kPoll
#pragma unroll
            for (int u = 0; u < kPoll; u++) {
                const int bi = bi0 + u;
                unsigned long long *ga = gaddr(bi);
                // oldest poll done: after it come kPoll-1 loads and kPoll-1 re-arm stores
                __builtin_amdgcn_s_waitcnt(vm_wait(2 * (kPoll - 1)));
                int spins = 0;
                const long long tw = TRACE ? (long long)__builtin_amdgcn_s_memtime() : 0;
                while (!dead && !__all(ready(v[u], bi))) {
                    __builtin_amdgcn_s_sleep(1);
                    v[u] = ld_agent(poll_addr(bi));
                    if (++spins > kSpinLimit) {
                        dead = true;
                        if (lane == 0) atomicOr(err, 1);
                    }
                    __builtin_amdgcn_s_waitcnt(vm_wait(0));
                }
                if constexpr (TRACE) {
                    bw_spins += spins;
                    if (spins) bw_cyc += (long long)__builtin_amdgcn_s_memtime() - tw;
                    if (lane == 0)
                        trace[(long long)band * (3 * nbatch + 8) + 2 * nbatch + 8 + bi] =
                            (long long)__builtin_amdgcn_s_memrealtime();
                }
                bring[(bi & 1) * 64 + lane] = __longlong_as_double((long long)v[u]);
                if constexpr (EB) {
                    // hand the values over first, then re-arm and poll ahead
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    raw_barrier();
                }
                st_agent(ga ? ga : dummy_st, kSentinel);       // re-arm for the next launch
                v[u] = ld_agent(poll_addr(bi + kPoll));
                if constexpr (!EB) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    raw_barrier();
                }
            }
        }
        raw_barrier();                      // final barrier (the writer drains the last batch)
        if (TRACE && lane == 0) {
            long long *trb = trace + (long long)band * (3 * nbatch + 8);
            trb[nbatch + 5] = bw_spins;
            trb[nbatch + 6] = bw_cyc;
        }
        if (prog_lane) {
            __builtin_amdgcn_s_waitcnt(vm_wait(0));
            st_agent(prog_prev, 0ull);              // re-arm for the next launch
        }
        continue;
    }

    // ---------------------------------------------------- compute wave(s)
    // One copy of the loop per compute wave, its share of the staging (pairs
    // kk with kk % NC == cw) a compile-time choice: a run-time test of the
    // wave index put a scalar branch around every staging store, splitting
    // the scheduled pair into basic blocks (C2 L / U 85 -> 93 / 97 us on one
    // box, profiles/r05/r05_vs_r04/)
    auto compute_wave = [&](auto cw_tag) {
    constexpr int cw = decltype(cw_tag)::value;
    constexpr int ctrl = FWD ? 0x138 : 0x130;   // wave_shr:1 / wave_shl:1
    long long *tr = TRACE && cw == 0 ? trace + (long long)band * (3 * nbatch + 8) : nullptr;
    long long ph[4] = {0, 0, 0, 0};     // TRACE: barrier wait, top->step0, step0->last, last->end
    long long t_top = 0;
    double xp = 0.0;                        // this lane's previous step value
    double xh1 = 0.0, xh2 = 0.0;            // skew > 1: the neighbour line's values 2 and 3 steps back
    // Operands of the current batch in registers, read kWaveLook step pairs
    // ahead of their use; the boundary values are read first (LDS returns in
    // order and they are needed at the batch's first step).
    double2 rg[C::PBN][C::A];
    constexpr int LK = (FS && (DIV == WD_UNIT || DIV == WD_UFMA)) ? kWaveLookL : kWaveLook;
    // one step pair's x into staging half h, pair kk (.x = the value at the
    // lower memory address)
    auto stage = [&](int h, int kk, double vx, double vy) {
        if constexpr (!GG_WAVE_NOSTAGE) {
            if (kk % NC == cw) xbuf[h * PB + kk * 64 + lane] = make_double2(vx, vy);
        }
    };
    raw_barrier();                          // barrier 0: batch 0 is in LDS
    for (int bi = 0; bi < nbatch; bi++) {
        if (bi > 0) {
            // x staging writes of batch bi-1 complete before the barrier (writer)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (TRACE) {
                const long long ta = (long long)__builtin_amdgcn_s_memtime();
                ph[3] += ta - t_top;
                raw_barrier();
                ph[0] += (long long)__builtin_amdgcn_s_memtime() - ta;
            } else {
                raw_barrier();              // batch bi's data and boundary values
            }
        }
        if constexpr (TRACE) {
            if (lane == 0 && tr) tr[bi] = (long long)__builtin_amdgcn_s_memrealtime();
        }
        const double2 *br = reinterpret_cast<const double2 *>(bring + (bi & 1) * 64);
        // issue order = need order: the first pair's boundary values and
        // operands, then the look-ahead pairs, then the remaining boundary
        // values (LDS returns in order, so the first step waits on ~A+1 reads)
        double2 bv[C::PBN];
        const double2 *sc = ring + (bi % C::R) * C::SLOT + lane;
        bv[0] = br[0];
#pragma unroll
        for (int a = 0; a < C::A; a++) rg[0][a] = sc[a * PB];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 1; kk < LK; kk++)
#pragma unroll
            for (int a = 0; a < C::A; a++) rg[kk][a] = sc[a * PB + kk * 64];
#pragma unroll
        for (int kk = 1; kk < C::PBN; kk++) bv[kk] = br[kk];    // broadcast reads
        if constexpr (TRACE) t_top = (long long)__builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        double xv[C::B];
#pragma unroll
        for (int kk = 0; kk < C::PBN; kk++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int tt = 2 * kk + h;
                const bool sx = FWD ? (h == 0) : (h == 1);     // even step <-> .x
                const double bb = sx ? rg[kk][0].x : rg[kk][0].y;
                const double e1 = sx ? rg[kk][1].x : rg[kk][1].y;
                const double e2 = sx ? rg[kk][2].x : rg[kk][2].y;
                const double old = h ? bv[kk].y : bv[kk].x;
                const double p2 = FM ? 0.0 : e2 * xp;
                // GG_DIV_FMA: the in-line term first, fused, while the line
                // value crosses lanes; b pre-scaled by y = RN(1/d) for U (the
                // coefficients arrive pre-scaled), off the recurrence
                double tf = 0.0;
                if constexpr (FM) {
                    double by = bb;
                    if constexpr (DIV == WD_SFMA) by = bb * (sx ? rg[kk][3].x : rg[kk][3].y);
                    tf = __builtin_fma(-e2, xp, by);
                }
                // 3D: the plane neighbour comes first in the canonical order
                // (|offset| = nx*ny); its term is off the recurrence
                double bz = bb;
                if constexpr (D3) {
                    const double e0 = sx ? rg[kk][C::A2].x : rg[kk][C::A2].y;
                    const double xz = sx ? rg[kk][C::A2 + 1].x : rg[kk][C::A2 + 1].y;
                    bz = bb - e0 * xz;
                }
                const double xs = dpp_shift_old<ctrl>(xp, old);
                if constexpr (SH) {
                    // LDS work of the pair in the cross-lane shift's latency:
                    // the look-ahead reads at the first step, the previous
                    // pair's x staging at the second
                    __builtin_amdgcn_sched_barrier(0);
                    if (h == 0 && kk + LK < C::PBN) {
#pragma unroll
                        for (int a = 0; a < C::A; a++) rg[kk + LK][a] = sc[a * PB + (kk + LK) * 64];
                    }
                    if (h == 1 && kk > 0) {
                        if (FWD) stage(bi & 1, kk - 1, xv[2 * kk - 2], xv[2 * kk - 1]);
                        else stage(bi & 1, kk - 1, xv[2 * kk - 1], xv[2 * kk - 2]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                // the neighbour line's terms oldest first (|offset| = nx, nx-1, ..),
                // then the in-line neighbour (|offset| = 1)
                double acc;
                if constexpr (FM && S == 1) {
                    acc = __builtin_fma(-e1, xs, tf);
                } else if constexpr (FM && S == 2) {
                    // nearest first: in-line (tf), fill nx-1 (xs), line nx (xh1)
                    const double f1 = sx ? rg[kk][C::AE].x : rg[kk][C::AE].y;
                    acc = __builtin_fma(-f1, xs, tf);
                    acc = __builtin_fma(-e1, xh1, acc);
                } else if constexpr (FM) {
                    // in-line, fill nx-2 (xs), fill nx-1 (xh1), line nx (xh2)
                    const double f1 = sx ? rg[kk][C::AE].x : rg[kk][C::AE].y;
                    const double f2 = sx ? rg[kk][C::AE + 1].x : rg[kk][C::AE + 1].y;
                    acc = __builtin_fma(-f2, xs, tf);
                    acc = __builtin_fma(-f1, xh1, acc);
                    acc = __builtin_fma(-e1, xh2, acc);
                } else if constexpr (IL) {
                    acc = bz - p2;
                    acc = acc - e1 * xs;
                } else if constexpr (S == 1) {
                    acc = bz - e1 * xs;
                } else if constexpr (S == 2) {
                    const double f1 = sx ? rg[kk][C::AE].x : rg[kk][C::AE].y;
                    acc = bz - e1 * xh1;
                    acc = acc - f1 * xs;
                } else {
                    const double f1 = sx ? rg[kk][C::AE].x : rg[kk][C::AE].y;
                    const double f2 = sx ? rg[kk][C::AE + 1].x : rg[kk][C::AE + 1].y;
                    acc = bz - e1 * xh2;
                    acc = acc - f1 * xh1;
                    acc = acc - f2 * xs;
                }
                if constexpr (S >= 3) xh2 = xh1;
                if constexpr (S >= 2) xh1 = xs;
                if constexpr (!IL && !FM) acc = acc - p2;
                if constexpr (DIV == WD_HW) {
                    acc = acc / (sx ? rg[kk][3].x : rg[kk][3].y);
                } else if constexpr (DIV == WD_MUL) {
                    acc = acc * (sx ? rg[kk][3].x : rg[kk][3].y);
                } else if constexpr (DIV == WD_RCP) {
                    const double d = sx ? rg[kk][3].x : rg[kk][3].y;
                    const double y = sx ? rg[kk][4].x : rg[kk][4].y;
                    const double q0 = acc * y;
                    const double q1 = __builtin_fma(-__builtin_fma(q0, d, -acc), y, q0);
                    acc = __builtin_fma(-__builtin_fma(q1, d, -acc), y, q1);
                }
                xp = acc;
                xv[tt] = acc;
                if constexpr (TRACE) {      // phase stamps at the first and last step
                    if (tt == 0 || tt == C::B - 1) {
                        const int f = __builtin_amdgcn_readfirstlane(__double2hiint(acc));
                        asm volatile("; use %0" ::"s"(f));
                        const long long now = (long long)__builtin_amdgcn_s_memtime();
                        ph[tt == 0 ? 1 : 2] += now - t_top;
                        t_top = now;
                    }
                }
            }
            // the pair's results go to LDS staging (the writer wave stores them
            // and publishes the edge values), then the pair kWaveLook ahead is
            // read; the scheduling fence keeps it all inside this pair, in the
            // recurrence's latency bubbles
            if (!SH || kk == C::PBN - 1) {
                if (FWD) stage(bi & 1, kk, xv[2 * kk], xv[2 * kk + 1]);
                else stage(bi & 1, kk, xv[2 * kk + 1], xv[2 * kk]);
            }

            if (!SH && kk + LK < C::PBN) {
#pragma unroll
                for (int a = 0; a < C::A; a++) rg[kk + LK][a] = sc[a * PB + (kk + LK) * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (GG_WAVE_DECOUPLE) {       // the batch's x staging, then the writer's counter
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&xdone, seq + bi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    seq += nbatch;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                          // final barrier: the writer drains the last batch
    if (TRACE && lane == 0 && tr) {
        tr[nbatch] = (long long)__builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int k = 0; k < 4; k++) tr[nbatch + 1 + k] = ph[k];
    }
    };
    if (NC == 1 || wave == 0) compute_wave(std::integral_constant<int, 0>{});
    else if (NC == 2 || wave == 1) compute_wave(std::integral_constant<int, NC >= 2 ? 1 : 0>{});
    else if (NC == 3 || wave == 2) compute_wave(std::integral_constant<int, NC >= 3 ? 2 : 0>{});
    else compute_wave(std::integral_constant<int, NC >= 4 ? 3 : 0>{});
    }   // task loop
}

template <bool FWD, int DIV, bool TRACE, bool D3 = false, int S = 1, bool IL = false>
__global__ __launch_bounds__((WaveCfg<DIV, D3, S>::THREADS)) void k_trsv_wave2d(
    Gate g, int T, int nbands, const double *__restrict__ b, const double *__restrict__ c1,
    const double *__restrict__ c2, const double *__restrict__ dv, const double *__restrict__ rv,
    double *__restrict__ x, unsigned long long *bnd, int *err, long long *trace,
    int nz, long long P2, const double *__restrict__ c0, unsigned long long *prog,
    const double *__restrict__ ce1, const double *__restrict__ ce2)
{
    trsv_wave2d_body<FWD, DIV, TRACE, D3, S, IL, false>(g, T, nbands, b, c1, c2, dv, rv, x, bnd, err, trace, nz,
                                                        P2, c0, prog, ce1, ce2, FusedSpmv{});
}

// forward 2D solve with b = A v computed by the launch's blocks < fs.ns (FusedSpmv)
template <int DIV>
__global__ __launch_bounds__((WaveCfg<DIV>::THREADS)) void k_trsv_wave2d_spmv(
    Gate g, int T, int nbands, const double *__restrict__ c1, const double *__restrict__ c2,
    const double *__restrict__ dv, const double *__restrict__ rv, double *__restrict__ x,
    unsigned long long *bnd, int *err, long long P2, FusedSpmv fs)
{
    trsv_wave2d_body<true, DIV, false, false, 1, false, true>(g, T, nbands, fs.w, c1, c2, dv, rv, x, bnd, err,
                                                              nullptr, 1, P2, nullptr, nullptr, nullptr, nullptr,
                                                              fs);
}

// batched 2D solve (the many-RHS solve): zS scenarios, nbands workgroups each
template <bool FWD, int DIV>
__global__ __launch_bounds__((WaveCfg<DIV>::THREADS)) void k_trsv_wave2d_batch(
    Gate g, int T, int nbands, const double *__restrict__ b, const double *__restrict__ c1,
    const double *__restrict__ c2, const double *__restrict__ dv, const double *__restrict__ rv,
    double *__restrict__ x, unsigned long long *bnd, int *err, long long P2, int zS, long long zs, int zmap)
{
    trsv_wave2d_body<FWD, DIV, false, false, 1, false, false, true>(g, T, nbands, b, c1, c2, dv, rv, x, bnd, err,
                                                                    nullptr, 1, P2, nullptr, nullptr, nullptr,
                                                                    nullptr, FusedSpmv{}, zS, zs, zmap);
}

// ================================================ 3D 7-point grids: tile wavefront
// Layout (gg_internal.h Wave2D, tile = true): one wave owns a tile of 8 lines
// x 8 planes, lane l = a + 8 g(c) with the Gray code g(c) = c ^ (c >> 1) for
// plane c = 0..7, and runs point (i, j, k) at step t = i + a + c.  Every term
// of a row is then a recent value of a neighbouring lane: the in-line term the
// lane's own previous step; the line term the previous step one lane down its
// 8-lane half-row (DPP row_shr:1, backward row_shl:1; the half-row's edge lane
// takes the neighbouring tile's value -- as the DPP `old` in half-row 0 of a
// row, by a select in half-row 1); the plane term the previous step's value in
// the predecessor plane's half-row, which differs in one bit of g: one DPP
// row_ror:8 (bit 0), in-place v_permlane16_swap (bit 1) or v_permlane32_swap
// (bit 2) plus selects.  The first plane's half-row takes the neighbouring
// tile's value.  Round 2 skewed planes by two steps so that the plane move ran
// a step ahead, off the recurrence; but the step is issue-bound (≈ 30
// instructions), not chain-bound, and the extra skew cost a K hop 16 steps and
// one more batch of granularity instead of 8: with skew 1 the plane move sits
// on the chain and every hop is 8 steps + one batch.  The dependency chain
// (nx + ny + nz - 2 steps) crosses a workgroup boundary every 8 lines and every
// 8 planes: 26 + 26 hand-offs at 216^3 (round 1: 216 plane hops through HBM).
// Hand-off granules (8 B, value = flag, kSentinel = not ready, re-armed by the
// consumer): per tile and step 16 words, [0, 8) the last plane's half-row for
// tile (J, K +- 1), [8, 16) the eight planes' edge lanes for tile (J +- 1, K).
// The consumer's step t needs the plane and the line granules of step t +- 7
// (same point i, skew a + c).
// Roles as k_trsv_wave2d: wave 0 computes, 1 polls the granules, 2 stores x
// and publishes, 3 streams b, c1, c2 (, d (, RN(1/d))), c0 into the LDS ring.
// Persistent grid, every workgroup co-resident, tiles taken in dependency
// order (host tile_order; the backward solve walks it from the end).
#ifndef GG_TILE_BATCH
#define GG_TILE_BATCH 8
#endif
// 3 slots: 59-70 KiB of LDS, two workgroups per CU -- at the C4 wavefront's
// peak more tiles are ready than there are CUs (C4 L 227 -> 222 us, U 234 ->
// 233 us against 5 slots, profiles/r03/r03_tile_ring.txt)
#ifndef GG_TILE_RING
#define GG_TILE_RING 3
#endif
// boundary wave retries: 0 = one poll at a time, n > 0 = two generations in
// flight, the second issued s_sleep(n) after the first (measured at C4: L/U
// 260-263 / 286-287 us against 246 / 269 -- the extra polls cost more than
// the earlier sight gains)
#ifndef GG_TILE_POLL2
#define GG_TILE_POLL2 0
#endif
template <int DIV>
struct TileCfg {
    static constexpr int A = (DIV == WD_UNIT || DIV == WD_UFMA) ? 4 : DIV == WD_RCP ? 6 : 5;   // WD_MUL / WD_SFMA stream y as d
    static constexpr int AC0 = A - 1;                   // the plane coefficient streams last
    static constexpr int B = GG_TILE_BATCH;
    static constexpr int PBN = B / 2;
    static constexpr int SLOT = A * PBN * 64;           // double2 per ring slot
    static constexpr int NPER = A * PBN;                // DMA instructions per batch
    static constexpr int NG = Wave2D::kTileGran;
    static constexpr int GL = (B * NG + 63) / 64;       // granule loads (stores) per lane per batch
    static constexpr int BND = 2 * PBN * NG;            // boundary values: double2 [2][PBN][NG]
    static constexpr int XST = 2 * PBN * 64;            // x staging: double2 [2][PBN][64]
    static constexpr int RFIT = (150 * 1024 / 16 - BND - XST) / SLOT;
    static constexpr int RVM = 2 + 63 / NPER;
    static constexpr int RING = GG_TILE_RING;
    static constexpr int R = RING < RFIT ? (RING < RVM ? RING : RVM) : (RFIT < RVM ? RFIT : RVM);
    static constexpr int LDS2 = R * SLOT + BND + XST;
    static constexpr int THREADS = 256;
    static_assert(R >= 3 && (R - 2) * NPER <= 63, "ring depth vs vmcnt range");
    static_assert(kTileTAlign % (B * GG_WAVE_POLL) == 0, "steps per tile: whole poll groups of batches");
    static_assert(2 * GL * (GG_WAVE_POLL - 1) <= 63, "boundary wave vmcnt");
    static constexpr int LOOK = kWaveLook < PBN ? kWaveLook : PBN;   // look-ahead pairs
    static_assert(LDS2 * 16 <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ unsigned bfi(unsigned m, unsigned a, unsigned b) { return (a & m) | (b & ~m); }
__device__ __forceinline__ double bfi64(unsigned m, double a, double b)
{
    return __hiloint2double((int)bfi(m, (unsigned)__double2hiint(a), (unsigned)__double2hiint(b)),
                            (int)bfi(m, (unsigned)__double2loint(a), (unsigned)__double2loint(b)));
}
// per-lane masks of the tile layout (all ones / zero)
struct TileMasks {
    unsigned kb;     // the first plane's half-row: plane term from the neighbouring tile
    unsigned r8;     // plane predecessor one row_ror:8 away (Gray bit 0)
    unsigned p16;    // one v_permlane16_swap away (bit 1); else v_permlane32_swap (bit 2)
    unsigned lfix;   // half-row edge lanes whose line term the DPP shift cannot give
};
// one register as both swap operands exchanges rows in place (checked on the
// GPU, tools/permlane_probe.hip): p16 -> rows (x1, x0, x3, x2), p32 -> (x2, x3,
// x0, x1).  The asm carries the VALU-write -> permlane-read wait states itself.
__device__ __forceinline__ unsigned p16_self(unsigned v)
{
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0" : "+v"(v));
    return v;
}
__device__ __forceinline__ unsigned p32_self(unsigned v)
{
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0" : "+v"(v));
    return v;
}
// the plane predecessor's value of x (any lane of the first plane: kb)
__device__ __forceinline__ double plane_move(double x, double kb, const TileMasks &tm)
{
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const unsigned r8l = (unsigned)__builtin_amdgcn_mov_dpp((int)lo, 0x128, 0xf, 0xf, false);   // row_ror:8
    const unsigned r8h = (unsigned)__builtin_amdgcn_mov_dpp((int)hi, 0x128, 0xf, 0xf, false);
    const unsigned l16 = p16_self(lo), h16 = p16_self(hi), l32 = p32_self(lo), h32 = p32_self(hi);
    const unsigned rlo = bfi(tm.r8, r8l, bfi(tm.p16, l16, l32));
    const unsigned rhi = bfi(tm.r8, r8h, bfi(tm.p16, h16, h32));
    return bfi64(tm.kb, kb, __hiloint2double((int)rhi, (int)rlo));
}

// TRACE (diagnostics, gg_trace_precond): per tile 8 + 5 nbatch words -- compute
// wave's start (barrier 0) and end (realtime, 10 ns), workgroup, boundary-wave
// poll retries and cycles spent retrying, realtime after batch 0 and at the
// loader's first issue; then per batch the compute wave's start, the writer's
// publication, the boundary wave's "all values seen", the loader's "landed"
// and the compute wave's end.
// boundary wave: barrier right after the values are in LDS (1), or after the
// re-arm stores and the next polls are issued (0)
#ifndef GG_TILE_EARLYBAR
#define GG_TILE_EARLYBAR 1
#endif
// writer: publish when the compute wave has staged the batch (1) or at the next
// barrier (0); GG_TILE_WSLEEP: s_sleep between its LDS counter polls
#ifndef GG_TILE_DECOUPLE
#define GG_TILE_DECOUPLE 1
#endif
#ifndef GG_TILE_WSLEEP
#define GG_TILE_WSLEEP 1
#endif

template <bool FWD, int DIV, bool TRACE = false>
__global__ __launch_bounds__(256) void k_trsv_tile3d(
    Gate g, int T, int NJ, int NK, const int *__restrict__ order, const double *__restrict__ b,
    const double *__restrict__ c1, const double *__restrict__ c2, const double *__restrict__ dv,
    const double *__restrict__ rv, const double *__restrict__ c0, double *__restrict__ x,
    unsigned long long *gran, int *err, long long *trace, int dyn)
{
    using C = TileCfg<DIV>;
    constexpr int PB = C::PBN * 64;             // double2 per array per slot
    constexpr int NG = C::NG;
    constexpr int GL = C::GL;
    if (gated(g)) return;
    __shared__ double2 lds[C::LDS2];
    __shared__ int xdone;                       // batches the compute wave has staged (this workgroup)
    double2 *bring = lds + C::R * C::SLOT;      // [2][PBN][32]: [0, 16) plane values, [16, 20) line values
    double2 *xbuf = bring + C::BND;             // [2][PBN][64]
    if (threadIdx.x == 0) xdone = 0;            // read only after the first barrier
    int seq = 0;                                // batches this workgroup has run (uniform)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int np = T / 2;
    const int nbatch = T / C::B;                // T is a multiple of kTileTAlign
    const long long TS = 8 + 5LL * nbatch;      // TRACE words per tile
    const int ntask = NJ * NK;
    const long long tgran = (long long)T * NG;  // granules per tile
    // dummy granules of this workgroup (64 zeros to read, 64 write-only words):
    // a line every boundary wave of the chip polled and re-armed would be a
    // hot spot on one memory channel
    unsigned long long *dummy_ld = gran + (long long)ntask * tgran + (long long)blockIdx.x * 128 + lane;
    unsigned long long *dummy_st = dummy_ld + 64;
    // Tiles are dealt statically (dyn = 0: workgroup w takes every
    // gridDim.x-th tile of the dependency order), which needs the whole grid
    // co-resident -- the grid is sized from the occupancy API, which this pool
    // has seen over-promise.  So the boundary wave's waits are
    // bounded by kResidSpin in that mode: a longer wait sets err bit 3 (8) and
    // the workgroup finishes without waiting (garbage, but the grid drains);
    // the host then reruns with dyn = 1 for the triangle's life: tiles CLAIMED
    // in dependency order from a queue (one agent-scope atomic per tile, issued
    // one tile ahead by the compute wave), where a workgroup claims a tile only
    // while it runs and the smallest unfinished tile's owner has finished every
    // tile it claimed before it -- any grid drains, resident or not.  (The
    // queue is the fallback, not the default: C4 L / U 221.6 / 230.1 us static
    // against 242.7 / 257.3 us claimed, profiles/r04/r04_tile_queue_ab.txt.)
    // q[0] = next tile, q[16] = workgroups finished; the last one re-arms both.
    unsigned long long *q = gran + (long long)ntask * tgran + 128LL * kTileDummyBlocks;
    __shared__ int tq[2];                       // the current and the next claimed tile
    if (threadIdx.x == 0) tq[0] = dyn ? (int)atomicAdd(q, 1ull) : (int)blockIdx.x;
    __syncthreads();
    int kq = 0;                                 // tiles this workgroup has run
    for (int task = tq[0]; task < ntask; task = tq[++kq & 1]) {
    const int band = order[FWD ? task : ntask - 1 - task];
    const int J = band % NJ, K = band / NJ;
    const long long boff = (long long)band * np * 64 + lane;     // double2 units
    if (wave == 3) {
        // ------------------------------------------------ loader wave
        const double2 *src[6] = {reinterpret_cast<const double2 *>(b) + boff,
                                 reinterpret_cast<const double2 *>(c1) + boff,
                                 reinterpret_cast<const double2 *>(c2) + boff,
                                 reinterpret_cast<const double2 *>(dv) + boff,
                                 reinterpret_cast<const double2 *>(rv) + boff, nullptr};
        src[C::AC0] = reinterpret_cast<const double2 *>(c0) + boff;
        if (TRACE && lane == 0) trace[(long long)band * TS + 6] = (long long)__builtin_amdgcn_s_memrealtime();
        wave_loader<FWD, C::R, C::SLOT, C::A, C::PBN>(src, lds, np, nbatch,
                                                      TRACE ? trace + (long long)band * TS + 8 + 3 * nbatch : nullptr);
        raw_barrier();                          // final barrier (the writer drains the last batch)
        continue;
    }
    if (wave == 2) {
        // ------------------------------------------------ writer wave
        // Batch bi's edge values as granules, then x, as soon as the compute
        // wave has staged the batch (LDS counter xdone), not at barrier bi+1:
        // that barrier also waits for batch bi+1's boundary values, and a tile's
        // sources must not hold back what it publishes.
        double2 *X2 = reinterpret_cast<double2 *>(x) + boff;
        unsigned long long *gmine = gran + (long long)band * tgran;
        const bool pub_k = FWD ? (K < NK - 1) : (K > 0);
        const bool pub_j = FWD ? (J < NJ - 1) : (J > 0);
        [[maybe_unused]] bool bad = false;
        raw_barrier();                          // barrier 0
        for (int pb = 0; pb < nbatch; pb++) {
            if constexpr (GG_TILE_DECOUPLE) {
                // wait for the compute wave's counter (its x staging precedes it)
                while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&xdone, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)) <= seq + pb)
                    __builtin_amdgcn_s_sleep(GG_TILE_WSLEEP);
            } else {
                raw_barrier();                  // barrier pb+1
            }
            const double2 *xb = xbuf + (pb & 1) * PB;
#pragma unroll
            for (int m = 0; m < GL; m++) {
                const int e = lane + 64 * m;
                const int tt = e / NG, idx = e - tt * NG;
                if (e < C::B * NG && (idx < 8 ? pub_k : pub_j)) {
                    // the last plane's half-row (forward: plane 7, g = 4; backward:
                    // plane 0, g = 0), or plane c's edge lane (a = 7 / a = 0)
                    const int cq = idx - 8;
                    const int sl = idx < 8 ? (FWD ? 32 + idx : idx) : (FWD ? 7 : 0) + 8 * (cq ^ (cq >> 1));
                    const double v = reinterpret_cast<const double *>(xb + (tt >> 1) * 64 + sl)
                        [FWD ? (tt & 1) : 1 - (tt & 1)];
                    const int t = FWD ? pb * C::B + tt : (T - 1) - (pb * C::B + tt);
                    st_agent(gmine + (long long)t * NG + idx, (unsigned long long)__double_as_longlong(v));
                }
            }
            if (TRACE && lane == 0) trace[(long long)band * TS + 8 + nbatch + pb] = (long long)__builtin_amdgcn_s_memrealtime();
            double2 v[C::PBN];
#pragma unroll
            for (int kk = 0; kk < C::PBN; kk++) v[kk] = xb[kk * 64 + lane];
#pragma unroll
            for (int kk = 0; kk < C::PBN; kk++) {
                const int p = pb * C::PBN + kk;
                X2[(long long)(FWD ? p : np - 1 - p) * 64] = v[kk];
                if constexpr (DIV == WD_RCP) bad |= !rcp_safe(v[kk].x) || !rcp_safe(v[kk].y);
            }
            if constexpr (GG_TILE_DECOUPLE) raw_barrier();   // barrier pb+1 (the last: the task's final one)
        }
        seq += nbatch;
        if constexpr (DIV == WD_RCP) {
            if (__any(bad) && lane == 0) atomicOr(err, 2);
        }
        continue;
    }
    if (wave == 1) {
        // ------------------------------------------------ boundary wave
        // Before barrier bi it places batch bi's boundary values in bring[bi & 1]:
        // entry e = lane + 64 m of the batch is (step tt = e / NG, index e % NG).
        // Polls run kPoll batches deep (GL loads per batch); every lane issues
        // every load and store (unused ones on the dummy granules), which keeps
        // the vmcnt arithmetic exact.
        constexpr int kPoll = GG_WAVE_POLL;
        const bool has_k = FWD ? (K > 0) : (K < NK - 1);
        const bool has_j = FWD ? (J > 0) : (J < NJ - 1);
        unsigned long long *gk = has_k ? gran + (long long)(FWD ? band - NJ : band + NJ) * tgran : gran;
        unsigned long long *gj = has_j ? gran + (long long)(FWD ? band - 1 : band + 1) * tgran : gran;
        auto gaddr = [&](int bj, int m) -> unsigned long long * {
            const int e = lane + 64 * m;
            const int tt = e / NG, idx = e - tt * NG;
            if (e >= C::B * NG || bj >= nbatch) return nullptr;
            const int t = FWD ? bj * C::B + tt : (T - 1) - (bj * C::B + tt);
            const bool pl = idx < 8;
            const int tp = FWD ? t + 7 : t - 7;
            if (!(pl ? has_k : has_j) || tp < 0 || tp >= T) return nullptr;
            return (pl ? gk : gj) + (long long)tp * NG + idx;
        };
        auto paddr = [&](int bj, int m) {
            unsigned long long *a = gaddr(bj, m);
            return a ? a : dummy_ld;
        };
        unsigned long long v[kPoll][GL];
#pragma unroll
        for (int u = 0; u < kPoll; u++) {
            if (u > 0) {
#pragma unroll
                for (int m = 0; m < GL; m++) st_agent(dummy_st, kSentinel);
            }
#pragma unroll
            for (int m = 0; m < GL; m++) v[u][m] = ld_agent(paddr(u, m));
        }
        bool dead = false;
        long long bw_spins = 0, bw_cyc = 0;     // TRACE
        for (int bi0 = 0; bi0 < nbatch; bi0 += kPoll) {     // nbatch is a multiple of kPoll
#pragma unroll
            for (int u = 0; u < kPoll; u++) {
                const int bi = bi0 + u;
                // this batch's polls done: after them come kPoll-1 batches of
                // GL re-arm stores and GL loads
                __builtin_amdgcn_s_waitcnt(vm_wait(2 * GL * (kPoll - 1)));
                int spins = 0;
                const long long tw = TRACE ? (long long)__builtin_amdgcn_s_memtime() : 0;
                auto ready = [&]() {
                    bool r = true;
#pragma unroll
                    for (int m = 0; m < GL; m++) r = r && v[u][m] != kSentinel;
                    return r;
                };
                if constexpr (GG_TILE_POLL2) {
                    // not ready: two poll generations in flight, staggered, so a
                    // value that lands is seen within about half a round trip
                    // (every load completes in order: vm_wait(GL) = the older
                    // generation is back)
                    if (!__all(ready())) {
                        unsigned long long pa[GL], pb2[GL];
#pragma unroll
                        for (int m = 0; m < GL; m++) pa[m] = ld_agent(paddr(bi, m));
                        __builtin_amdgcn_s_sleep(GG_TILE_POLL2);
#pragma unroll
                        for (int m = 0; m < GL; m++) pb2[m] = ld_agent(paddr(bi, m));
                        auto rdy = [&](const unsigned long long *q) {
                            bool r = true;
#pragma unroll
                            for (int m = 0; m < GL; m++) r = r && q[m] != kSentinel;
                            return r;
                        };
                        while (true) {
                            __builtin_amdgcn_s_waitcnt(vm_wait(GL));
                            if (dead || __all(rdy(pa))) {
#pragma unroll
                                for (int m = 0; m < GL; m++) v[u][m] = pa[m];
                                break;
                            }
#pragma unroll
                            for (int m = 0; m < GL; m++) pa[m] = ld_agent(paddr(bi, m));
                            __builtin_amdgcn_s_waitcnt(vm_wait(GL));
                            if (__all(rdy(pb2))) {
#pragma unroll
                                for (int m = 0; m < GL; m++) v[u][m] = pb2[m];
                                break;
                            }
#pragma unroll
                            for (int m = 0; m < GL; m++) pb2[m] = ld_agent(paddr(bi, m));
                            spins += 2;
                            if (spins > kSpinLimit) {
                                dead = true;
                                if (lane == 0) atomicOr(err, 1);
                            }
                        }
                        __builtin_amdgcn_s_waitcnt(vm_wait(0));   // the other generation
                    }
                } else {
                    while (!dead && !__all(ready())) {
                        __builtin_amdgcn_s_sleep(1);
#pragma unroll
                        for (int m = 0; m < GL; m++) v[u][m] = ld_agent(paddr(bi, m));
                        if (++spins > (dyn ? kSpinLimit : kResidSpin)) {
                            dead = true;
                            if (lane == 0) atomicOr(err, dyn ? 1 : 8);   // 8: static grid not resident
                        }
                        __builtin_amdgcn_s_waitcnt(vm_wait(0));
                    }
                }
                if constexpr (TRACE) {
                    bw_spins += spins;
                    if (spins) bw_cyc += (long long)__builtin_amdgcn_s_memtime() - tw;
                    if (lane == 0) trace[(long long)band * TS + 8 + 2 * nbatch + bi] = (long long)__builtin_amdgcn_s_memrealtime();
                }
                double *bd = reinterpret_cast<double *>(bring + (bi & 1) * (C::PBN * NG));
#pragma unroll
                for (int m = 0; m < GL; m++) {
                    const int e = lane + 64 * m;
                    const int tt = e / NG, idx = e - tt * NG;
                    if (e < C::B * NG) bd[((tt >> 1) * NG + idx) * 2 + (tt & 1)] = __longlong_as_double((long long)v[u][m]);
                }
                if constexpr (GG_TILE_EARLYBAR) {
                    // hand the values over first, then re-arm and poll ahead
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    raw_barrier();
                }
#pragma unroll
                for (int m = 0; m < GL; m++) {
                    unsigned long long *ga = gaddr(bi, m);
                    st_agent(ga ? ga : dummy_st, kSentinel);     // re-arm for the next launch
                }
#pragma unroll
                for (int m = 0; m < GL; m++) v[u][m] = ld_agent(paddr(bi + kPoll, m));
                if constexpr (!GG_TILE_EARLYBAR) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    raw_barrier();
                }
            }
        }
        raw_barrier();                      // final barrier (the writer drains the last batch)
        if (TRACE && lane == 0) {
            trace[(long long)band * TS + 3] = bw_spins;
            trace[(long long)band * TS + 4] = bw_cyc;
        }
        continue;
    }

    // ---------------------------------------------------- compute wave
    constexpr int ctrl = FWD ? 0x111 : 0x101;   // row_shr:1 / row_shl:1
    const int la = lane & 7, hr = lane >> 3;
    const int cp = hr ^ (hr >> 1) ^ (hr >> 2);  // this lane's plane (inverse Gray code)
    const int cs = FWD ? cp : cp + 1;           // the plane whose predecessor move applies
    const TileMasks tm{(FWD ? cp == 0 : cp == 7) ? ~0u : 0u, (cs & 1) ? ~0u : 0u, (cs & 3) == 2 ? ~0u : 0u,
                       (lane & 15) == (FWD ? 8 : 7) ? ~0u : 0u};
    double xp = 0.0;                        // this lane's value of the previous step
    double2 rg[C::PBN][C::A];
    raw_barrier();                          // barrier 0: batch 0 is in LDS
    // the next tile, claimed now (its latency hides in this tile's batches)
    // and handed to every wave through LDS before the task's final barrier
    int next_task = 0;
    if (lane == 0) next_task = dyn ? (int)atomicAdd(q, 1ull) : task + (int)gridDim.x;
    if (TRACE && lane == 0) {
        trace[(long long)band * TS + 0] = (long long)__builtin_amdgcn_s_memrealtime();
        trace[(long long)band * TS + 2] = blockIdx.x;
    }
    for (int bi = 0; bi < nbatch; bi++) {
        // the first step's plane neighbour (the previous step) is moved before
        // the barrier; only the first plane's row waits for the boundary value
        const double xzp = plane_move(xp, 0.0, tm);
        if (bi > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // x staging of batch bi-1 written
            raw_barrier();                  // batch bi's data and boundary values
            if (TRACE && bi == 1 && lane == 0) trace[(long long)band * TS + 5] = (long long)__builtin_amdgcn_s_memrealtime();
        }
        if (TRACE && lane == 0) trace[(long long)band * TS + 8 + bi] = (long long)__builtin_amdgcn_s_memrealtime();
        const double2 *br = bring + (bi & 1) * (C::PBN * NG);
        const double2 *sc = lds + (bi % C::R) * C::SLOT + lane;
        double2 bk[C::PBN], bj[C::PBN];     // plane / line boundary values of each step pair
        bk[0] = br[la];
        bj[0] = br[8 + cp];
#pragma unroll
        for (int a = 0; a < C::A; a++) rg[0][a] = sc[a * PB];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 1; kk < C::LOOK; kk++)
#pragma unroll
            for (int a = 0; a < C::A; a++) rg[kk][a] = sc[a * PB + kk * 64];
#pragma unroll
        for (int kk = 1; kk < C::PBN; kk++) {
            bk[kk] = br[kk * NG + la];
            bj[kk] = br[kk * NG + 8 + cp];
        }
        __builtin_amdgcn_sched_barrier(0);
        double xv[C::B];
        // the plane neighbour's value for the batch's first step
        const double xz0 = bfi64(tm.kb, bk[0].x, xzp);
#pragma unroll
        for (int kk = 0; kk < C::PBN; kk++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int tt = 2 * kk + h;
                const bool sx = FWD ? (h == 0) : (h == 1);     // even storage step <-> .x
                const double bb = sx ? rg[kk][0].x : rg[kk][0].y;
                const double e1 = sx ? rg[kk][1].x : rg[kk][1].y;
                const double e2 = sx ? rg[kk][2].x : rg[kk][2].y;
                const double e0 = sx ? rg[kk][C::AC0].x : rg[kk][C::AC0].y;
                const double oj = h ? bj[kk].y : bj[kk].x;      // boundary entries by sweep step
                // the plane neighbour: the predecessor plane's value of the previous step
                const double xz = tt == 0 ? xz0 : plane_move(xp, h ? bk[kk].y : bk[kk].x, tm);
                const double p2 = (DIV == WD_UFMA || DIV == WD_SFMA) ? 0.0 : e2 * xp;
                const double xs = bfi64(tm.lfix, oj, dpp_shift_old<ctrl>(xp, oj));
                if constexpr (kWaveShadow) {
                    __builtin_amdgcn_sched_barrier(0);
                    if (h == 0 && kk + C::LOOK < C::PBN) {
#pragma unroll
                        for (int a = 0; a < C::A; a++) rg[kk + C::LOOK][a] = sc[a * PB + (kk + C::LOOK) * 64];
                    }
                    if (h == 1 && kk > 0) {
                        xbuf[(bi & 1) * PB + (kk - 1) * 64 + lane] =
                            FWD ? make_double2(xv[2 * kk - 2], xv[2 * kk - 1])
                                : make_double2(xv[2 * kk - 1], xv[2 * kk - 2]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                // canonical order: plane term, line term, in-line term;
                // GG_DIV_FMA: nearest first, fused (in-line, line, plane: the
                // order the operands arrive in), b pre-scaled for U
                double acc;
                if constexpr (DIV == WD_UFMA || DIV == WD_SFMA) {
                    double by = bb;
                    if constexpr (DIV == WD_SFMA) by = bb * (sx ? rg[kk][3].x : rg[kk][3].y);
                    acc = __builtin_fma(-e2, xp, by);
                    acc = __builtin_fma(-e1, xs, acc);
                    acc = __builtin_fma(-e0, xz, acc);
                } else {
                    acc = bb - e0 * xz;
                    acc = acc - e1 * xs;
                    acc = acc - p2;
                }
                if constexpr (DIV == WD_HW) {
                    acc = acc / (sx ? rg[kk][3].x : rg[kk][3].y);
                } else if constexpr (DIV == WD_MUL) {
                    acc = acc * (sx ? rg[kk][3].x : rg[kk][3].y);
                } else if constexpr (DIV == WD_RCP) {
                    const double d = sx ? rg[kk][3].x : rg[kk][3].y;
                    const double y = sx ? rg[kk][4].x : rg[kk][4].y;
                    const double q0 = acc * y;
                    const double q1 = __builtin_fma(-__builtin_fma(q0, d, -acc), y, q0);
                    acc = __builtin_fma(-__builtin_fma(q1, d, -acc), y, q1);
                }
                xp = acc;
                xv[tt] = acc;
            }
            if (!kWaveShadow || kk == C::PBN - 1)
                xbuf[(bi & 1) * PB + kk * 64 + lane] =
                    FWD ? make_double2(xv[2 * kk], xv[2 * kk + 1]) : make_double2(xv[2 * kk + 1], xv[2 * kk]);
            if (!kWaveShadow && kk + C::LOOK < C::PBN) {
#pragma unroll
                for (int a = 0; a < C::A; a++) rg[kk + C::LOOK][a] = sc[a * PB + (kk + C::LOOK) * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // the batch's x staging, then the writer's counter
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (TRACE && lane == 0) trace[(long long)band * TS + 8 + 4 * nbatch + bi] = (long long)__builtin_amdgcn_s_memrealtime();
        if (GG_TILE_DECOUPLE && lane == 0)
            __hip_atomic_store(&xdone, seq + bi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    seq += nbatch;
    if (lane == 0) tq[(kq + 1) & 1] = next_task;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                          // final barrier: the writer drains the last batch
    if (TRACE && lane == 0) trace[(long long)band * TS + 1] = (long long)__builtin_amdgcn_s_memrealtime();
    }   // task loop
    // every claim of this workgroup has returned: count it out; the last
    // workgroup re-arms the queue (the next launch follows a kernel boundary)
    if (dyn && threadIdx.x == 0) {
        if (atomicAdd(q + 16, 1ull) == (unsigned long long)gridDim.x - 1) {
            st_agent(q, 0ull);
            st_agent(q + 16, 0ull);
        }
    }
}

// ================================================ ILU(0) factorization (device)
// leftILU's column elimination (src/leftILU.cu:27-336: cpuSequentialTriSolve
// :769-825 per column, columns in generateLevel :339-368 order) as a dataflow
// kernel.  Lane = column c; a wave takes 64 consecutive columns, the grid
// strides over the columns in ascending order (all blocks co-resident, so the
// smallest unfinished column can always progress).  Per column:
//  1. its level: max(level[r] + 1) over the rows r < c of its U part whose
//     ORIGINAL value is not |a| < 1e-9 (generateLevel), published in level[c];
//  2. the serial order of the reference processes columns by (level, index),
//     so a source column r < c (a U-part row of c) was finished before c iff
//     level[r] <= level[c]: then wait for done[r] and read r's factored
//     values, otherwise read r's ORIGINAL values (r had not been processed);
//  3. the column update in the reference's order (ascending U-part rows, then
//     the L part divided by the diagonal, 0 when |diag| < 1e-9), written with
//     agent-scope stores, drained, then done[c] published.
// Lanes of one wave can depend on each other, so every lane retries inside a
// wave-uniform loop instead of spinning alone.  Spins are bounded (err bit 0).
__device__ __forceinline__ int ld_agent_i(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_i(int *p, int v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent_d(const double *p)
{
    return __longlong_as_double((long long)ld_agent(reinterpret_cast<const unsigned long long *>(p)));
}
__device__ __forceinline__ void st_agent_d(double *p, double v)
{
    st_agent(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v));
}
__device__ __forceinline__ bool ilu_zero(double a) { return __builtin_fabs(a) < 1e-9; }   // Equal(a, 0)

__global__ __launch_bounds__(kBlock) void k_ilu0_columns(int n, const int *__restrict__ cp,
                                                         const int *__restrict__ ri,
                                                         const double *__restrict__ cv0, double *cv,
                                                         int *level, int *done, int *err)
{
    const int lane = threadIdx.x & 63;
    const long long wid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long nw = (gridDim.x * (long long)blockDim.x) >> 6;
    for (long long base = wid * 64; base < n; base += nw * 64) {
        const int c = (int)(base + lane);
        int state = c < n ? 0 : 2;             // 0: level, 1: factor, 2: finished
        int lev = 0;
        int spins = 0;
        const int lb = c < n ? cp[c] : 0, ub = c < n ? cp[c + 1] : 0;
        while (__any(state != 2)) {
            bool moved = false;
            if (state == 0) {
                bool ready = true;
                int l = 0;
                for (int k = lb; k < ub; k++) {
                    const int r = ri[k];
                    if (r >= c) break;
                    const int lr = ld_agent_i(level + r);
                    if (lr < 0) { ready = false; break; }
                    if (!ilu_zero(cv0[k]) && lr + 1 > l) l = lr + 1;
                }
                if (ready) {
                    lev = l;
                    st_agent_i(level + c, l);
                    state = 1;
                    moved = true;
                }
            }
            if (state == 1) {
                bool ready = true;
                for (int k = lb; k < ub; k++) {
                    const int r = ri[k];
                    if (r >= c) break;
                    if (ld_agent_i(level + r) <= lev && ld_agent_i(done + r) == 0) { ready = false; break; }
                }
                if (ready) {
                    double u_diag = 0.0;
                    for (int k = lb; k < ub - 1; k++) {
                        const int cr = ri[k];
                        if (cr > c) break;
                        if (cr == c) { u_diag = ld_agent_d(cv + k); break; }
                        const bool fin = ld_agent_i(level + cr) <= lev;
                        int q = cp[cr];
                        const int qe = cp[cr + 1];
                        const double ukt = ld_agent_d(cv + k);
                        for (int p = k + 1; p < ub; p++) {
                            const int r2 = ri[p];
                            while (q < qe && ri[q] < r2) q++;
                            if (q == qe) break;
                            if (ri[q] == r2) {
                                const double lq = fin ? ld_agent_d(cv + q) : cv0[q];
                                st_agent_d(cv + p, ld_agent_d(cv + p) - lq * ukt);
                            }
                        }
                    }
                    for (int k = lb; k < ub; k++) {
                        if (ri[k] <= c) continue;
                        st_agent_d(cv + k, ilu_zero(u_diag) ? 0.0 : ld_agent_d(cv + k) / u_diag);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // values out before the flag
                    st_agent_i(done + c, 1);
                    state = 2;
                    moved = true;
                }
            }
            if (!moved && state != 2) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > kSpinLimit) {
                    atomicOr(err, 1);
                    state = 2;
                }
            }
        }
    }
}

// ILU(k) numeric factorization (ilukC, src/iluk.cpp:108-188) on lofC's pattern
// (host, iluk_pattern): row i = prow[i] .. prow[i+1], every row ascending (its
// nl[i] L entries, the diagonal, its U part).  One WAVE per row; a row's pivots
// (its L entries) are taken one after the other in ascending column order --
// the order ilukC applies them, so every entry sees the same updates in the
// same order and the factors are bit-identical:
//   wait done[k]; l = val[t] * Dinv[k]; for the U entries (k, c) of row k, in
//   parallel over the lanes: if c is in row i's pattern, val[i, c] -= l * u
// then Dinv[i] = 1 / val[diag] (err bit 2 on a zero pivot, src/iluk.cpp:175-185),
// the row's values stored write-through, drained, done[i] published.
// Ordinary rows (<= kIlukCap entries) are staged in the wave's LDS (columns
// and values; a column is found by binary search above the pivot's position);
// longer rows (the hub rows of circuit matrices) keep their values in HBM and
// find columns through a dense column -> position map of their own (scratch,
// n ints per long-row wave, -1 outside the row).  Rows are split into the two
// lists (ascending); the first `long_blocks` blocks take the long list, the
// rest the short one, each wave its list's rows in ascending order: with every
// block co-resident the smallest unfinished row always progresses.  Spins are
// bounded (err bit 0).
constexpr int kIlukCap = 3200;
__device__ __forceinline__ int lds_bsearch(const int *a, int lo, int hi, int c)
{
    const int end = hi;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    return (lo < end && a[lo] == c) ? lo : -1;
}

__global__ __launch_bounds__(kBlock) void k_iluk_wave(int n, const long long *__restrict__ prow,
                                                      const int *__restrict__ nl,
                                                      const int *__restrict__ pcol, double *val,
                                                      double *dinv, int *done,
                                                      const int *__restrict__ rows_short, int nshort,
                                                      const int *__restrict__ rows_long, int nlong,
                                                      int long_blocks, int *scratch, int *err)
{
    __shared__ int scol[kBlock / 64][kIlukCap];
    __shared__ double sval[kBlock / 64][kIlukCap];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool lng = (int)blockIdx.x < long_blocks;
    const int gw = (lng ? (int)blockIdx.x : (int)blockIdx.x - long_blocks) * (kBlock / 64) + w;
    const int nw = (lng ? long_blocks : (int)gridDim.x - long_blocks) * (kBlock / 64);
    const int cnt = lng ? nlong : nshort;
    const int *rows = lng ? rows_long : rows_short;
    int *jw = lng ? scratch + (long long)gw * n : nullptr;
    int *sc = scol[w];
    double *sv = sval[w];
    bool dead = false;
    for (int q = gw; q < cnt && !dead; q += nw) {
        const int i = rows[q];
        const long long p0 = prow[i];
        const int len = (int)(prow[i + 1] - p0), nli = nl[i];
        if (!lng) {
            for (int t = lane; t < len; t += 64) {
                sc[t] = pcol[p0 + t];
                sv[t] = val[p0 + t];
            }
        } else {
            for (int t = lane; t < len; t += 64) __hip_atomic_store(jw + pcol[p0 + t], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        for (int j = 0; j < nli && !dead; j++) {
            const int k = lng ? pcol[p0 + j] : sc[j];
            int spins = 0;
            while (__builtin_amdgcn_readfirstlane(ld_agent_i(done + k)) == 0) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > kSpinLimit) {
                    if (lane == 0) atomicOr(err, 1);
                    dead = true;
                    break;
                }
            }
            const double l = (lng ? ld_agent_d(val + p0 + j) : sv[j]) * ld_agent_d(dinv + k);
            if (lane == 0) {
                if (lng) st_agent_d(val + p0 + j, l);
                else sv[j] = l;
            }
            const long long u0 = prow[k] + nl[k] + 1, u1 = prow[k + 1];
            for (long long e = u0 + lane; e < u1; e += 64) {
                const int c = pcol[e];
                const double u = ld_agent_d(val + e);
                if (lng) {
                    const int pos = __hip_atomic_load(jw + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (pos >= 0) st_agent_d(val + p0 + pos, ld_agent_d(val + p0 + pos) - l * u);
                } else {
                    const int pos = lds_bsearch(sc, j + 1, len, c);
                    if (pos >= 0) sv[pos] = sv[pos] - l * u;
                }
            }
            if (lng) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const double dg = lng ? ld_agent_d(val + p0 + nli) : sv[nli];
        if (!lng)
            for (int t = lane; t < len; t += 64) st_agent_d(val + p0 + t, sv[t]);
        if (lane == 0) {
            if (dg == 0.0) atomicOr(err, 2);
            st_agent_d(dinv + i, 1.0 / dg);
        }
        if (lng)
            for (int t = lane; t < len; t += 64) __hip_atomic_store(jw + pcol[p0 + t], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the row's values out before the flag
        if (lane == 0) st_agent_i(done + i, 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // LDS reads done before the next row's staging
    }
}

// A's values into the ILU(k) pattern (val pre-zeroed), ilukC's initial
// scatter (src/iluk.cpp:120-133): one thread per row, entries in CSR order (a
// repeated column keeps its last value, as the reference's assignment does),
// each position found by binary search in the row's ascending columns
__global__ __launch_bounds__(kBlock) void k_iluk_scatter(int n, const int *__restrict__ arp,
                                                         const int *__restrict__ aci,
                                                         const double *__restrict__ av,
                                                         const long long *__restrict__ prow,
                                                         const int *__restrict__ pcol, double *val)
{
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const long long p0 = prow[i], p1 = prow[i + 1];
        for (int e = arp[i]; e < arp[i + 1]; e++) {
            const int c = aci[e];
            long long lo = p0, hi = p1;
            while (lo < hi) {
                const long long mid = (lo + hi) >> 1;
                if (pcol[mid] < c) lo = mid + 1;
                else hi = mid;
            }
            val[lo] = av[e];                     // every entry of A is in its row's pattern
        }
    }
}

// ================================================== transient step (C5)
// PULSE source values at time index it (gen_PULSEut_kernel, src/kernels.cu:223-245);
// pulse[k] = {vlo, vhi, td, tr, tf, tw, tp}
// Source values at time index it, t = it * h (mytime = idxt * tstep), one
// thread per source, kind[k] / data[dptr[k] .. dptr[k+1]):
//   GG_SRC_DC     {value}                              gen_dcVt_kernel   src/kernels.cu:73-85
//   GG_SRC_PULSE  {vlo, vhi, td, tr, tf, tw, tp}       gen_PULSEut_kernel src/kernels.cu:223-245
//   GG_SRC_PWL    {t0, v0, t1, v1, ...}                gen_PWLut_kernel  src/kernels.cu:146-176
// (PWL before t0: v0; the reference reads v[-1] there)
__device__ __forceinline__ double pulse_value(const double *q, double t)
{
    const double vlo = q[0], vhi = q[1], td = q[2], tr = q[3], tf = q[4], tw = q[5], tp = q[6];
    t = t - floor(t / tp) * tp;
    if (t < td) return vlo;
    if (t < td + tr) return vlo + (t - td) * (vhi - vlo) / tr;
    if (t < td + tr + tw) return vhi;
    if (t < td + tr + tw + tf) return vhi - (t - td - tr - tw) * (vhi - vlo) / tf;
    return vlo;
}
__device__ __forceinline__ double pwl_value(const double *tv, int np, double t)
{
    if (np <= 0) return 0.0;
    double value = tv[1];
    int i;
    for (i = 0; i < np; i++) {
        if (t < tv[2 * i]) {
            if (i > 0)
                value = tv[2 * i + 1] - (tv[2 * i] - t) * (tv[2 * i + 1] - tv[2 * i - 1]) /
                                            (tv[2 * i] - tv[2 * i - 2]);
            break;
        }
    }
    if (i == np) value = tv[2 * np - 1];
    return value;
}
__global__ void k_sources(int nsrc, const int *kind, const int *dptr, const double *data, int it, double h,
                          double *u)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nsrc) return;
    const double *q = data + dptr[k];
    const double t = it * h;
    double value = 0.0;
    if (kind[k] == GG_SRC_DC) value = q[0];
    else if (kind[k] == GG_SRC_PULSE) value = pulse_value(q, t);
    else value = pwl_value(q, (dptr[k + 1] - dptr[k]) / 2, t);
    u[k] = value;
}

// w = B u + (C/h) x_prev as the reference step driver forms it
// (src/mna_solve_gpu_gmres.cpp:585-591): w = 0; w += B u (cs_dl_gaxpy, sources
// of a row in column order); xnr = 0; xnr += (C/h) x; w += xnr.  B is an
// incidence matrix (+1 per source), C/h diagonal.
__global__ void k_transient_rhs(int n, const int *src_ptr, const int *src_idx, const double *u,
                                const double *cdiag, const double *x, double *w)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    double bu = 0.0;
    for (int q = src_ptr[r]; q < src_ptr[r + 1]; q++) bu = bu + 1.0 * u[src_idx[q]];
    double xnr = 0.0;
    xnr = xnr + cdiag[r] * x[r];
    w[r] = bu + xnr;
}

// w = B u + R x_prev for a general MNA system (gg_transient_mna, the
// wrapperGMRESforPG path): B (n x nsrc) and R = C/h (n x n, capacitor stamps
// between nodes included) in CSR.  cs_dl_gaxpy (y += A x, column by column)
// accumulates each row in ascending column order from 0.0, which is the CSR
// row order here: bu = B u, xnr = R x, w = bu + xnr (the driver's w += xnr).
__global__ void k_transient_rhs_csr(int n, const int *bp, const int *bi, const double *bv, const double *u,
                                    const int *rp, const int *ri, const double *rv, const double *x,
                                    double *w)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    double bu = 0.0;
    for (int q = bp[r]; q < bp[r + 1]; q++) bu = bu + bv[q] * u[bi[q]];
    double xnr = 0.0;
    for (int q = rp[r]; q < rp[r + 1]; q++) xnr = xnr + rv[q] * x[ri[q]];
    w[r] = bu + xnr;
}

// tap-node voltage statistics of the transient run (the ir_info block of the
// step driver, src/mna_solve_gpu_gmres.cpp:285-292, 633-645, 780-797): max,
// min and the running sum, seeded with the initial state; avg = sum / time
// points, IR = max - min at the end
__global__ void k_taps(int ntap, const int *tap, const double *x, double *mx, double *mn, double *sm, int mode,
                       double npts)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ntap) return;
    if (mode == 2) {                       // finish: sum -> avg (IR = max - min on the host)
        sm[j] = sm[j] / npts;
        return;
    }
    const double v = x[tap[j]];
    if (mode == 0) {
        mx[j] = v;
        mn[j] = v;
        sm[j] = v;
        return;
    }
    if (mx[j] < v) mx[j] = v;
    if (v < mn[j]) mn[j] = v;
    sm[j] += v;
}

__global__ void k_gather_ports(int nport, const int *port, const double *x, double *out)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nport) out[j] = x[port[j]];
}

// ---- batched (many-RHS) helpers: blockIdx.y = scenario ----------------------
// out_sc[i] = idx[i] < 0 ? 0 : in_sc[idx[i]], in / out strides zin / zout bytes
__global__ void k_gather_b(const double *in, long long zin, const long long *idx, double *out, long long zout,
                           long long n)
{
    in = zp(in, zin, blockIdx.y);
    out = zp(out, zout, blockIdx.y);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const long long s = idx[i];
        out[i] = s < 0 ? 0.0 : in[s];
    }
}
// every scenario's control block at the start of a solve (as the host writes
// the single solver's)
__global__ void k_init_state_b(DevState *ds, long long zs, int nsc, double tol, int max_iter, int m)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nsc) return;
    DevState h{};
    h.tol = tol;
    h.max_iter = max_iter;
    h.m = m;
    h.j = 1;
    *zp(ds, zs, q) = h;
}
// the scenarios' control blocks side by side (one copy to the host per cycle)
__global__ void k_pack_states_b(const DevState *ds, long long zs, int nsc, DevState *out, const int *err)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nsc) out[q] = *zp(ds, zs, q);
    if (q == nsc) out[nsc].err = *err;          // the error word after every launch before this one
}
// transient step of every scenario: u_sc = its sources at time index it; w_sc
// = B_sc u_sc + (C/h) x_sc (k_sources + k_transient_rhs per scenario; tables
// concatenated, scenario sc's sources [soff[sc], soff[sc+1]) and its B^T rows
// at sptr + sc * (n + 1); x and w natural order, stride ldx doubles)
__global__ void k_sources_b(const int *soff, const int *kind, const int *dptr, const double *data, int it,
                            double h, double *u)
{
    const int q = blockIdx.y;
    const int k = soff[q] + blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= soff[q + 1]) return;
    const double *d = data + dptr[k];
    const double t = it * h;
    double value = 0.0;
    if (kind[k] == GG_SRC_DC) value = d[0];
    else if (kind[k] == GG_SRC_PULSE) value = pulse_value(d, t);
    else value = pwl_value(d, (dptr[k + 1] - dptr[k]) / 2, t);
    u[k] = value;
}
__global__ void k_transient_rhs_b(int n, const int *sptr, const int *sidx, const double *u, const double *cdiag,
                                  const double *x, double *w, long long ldx)
{
    const int q = blockIdx.y;
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int *sp = sptr + (long long)q * (n + 1);
    double bu = 0.0;
    for (int k = sp[r]; k < sp[r + 1]; k++) bu = bu + 1.0 * u[sidx[k]];
    double xnr = 0.0;
    xnr = xnr + cdiag[r] * x[(long long)q * ldx + r];
    w[(long long)q * ldx + r] = bu + xnr;
}
__global__ void k_gather_ports_b(int nport, const int *port, const double *x, long long ldx, double *out,
                                 long long ldo)
{
    const int q = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nport) out[(long long)q * ldo + j] = x[(long long)q * ldx + port[j]];
}

// ============================================================ GMRES kernels
__global__ void k_set_normb(const double *part, int G, DevState *ds, long long zs = 0)
{
    part = zp(part, zs, blockIdx.y);
    ds = zp(ds, zs, blockIdx.y);
    double s = sum_partials(part, G);
    if (threadIdx.x == 0) {
        double nb = sqrt(s);
        ds->normb = (nb == 0.0) ? 1.0 : nb;     // src/gmres.cu:604
    }
}

__global__ void k_init_beta(const double *part, int G, DevState *ds, double *hist, long long zs = 0)
{
    part = zp(part, zs, blockIdx.y);
    ds = zp(ds, zs, blockIdx.y);
    hist = zp(hist, zs, blockIdx.y);
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
                                                       double *s, long long units, long long zs = 0)
{
    ds = zp(ds, zs, blockIdx.y);
    r = zp(r, zs, blockIdx.y);
    v0 = zp(v0, zs, blockIdx.y);
    s = zp(s, zs, blockIdx.y);
    if (ds->done) return;
    if (ds->max_iter - ds->j + 1 <= 0) {   // a cycle past max_iter (pipelined): nothing runs
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ds->nit = 0;
            ds->done |= DONE_EXH;
        }
        return;
    }
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
// Each thread owns units u = g*256 + t + j*G*256 (j = 0, 1, ...), accumulated in
// ascending j (the oracle's blocked dot order); kUnroll of them are loaded
// before any is used so a thread keeps several 16-B loads per stream in flight.
constexpr int kUnroll = 4;

template <bool NORM>
__global__ __launch_bounds__(kBlock) void k_mgs_step(Gate g, int i, int k, int m,
                                                     double *__restrict__ w,
                                                     const double *__restrict__ vk,
                                                     const double *__restrict__ vnext,
                                                     const double *part_in, double *part_out,
                                                     double *H, int G, long long units,
                                                     long long dunits, long long zs = 0)
{
    // the AXPY runs over [0, units); the next dot accumulates over [0, dunits)
    // (dunits < units on the shards of a sharded solve that do not own the
    // separator replica); part_in holds G partials (all shards' in that case)
    if (gated_z(g, zs, blockIdx.y)) return;
    if (zs) {
        const int sc = blockIdx.y;
        w = zp(w, zs, sc);
        vk = zp(vk, zs, sc);
        vnext = zp(vnext, zs, sc);
        part_in = zp(part_in, zs, sc);
        part_out = zp(part_out, zs, sc);
        H = zp(H, zs, sc);
    }
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    long long u0 = blockIdx.x * (long long)kBlock + threadIdx.x;
    double2 wv[kUnroll], vv[kUnroll], nv[kUnroll];
    auto load = [&]() {
#pragma unroll
        for (int j = 0; j < kUnroll; j++) {
            const long long u = u0 + j * stride;
            if (u < units) {
                wv[j] = ld2(w, u);          // w: re-read every step, kept in the caches
                vv[j] = ld2_nt(vk, u);      // the basis vectors are streamed
                if (!NORM) nv[j] = ld2_nt(vnext, u);
            }
        }
    };
    load();                 // the first chunk is in flight while h is summed
    const double h = sum_partials(part_in, G);
    if (blockIdx.x == 0 && threadIdx.x == 0) H[k + i * (m + 1)] = h;
    const double a = -h;
    while (u0 < units) {
#pragma unroll
        for (int j = 0; j < kUnroll; j++) {
            const long long u = u0 + j * stride;
            if (u < units) {
                wv[j].x = a * vv[j].x + wv[j].x;
                wv[j].y = a * vv[j].y + wv[j].y;
                st2(w, u, wv[j]);
                if (NORM) nv[j] = wv[j];
                if (u < dunits) {
                    acc += wv[j].x * nv[j].x;
                    acc += wv[j].y * nv[j].y;
                }
            }
        }
        u0 += kUnroll * stride;
        load();
    }
    acc = block_sum(acc);
    if (threadIdx.x == 0) part_out[blockIdx.x] = acc;
}

// ---- CGS2 (the sharded solve's GG_SOLVE_CGS2): classical Gram-Schmidt with
// one re-orthogonalization, h = V^T w; w -= V h; h2 = V^T w; w -= V h2;
// H[:, i] = h + h2 -- three all-gathers per inner iteration (h, h2, ||w||)
// instead of MGS's i + 2.  Every dot keeps k_dot's tree (thread t of block b:
// units b*256 + t + j*G*256 ascending, block_sum), so the oracle restates it
// bit for bit (orc_set_orth).
__global__ __launch_bounds__(kBlock) void k_multidot(Gate g, const double *__restrict__ w,
                                                     const double *__restrict__ V, long long ldv, int nk,
                                                     double *part, int G, long long dunits)
{
    // part[k*G + blockIdx.x] = block partial of <w, v_k>, k = blockIdx.y*kCgsKC + kk < nk
    if (gated(g)) return;
    const int k0 = blockIdx.y * kCgsKC;
    const int kc = nk - k0 < kCgsKC ? nk - k0 : kCgsKC;
    double acc[kCgsKC];
#pragma unroll
    for (int kk = 0; kk < kCgsKC; kk++) acc[kk] = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < dunits; u += stride) {
        const double2 a = ld2(w, u);
#pragma unroll
        for (int kk = 0; kk < kCgsKC; kk++) {
            if (kk < kc) {
                const double2 b = ld2_nt(V + (long long)(k0 + kk) * ldv, u);
                acc[kk] += a.x * b.x;
                acc[kk] += a.y * b.y;
            }
        }
    }
    block_sum_store<kCgsKC>(acc, kc, part + (long long)k0 * G + blockIdx.x, G);
}
// h[k] = sum of every shard's partials of dot k (shard q's at part + q*cnt + k*G,
// summed in sum_partials' order over the P*G partials, shard-major);
// add = 0: H[k, i] = h[k]; add = 1: H[k, i] += h[k].  One block per k.
__global__ __launch_bounds__(kBlock) void k_cgs_reduce(Gate g, const double *part, int P, int G, long long cnt,
                                                       double *h, double *H, int i, int m, int add)
{
    if (gated(g)) return;
    const int k = blockIdx.x;
    double v = 0.0;
    for (int e = threadIdx.x; e < P * G; e += kBlock) v += part[(long long)(e / G) * cnt + (long long)k * G + e % G];
    v = block_sum(v);
    if (threadIdx.x == 0) {
        h[k] = v;
        double *hk = H + k + (long long)i * (m + 1);
        *hk = add ? *hk + v : v;
    }
}
// a = a - sum_k h[k] v_k(u), k ascending (a = (-h_k) v_k + a, the MGS AXPY's
// rounding), the loads of up to kCgsChunk v_k issued before their
// multiply-adds (a thread owns one or a few units: one load round trip per
// chunk, not per vector); the chunk's values are left in b for the caller.
constexpr int kCgsChunk = 32;
__device__ __forceinline__ void cgs_axpy_chunk(double2 &a, double2 (&b)[kCgsChunk], const double *__restrict__ V,
                                               long long ldv, const double *h, int k0, int nk, long long u)
{
#pragma unroll
    for (int kk = 0; kk < kCgsChunk; kk++)
        if (k0 + kk < nk) b[kk] = ld2_nt(V + (long long)(k0 + kk) * ldv, u);
#pragma unroll
    for (int kk = 0; kk < kCgsChunk; kk++) {
        if (k0 + kk < nk) {
            const double c = -h[k0 + kk];
            a.x = c * b[kk].x + a.x;
            a.y = c * b[kk].y + a.y;
        }
    }
}
// w = w - sum_k h[k] v_k (per element, k ascending: w = (-h_k) v_k + w as the
// MGS AXPY); norm: block partials of <w, w> over [0, dunits) into part_norm
template <bool NORM>
__global__ __launch_bounds__(kBlock) void k_cgs_update(Gate g, double *__restrict__ w,
                                                       const double *__restrict__ V, long long ldv,
                                                       const double *h, int nk, long long units,
                                                       long long dunits, double *part_norm)
{
    if (gated(g)) return;
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units; u += stride) {
        double2 a = ld2(w, u);
        double2 b[kCgsChunk];
        for (int k0 = 0; k0 < nk; k0 += kCgsChunk) cgs_axpy_chunk(a, b, V, ldv, h, k0, nk, u);
        st2(w, u, a);
        if (NORM && u < dunits) {
            acc += a.x * a.x;
            acc += a.y * a.y;
        }
    }
    if (NORM) {
        acc = block_sum(acc);
        if (threadIdx.x == 0) part_norm[blockIdx.x] = acc;
    }
}

// CGS2's first update fused with the second pass's dot partials: w = w - sum_k
// h[k] v_k (as k_cgs_update), then the block partials of <w, v_k>, k < nk, over
// [0, dunits) into part[k*G + block] -- the same unit -> thread assignment and
// accumulation order as k_multidot (G blocks, grid stride), so bit-identical to
// the two launches; each v_k(u) is read once (kept in registers between the
// update and the dots).
constexpr int kCgsFuseMax = kCgsChunk;       // dots held per thread (else two launches)
__global__ __launch_bounds__(kBlock) void k_cgs_update_dot(Gate g, double *__restrict__ w,
                                                           const double *__restrict__ V, long long ldv,
                                                           const double *h, int nk, long long units,
                                                           long long dunits, double *part, int G)
{
    if (gated(g)) return;
    double acc[kCgsFuseMax];
#pragma unroll
    for (int k = 0; k < kCgsFuseMax; k++) acc[k] = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units; u += stride) {
        double2 a = ld2(w, u);
        double2 b[kCgsChunk];
        cgs_axpy_chunk(a, b, V, ldv, h, 0, nk, u);
        st2(w, u, a);
        if (u < dunits) {
#pragma unroll
            for (int k = 0; k < kCgsFuseMax; k++) {
                if (k < nk) {
                    acc[k] += a.x * b[k].x;
                    acc[k] += a.y * b[k].y;
                }
            }
        }
    }
    block_sum_store<kCgsFuseMax>(acc, nk, part + blockIdx.x, G);   // static indices: acc stays in registers
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
                                                             long long units, long long zs = 0)
{
    if (gated_z(g, zs, blockIdx.y)) return;
    if (zs) {
        const int sc = blockIdx.y;
        ds = zp(ds, zs, sc);
        part = zp(part, zs, sc);
        w = zp(w, zs, sc);
        vnext = zp(vnext, zs, sc);
        H = zp(H, zs, sc);
        cs = zp(cs, zs, sc);
        sn = zp(sn, zs, sc);
        s = zp(s, zs, sc);
        hist = zp(hist, zs, sc);
    }
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
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u0 = blockIdx.x * (long long)kBlock + threadIdx.x; u0 < units; u0 += 4 * stride) {
        double2 a[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (u0 + j * stride < units) a[j] = ld2(w, u0 + j * stride);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (u0 + j * stride < units) {
                a[j].x = inv * a[j].x;
                a[j].y = inv * a[j].y;
                st2(vnext, u0 + j * stride, a[j]);
            }
        }
    }
}

// ---- CGS2 with its exchanges inside the kernels (kernels.h, Xch) ------------
// Four launches per inner iteration instead of nine plus three all-gathers:
// k_multidot_x -> k_cgs_update_x<dots> -> k_cgs_update_x<norm> ->
// k_arnoldi_finalize_x, each producer publishing its block partials into every
// rank's area itself and each consumer reducing them in k_cgs_reduce's order
// (so every value has the bits of the launch-per-step path).  A consumer waits
// only for exchanges its peers' EARLIER launches produce, so the waits form no
// cycle; inside a launch the reducer blocks (blockIdx < nk) hand their values to
// the rest through hx / hf -- they are dispatched first and wait on nothing of
// this launch.  Every spin is bounded (~30 s, err |= 4); after one time-out the
// others give up at once (the broken word hf[kCgsXMax + 1]).
// Memory ordering without cache maintenance: the areas and hx / hf are
// uncached device memory, so a producer's stores are in memory once its
// s_waitcnt has drained them, and a consumer's relaxed system-scope loads
// issued after it saw the flag read memory.  No release / acquire here: on
// gfx950 those write back / invalidate the whole L2 (the first version of this
// path, with them: CGS2 64 -> 278 us per iteration at C2/8).
__device__ __forceinline__ unsigned long long *xk_flag(void *base, int P, long long capd, int src)
{
    return reinterpret_cast<unsigned long long *>(base) + (long long)kMaxShards * kIpcXB + 2LL * P * capd +
           (long long)src * kIpcXF;
}
__device__ __forceinline__ double *xk_slot(void *base, int P, long long capd, unsigned long long seq, int src)
{
    return reinterpret_cast<double *>(base) + (long long)kMaxShards * kIpcXB +
           ((long long)(seq & 1) * P + src) * capd;
}
__device__ __noinline__ bool xk_wait_slow(const unsigned long long *f, unsigned long long seq, const Xch &x)
{
    unsigned long long *broken = x.hf + kCgsXMax + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned n = 1;; n++) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= seq) return true;
        if ((n & 255) == 0) {
            if (__hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {     // ~30 s of the 100 MHz clock
                atomicOr(x.err, 4);
                __hip_atomic_store(broken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
        }
    }
}
__device__ __forceinline__ bool xk_wait(const unsigned long long *f, unsigned long long seq, const Xch &x)
{
    bool ok = true;
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) ok = xk_wait_slow(f, seq, x);
    asm volatile("" ::: "memory");        // what follows reads after the flag was seen
    return ok;
}
// thread t < n holds v for index idx of this rank's slot: into the own slot
// and every peer's area, then this block's flag in every peer's area
__device__ __forceinline__ void st_sys(double *p, double v)
{
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys(const double *p)
{
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ void xk_publish(const Xch &x, unsigned long long seq, double *own, bool has,
                                           long long idx, double v, int fblock)
{
    // (loopback: this rank's area stands in for every peer's and receives the
    // values in the slots and flags the peers' would use, q's for peer q)
    if (has) {
        own[idx] = v;
        for (int q = 0; q < x.P; q++)
            if (q != x.me) st_sys(xk_slot(x.pp.base[q], x.P, x.capd, seq, x.loop ? q : x.me) + idx, v);
    }
    __builtin_amdgcn_s_waitcnt(0);          // this thread's stores are in memory
    __syncthreads();
    const int t = threadIdx.x;
    if (t < x.P && t != x.me)
        __hip_atomic_store(xk_flag(x.pp.base[t], x.P, x.capd, x.loop ? t : x.me) + fblock, seq, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
// dot k over every rank's G block partials, in k_cgs_reduce's order (e = q*G + b,
// thread-strided, block_sum); own = this rank's slot.  A thread takes its
// partials kXkChunk at a time: the chunk's flags polled together (relaxed,
// only the pending ones re-polled), one acquire fence, the chunk's values
// loaded together -- two memory round trips per chunk, not two per partial.
constexpr int kXkChunk = 8;
__device__ __forceinline__ double xk_reduce(const Xch &x, unsigned long long seq, const double *own, int G, int k,
                                           int kfl = 0)
{
    // kfl: the producer's grid took kfl dots per block row (flag (k / kfl) * G + b), 0: one row
    double v = 0.0;
    void *mine = x.pp.base[x.me];
    const int PG = x.P * G;
    const int frow = kfl ? (k / kfl) * G : 0;
    for (int e0 = threadIdx.x; e0 < PG; e0 += kXkChunk * kBlock) {
        unsigned long long f[kXkChunk];
#pragma unroll
        for (int j = 0; j < kXkChunk; j++) {
            const int e = e0 + j * kBlock, q = e / G;
            f[j] = ~0ull;
            if (e < PG && q != x.me)
                f[j] = __hip_atomic_load(xk_flag(mine, x.P, x.capd, q) + frow + e % G, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
        }
#pragma unroll
        for (int j = 0; j < kXkChunk; j++) {
            if (f[j] < seq) {
                const int e = e0 + j * kBlock, q = e / G;
                (void)xk_wait(xk_flag(mine, x.P, x.capd, q) + frow + e % G, seq, x);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        asm volatile("" ::: "memory");
        double val[kXkChunk];
#pragma unroll
        for (int j = 0; j < kXkChunk; j++) {
            const int e = e0 + j * kBlock, q = e / G, b = e % G;
            const long long idx = (long long)k * G + b;
            val[j] = 0.0;
            if (e < PG)
                val[j] = q == x.me ? own[idx] : ld_sys(xk_slot(mine, x.P, x.capd, seq, q) + idx);
        }
#pragma unroll
        for (int j = 0; j < kXkChunk; j++)
            if (e0 + j * kBlock < PG) v += val[j];
    }
    return block_sum(v);
}
// a reducer's value to every block of the launch (thread 0)
__device__ __forceinline__ void xk_post(const Xch &x, int slot, double v, unsigned long long seq)
{
    st_sys(x.hx + slot, v);
    __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(x.hf + slot, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// block_sum_store's sums, thread k < nk receiving sum k
template <int NK>
__device__ __forceinline__ double block_sum_pick(const double (&acc)[NK], int nk)
{
    __shared__ double sh[kBlock / 64][NK];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NK; k++) {
        if (k < nk) {
            const double v = wave_sum(acc[k]);
            if (lane == 0) sh[w][k] = v;
        }
    }
    __syncthreads();
    const int k = threadIdx.x < nk ? threadIdx.x : 0;
    return (sh[0][k] + sh[1][k]) + (sh[2][k] + sh[3][k]);
}

__global__ __launch_bounds__(kBlock) void k_multidot_x(Gate g, const double *__restrict__ w,
                                                       const double *__restrict__ V, long long ldv, int nk,
                                                       double *part, int G, long long dunits, Xch x,
                                                       unsigned long long seq)
{
    // block (b, y): dots y*kCgsKC + kk as k_multidot; flag y*G + b
    if (gated(g)) return;
    const int k0 = blockIdx.y * kCgsKC;
    const int kc = nk - k0 < kCgsKC ? nk - k0 : kCgsKC;
    double acc[kCgsKC];
#pragma unroll
    for (int kk = 0; kk < kCgsKC; kk++) acc[kk] = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < dunits; u += stride) {
        const double2 a = ld2(w, u);
#pragma unroll
        for (int kk = 0; kk < kCgsKC; kk++) {
            if (kk < kc) {
                const double2 b = ld2_nt(V + (long long)(k0 + kk) * ldv, u);
                acc[kk] += a.x * b.x;
                acc[kk] += a.y * b.y;
            }
        }
    }
    const double v = block_sum_pick<kCgsKC>(acc, kc);
    xk_publish(x, seq, part, threadIdx.x < kc, (long long)(k0 + threadIdx.x) * G + blockIdx.x, v,
               blockIdx.y * gridDim.x + blockIdx.x);
}

// h = reduced exchange sin (H[k, i] = h, or += with add); w -= V h; then
// DOTS: the partials of <w, v_k> (k_cgs_update_dot), else the norm's
// (k_cgs_update<true>), published as exchange sout into part_out
template <bool DOTS>
__global__ __launch_bounds__(kBlock) void k_cgs_update_x(Gate g, double *__restrict__ w,
                                                         const double *__restrict__ V, long long ldv, int nk,
                                                         long long units, long long dunits, int G,
                                                         const double *part_in, unsigned long long sin, double *H,
                                                         int i, int m, int add, double *part_out, Xch x,
                                                         unsigned long long sout, int kfl)
{
    if (gated(g)) return;
    __shared__ double hs[kCgsXMax];
    for (int k = blockIdx.x; k < nk; k += gridDim.x) {
        const double v = xk_reduce(x, sin, part_in, G, k, kfl);
        if (threadIdx.x == 0) {
            double *hk = H + k + (long long)i * (m + 1);
            *hk = add ? *hk + v : v;
            xk_post(x, k, v, sin);
        }
    }
    if (threadIdx.x < nk) {
        (void)xk_wait(x.hf + threadIdx.x, sin, x);
        hs[threadIdx.x] = ld_sys(x.hx + threadIdx.x);
    }
    __syncthreads();
    double acc[DOTS ? kCgsXMax : 1];
#pragma unroll
    for (int k = 0; k < (DOTS ? kCgsXMax : 1); k++) acc[k] = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units; u += stride) {
        double2 a = ld2(w, u);
        double2 b[kCgsChunk];
        cgs_axpy_chunk(a, b, V, ldv, hs, 0, nk, u);
        st2(w, u, a);
        if (u < dunits) {
            if constexpr (DOTS) {
#pragma unroll
                for (int k = 0; k < kCgsXMax; k++) {
                    if (k < nk) {
                        acc[k] += a.x * b[k].x;
                        acc[k] += a.y * b[k].y;
                    }
                }
            } else {
                acc[0] += a.x * a.x;
                acc[0] += a.y * a.y;
            }
        }
    }
    if constexpr (DOTS) {
        const double v = block_sum_pick<kCgsXMax>(acc, nk);
        xk_publish(x, sout, part_out, threadIdx.x < nk, (long long)threadIdx.x * G + blockIdx.x, v, blockIdx.x);
    } else {
        const double v = block_sum(acc[0]);
        xk_publish(x, sout, part_out, threadIdx.x == 0, blockIdx.x, v, blockIdx.x);
    }
}

// MGS of the sharded solve on the same exchanges (the reference's
// orthogonalization, i + 3 launches per inner iteration instead of 2i + 5):
// k_dot_x = k_dot publishing its partials; k_mgs_step_x = k_mgs_step with h
// reduced from exchange sin by block 0 (sum_partials' order over the P*G
// partials) and its partials published as exchange sout
__global__ __launch_bounds__(kBlock) void k_dot_x(Gate g, const double *a, const double *b, double *part,
                                                  long long units, Xch x, unsigned long long seq)
{
    if (gated(g)) return;
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u0 = blockIdx.x * (long long)kBlock + threadIdx.x; u0 < units; u0 += 4 * stride) {
        double2 p[4], q[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const long long u = u0 + j * stride;
            if (u < units) { p[j] = ld2(a, u); q[j] = ld2(b, u); }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (u0 + j * stride < units) {
                acc += p[j].x * q[j].x;
                acc += p[j].y * q[j].y;
            }
        }
    }
    acc = block_sum(acc);
    xk_publish(x, seq, part, threadIdx.x == 0, blockIdx.x, acc, blockIdx.x);
}
template <bool NORM>
__global__ __launch_bounds__(kBlock) void k_mgs_step_x(Gate g, int i, int k, int m, double *__restrict__ w,
                                                       const double *__restrict__ vk,
                                                       const double *__restrict__ vnext, const double *part_in,
                                                       unsigned long long sin, double *part_out, double *H, int G,
                                                       long long units, long long dunits, Xch x,
                                                       unsigned long long sout)
{
    if (gated(g)) return;
    __shared__ double hsh;
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    long long u0 = blockIdx.x * (long long)kBlock + threadIdx.x;
    double2 wv[kUnroll], vv[kUnroll], nv[kUnroll];
    auto load = [&]() {
#pragma unroll
        for (int j = 0; j < kUnroll; j++) {
            const long long u = u0 + j * stride;
            if (u < units) {
                wv[j] = ld2(w, u);
                vv[j] = ld2_nt(vk, u);
                if (!NORM) nv[j] = ld2_nt(vnext, u);
            }
        }
    };
    load();                 // the first chunk is in flight while h is summed
    if (blockIdx.x == 0) {
        const double v = xk_reduce(x, sin, part_in, G, 0);
        if (threadIdx.x == 0) {
            H[k + i * (m + 1)] = v;
            xk_post(x, 0, v, sin);
        }
    }
    if (threadIdx.x == 0) {
        (void)xk_wait(x.hf, sin, x);
        hsh = ld_sys(x.hx);
    }
    __syncthreads();
    const double a = -hsh;
    while (u0 < units) {
#pragma unroll
        for (int j = 0; j < kUnroll; j++) {
            const long long u = u0 + j * stride;
            if (u < units) {
                wv[j].x = a * vv[j].x + wv[j].x;
                wv[j].y = a * vv[j].y + wv[j].y;
                st2(w, u, wv[j]);
                if (NORM) nv[j] = wv[j];
                if (u < dunits) {
                    acc += wv[j].x * nv[j].x;
                    acc += wv[j].y * nv[j].y;
                }
            }
        }
        u0 += kUnroll * stride;
        load();
    }
    acc = block_sum(acc);
    xk_publish(x, sout, part_out, threadIdx.x == 0, blockIdx.x, acc, blockIdx.x);
}

// k_arnoldi_finalize, ||w||^2 reduced from exchange sin by block 0
__global__ __launch_bounds__(kBlock) void k_arnoldi_finalize_x(Gate g, int i, int m, DevState *ds,
                                                               const double *part_in, unsigned long long sin,
                                                               int G, const double *w, double *vnext, double *H,
                                                               double *cs, double *sn, double *s, double *hist,
                                                               long long units, Xch x)
{
    if (gated(g)) return;
    __shared__ double nrm2;
    if (blockIdx.x == 0) {
        const double v = xk_reduce(x, sin, part_in, G, 0);
        if (threadIdx.x == 0) xk_post(x, kCgsXMax, v, sin);
    }
    if (threadIdx.x == 0) {
        (void)xk_wait(x.hf + kCgsXMax, sin, x);
        nrm2 = ld_sys(x.hx + kCgsXMax);
    }
    __syncthreads();
    const double hn = sqrt(nrm2);
    if (blockIdx.x == 0 && threadIdx.x == 0) {      // as k_arnoldi_finalize
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
        if (resid < ds->tol) {
            ds->conv_i = i;
            ds->done = DONE_INNER;
        }
    }
    const double inv = (hn != 0.0) ? 1.0 / hn : 0.0;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units; u += stride) {
        double2 a = ld2(w, u);
        a.x = inv * a.x;
        a.y = inv * a.y;
        st2(vnext, u, a);
    }
}

// ---- persistent Arnoldi orthogonalization: <w,v_0>, the i+1 MGS steps, the
// norm, Givens and v_{i+1} = w/||w|| of inner iteration i in ONE launch.
// Block g owns the same units as in the per-step kernels (u = g*256 + t +
// j*G*256) and keeps them of w and of the current basis vector in registers
// across the steps, so a step reads one basis vector from HBM instead of
// w, v_k, v_{k+1} and writing w.  The per-step global sum is an all-gather of
// the G block partials through 8-byte granules (sentinel = not ready, relaxed
// agent-scope stores and polls, one row of G per step, re-armed per cycle);
// every block sums them in sum_partials' fixed order, so h is bit-identical to
// the per-step kernels'.  Needs all G blocks resident (checked on the host);
// every spin is bounded (err bit 0).
// Co-residency: the grid is sized from the occupancy API, which
// has over-promised on this pool (profiles/r03/r03_gather_ab.txt).  So the kernels
// do not trust it: the FIRST all-gather of a launch waits at most kResidSpin
// polls; a block that times out there sets DONE_ABORT in the control block
// (agent-scope atomic, drained before the block exits) and leaves.  A block
// entering the kernel returns at once when DONE_ABORT is set -- a block that
// was not resident can only be dispatched after some block exited, and only
// an aborting block exits early -- and every later poll that has to retry
// checks the flag every 256 retries, so the grid drains either way.
// DONE_ABORT gates the rest of the enqueued cycle off; the host restores the
// control block and reruns the cycle on the per-step kernels (same bits).

__device__ __forceinline__ int ld_agent_int(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the whole block: was the cycle aborted?  (entry check, one sc1 load)
__device__ __forceinline__ bool block_aborted(const DevState *ds)
{
    __shared__ int ab;
    if (threadIdx.x == 0) ab = ld_agent_int(&ds->done) & DONE_ABORT;
    __syncthreads();
    return ab != 0;
}
__device__ __forceinline__ void set_abort(DevState *ds)
{
    atomicOr(&ds->done, DONE_ABORT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // performed before this block exits
}

__device__ __forceinline__ unsigned long long poll_granule(const unsigned long long *p, int *err,
                                                          const int *abortw = nullptr)
{
    unsigned long long a = ld_agent(p);
    int spins = 0;
    while (a == kSentinel) {
        __builtin_amdgcn_s_sleep(1);
        a = ld_agent(p);
        if (abortw && (spins & 255) == 255 && (ld_agent_int(abortw) & DONE_ABORT)) break;
        if (++spins > kSpinLimit) {
            atomicOr(err, 1);
            break;
        }
    }
    return a;
}

// A thread's granules of a G-partial row (q = threadIdx.x + r*kBlock, G <=
// 1024): all of them loaded at once, then only the pending ones polled again --
// one memory round trip for the row instead of one per granule (a poll loop
// per granule serializes them: G = 544 put three sc1 round trips on every
// all-gather).  The sum is taken afterwards in q order, as before: same bits.
// Measured and not kept (round 5, profiles/r05/stage_ab.txt): two poll rounds
// in flight (a second load of every pending granule half a round trip after
// the first, here and in the blocks' slot poll): MGS 59.7 -> 75 us -- the
// extra polls slow the hand-offs more than they shorten the detection.
constexpr int kGatherPer = 4;
template <int NP>
__device__ __forceinline__ bool gather_row(const unsigned long long *row, int G, unsigned long long (&a)[NP],
                                           int limit, const int *abortw)
{
#pragma unroll
    for (int r = 0; r < NP; r++) {
        const int q = threadIdx.x + r * kBlock;
        a[r] = q < G ? ld_agent(row + q) : 0ull;
    }
    int spins = 0;
    while (true) {
        bool pend = false;
#pragma unroll
        for (int r = 0; r < NP; r++) pend |= a[r] == kSentinel;
        if (!pend) return true;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int r = 0; r < NP; r++)
            if (a[r] == kSentinel) a[r] = ld_agent(row + threadIdx.x + r * kBlock);
        if (abortw && (spins & 255) == 255 && (ld_agent_int(abortw) & DONE_ABORT)) return false;
        if (++spins > limit) return false;
    }
}
template <int NP>
__device__ __forceinline__ double gather_row_sum(const unsigned long long (&a)[NP], int G)
{
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < NP; r++)
        if (threadIdx.x + r * kBlock < G) v += __longlong_as_double((long long)a[r]);
    return v;
}

// NP: granules per thread the row may have (G <= NP * kBlock); NP = 0: one
// poll loop per granule (k_arnoldi_wide, whose 256 VGPRs are taken by w and
// the stream: the parallel form spills there)
template <int NP = kGatherPer>
__device__ __forceinline__ double gather_sum(const unsigned long long *row, int G, int *err, int &par,
                                             const int *abortw = nullptr)
{
    if constexpr (NP == 0) {
        double v = 0.0;
        for (int q = threadIdx.x; q < G; q += kBlock)
            v += __longlong_as_double((long long)poll_granule(row + q, err, abortw));
        return block_sum_pp(v, par);
    } else {
        unsigned long long a[NP];
        if (!gather_row<NP>(row, G, a, kSpinLimit, abortw) && !(abortw && (ld_agent_int(abortw) & DONE_ABORT)))
            atomicOr(err, 1);
        return block_sum_pp(gather_row_sum<NP>(a, G), par);
    }
}

// The launch's first all-gather with the co-residency bound: false = this
// block timed out (DONE_ABORT set) and must return (block-uniform)
template <int NP = kGatherPer>
__device__ __forceinline__ bool gather_first(const unsigned long long *row, int G, DevState *ds, int &par,
                                             double &h)
{
    double v = 0.0;
    int miss = 0;
    if constexpr (NP == 0) {
        for (int q = threadIdx.x; q < G; q += kBlock) {
            unsigned long long a = ld_agent(row + q);
            int spins = 0;
            while (a == kSentinel && !miss) {
                __builtin_amdgcn_s_sleep(1);
                a = ld_agent(row + q);
                if (++spins > kResidSpin) miss = 1;
            }
            v += __longlong_as_double((long long)a);
        }
    } else {
        unsigned long long a[NP];
        miss = gather_row<NP>(row, G, a, kResidSpin, nullptr) ? 0 : 1;
        v = gather_row_sum<NP>(a, G);
    }
    if (__syncthreads_or(miss)) {
        if (threadIdx.x == 0) set_abort(ds);
        return false;
    }
    h = block_sum_pp(v, par);
    return true;
}

// The sum of step k's partials as every block needs it.  LEADER: block 0
// alone gathers the row (gather_sum: the same order, the same bits) and
// publishes the sum in one granule hg; the other blocks' thread 0 polls that
// granule and hands the value over through LDS -- G line requests per poll
// round instead of G x G/32 on the few channels that hold the row, for one
// more hop.  Measured (C2 / C4, profiles/r03/r03_gather_ab.txt): k_arnoldi_wide
// (C4, streaming the basis beside the polls) 472.5 -> 456.6 us, so it leads;
// k_arnoldi_persist (C2) 73.2 -> 77.5 us, so every block gathers there.
template <bool LEADER, int NP = kGatherPer>
__device__ __forceinline__ double gather_h(const unsigned long long *row, unsigned long long *hg, int k, int G,
                                           int *err, int &par, const int *abortw)
{
    if (!LEADER || blockIdx.x == 0) {
        const double h = gather_sum<LEADER ? 0 : NP>(row, G, err, par, abortw);
        if (LEADER && threadIdx.x == 0) st_agent(hg, (unsigned long long)__double_as_longlong(h));
        return h;
    }
    __shared__ double hb[2];                    // alternating: steps k and k+2 are a block_sum apart
    if (threadIdx.x == 0) hb[k & 1] = __longlong_as_double((long long)poll_granule(hg, err, abortw));
    __syncthreads();
    return hb[k & 1];
}
// step 0 of a launch: gather_h with the co-residency bound on every wait
// (LEADER: block 0 gathers with the bound, the others' poll of its sum granule
// is bounded alike -- whichever block is missing, every waiting block times out)
template <bool LEADER, int NP = kGatherPer>
__device__ __forceinline__ bool gather_h_first(const unsigned long long *row, unsigned long long *hg, int G,
                                               DevState *ds, int &par, double &h)
{
    if (!LEADER || blockIdx.x == 0) {
        if (!gather_first<LEADER ? 0 : NP>(row, G, ds, par, h)) return false;
        if (LEADER && threadIdx.x == 0) st_agent(hg, (unsigned long long)__double_as_longlong(h));
        return true;
    }
    __shared__ double hb0;
    int miss = 0;
    if (threadIdx.x == 0) {
        unsigned long long a = ld_agent(hg);
        int spins = 0;
        while (a == kSentinel && !miss) {
            __builtin_amdgcn_s_sleep(1);
            a = ld_agent(hg);
            if (++spins > kResidSpin) miss = 1;
        }
        hb0 = __longlong_as_double((long long)a);
    }
    if (__syncthreads_or(miss)) {
        if (threadIdx.x == 0) set_abort(ds);
        return false;
    }
    h = hb0;
    return true;
}

// XCD-local form (GG_MGS_GATHER=2): ONE block per XCD (the first to arrive,
// elected per launch) gathers the step's G partials -- gather_sum, the same
// order, the same bits -- and stores the sum with a PLAIN store into its
// XCD's slot; the XCD's other blocks poll that slot (thread 0, sc1 loads).
// A plain store keeps the line in the XCD's L2, where the sc1 (L1-bypassing)
// polls of the same XCD find it: 234 / 677 ns a hop idle / streaming against
// 470 / 740 for sc1 stores (profiles/r04/r04_xcd_handoff.txt).  Correct by
// construction, not by placement: a block polls only the slot of the XCD it
// runs on (HW_REG_XCC_ID), which only a reducer ON that XCD writes.  8 pollers
// of the G-granule row instead of G.
constexpr int kXcdSlot = 16;                 // words per XCD slot (own 128-B line)
constexpr int kXcds = 8;
__device__ __forceinline__ unsigned xcc_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & (kXcds - 1);
}
__device__ __forceinline__ void st_plain(unsigned long long *p, unsigned long long v)
{
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
// this block's role for the launch: the first block of its XCD to raise the
// XCD's election word to `seq` (strictly increasing per launch) reduces
__device__ __forceinline__ void xcd_elect(unsigned long long *elect, unsigned long long seq, bool &red,
                                          unsigned &xcc)
{
    __shared__ unsigned sx;
    __shared__ int sr;
    if (threadIdx.x == 0) {
        const unsigned x = xcc_id();
        sx = x;
        sr = atomicMax(elect + x * kXcdSlot, seq) < seq;
    }
    __syncthreads();
    red = sr != 0;
    xcc = sx;
}
// XG 3: a unit-holding block reduces for its XCD only when no reducer-only
// block has claimed the XCD for this launch (word 1 of the XCD's election
// slot).  The reducer-only blocks are blocks 0..kXcds-1, dispatched first and
// (round-robin) one per XCD, so the claim is normally there already; a short
// bounded wait covers its landing, and an XCD left without one (placement is
// not guaranteed) elects a unit-holding block as in XG 2.  Two reducers on one
// XCD store the same bits into its slot: harmless.
__device__ __forceinline__ void xcd_elect3(unsigned long long *elect, unsigned long long seq, bool &red,
                                           unsigned &xcc)
{
    __shared__ unsigned sx;
    __shared__ int sr;
    if (threadIdx.x == 0) {
        const unsigned x = xcc_id();
        sx = x;
        bool claimed = false;
        for (int t = 0; t < 16 && !claimed; t++) {
            claimed = ld_agent(elect + x * kXcdSlot + 1) == seq;
            if (!claimed) __builtin_amdgcn_s_sleep(8);
        }
        sr = !claimed && atomicMax(elect + x * kXcdSlot, seq) < seq;
    }
    __syncthreads();
    red = sr != 0;
    xcc = sx;
}
// step k's sum: slot = this XCD's word of step k
template <int NP>
__device__ __forceinline__ double gather_xcd(const unsigned long long *row, unsigned long long *slot, int k, int G,
                                            bool red, int *err, int &par, const int *abortw)
{
    if (red) {
        const double h = gather_sum<NP>(row, G, err, par, abortw);
        if (threadIdx.x == 0) st_plain(slot, (unsigned long long)__double_as_longlong(h));
        return h;
    }
    __shared__ double hb[2];                    // alternating: steps k and k+2 are a barrier apart
    if (threadIdx.x == 0) hb[k & 1] = __longlong_as_double((long long)poll_granule(slot, err, abortw));
    __syncthreads();
    return hb[k & 1];
}
template <int NP>
__device__ __forceinline__ bool gather_xcd_first(const unsigned long long *row, unsigned long long *slot, int G,
                                                 bool red, DevState *ds, int &par, double &h)
{
    if (red) {
        if (!gather_first<NP>(row, G, ds, par, h)) return false;
        if (threadIdx.x == 0) st_plain(slot, (unsigned long long)__double_as_longlong(h));
        return true;
    }
    __shared__ double hb0;
    int miss = 0;
    if (threadIdx.x == 0) {
        unsigned long long a = ld_agent(slot);
        int spins = 0;
        while (a == kSentinel && !miss) {
            __builtin_amdgcn_s_sleep(1);
            a = ld_agent(slot);
            if (++spins > kResidSpin) miss = 1;
        }
        hb0 = __longlong_as_double((long long)a);
    }
    if (__syncthreads_or(miss)) {
        if (threadIdx.x == 0) set_abort(ds);
        return false;
    }
    h = hb0;
    return true;
}

// XG: the all-gather's form -- 0 every block gathers, 2 XCD-local reducers
// (gather_xcd; xb = per step kXcds slots of kXcdSlot words, elect / seq the
// per-launch election)
// PF: v_{k+1} streamed while step k's sum is gathered (1), or after it (0):
// polls issued behind a wave's own in-flight basis loads wait for them (the
// memory returns in order) and the gather then also pays the stream's latency
constexpr int persist_np(int J) { return J >= 8 ? 0 : kGatherPer; }
template <int J, int XG, int PF>
__global__ __launch_bounds__(kBlock) void k_arnoldi_persist(Gate g, int i, int m, DevState *ds,
                                                            const double *__restrict__ w_in,
                                                            double *__restrict__ V, long long ldv,
                                                            double *H, double *cs, double *sn,
                                                            double *s, double *hist,
                                                            unsigned long long *gran, unsigned long long *hg,
                                                            long long units, int *err, unsigned long long *xb,
                                                            unsigned long long *elect, unsigned long long seq,
                                                            UnitMap um, long long *trace, const double *msc,
                                                            double *mout, unsigned long long *fill, long long nfill)
{
    // msc / mout (the split engine): also mout = v_{i+1} * msc, k_mul's product
    // for the next iteration's Mr (one pass fewer per iteration); fill: slots
    // < nfill set to the sentinel (the next flow U solve's x, its fill launch)
    // granules per thread loaded at once in the all-gathers (persist_np; J =
    // 8 polls them one by one: the parallel form would cost it an occupancy step)
    constexpr int kNP = persist_np(J);
    if (gated(g)) return;
    if (block_aborted(ds)) return;                            // co-residency (gather_first)
    // XG 3: the first kXcds blocks hold no units; they only reduce (below)
    constexpr int XR = XG == 3 ? kXcds : 0;
    const int G = gridDim.x - XR;                             // the blocks holding units
    const int ub = (int)blockIdx.x - XR;                      // this block's unit-block index
    const int *abortw = &ds->done;
    bool red = true;
    unsigned xcc = 0;
    auto xslot = [&](int k) { return xb + ((long long)k * kXcds + xcc) * kXcdSlot; };
    if constexpr (XG == 3) {
        if (ub < 0) {
            // reducer-only block: claim this XCD for the launch, then gather
            // every step's row (no basis loads in front of its polls) and
            // store the sum into the XCD's slot -- gather_xcd's reducer half
            int par = 0;
            __shared__ unsigned sxr;
            if (threadIdx.x == 0) {
                sxr = xcc_id();
                atomicMax(elect + sxr * kXcdSlot + 1, seq);
            }
            __syncthreads();
            xcc = sxr;
            double h;
            if (!gather_first<kNP>(gran, G, ds, par, h)) return;
            if (threadIdx.x == 0) st_plain(xslot(0), (unsigned long long)__double_as_longlong(h));
            for (int k = 1; k <= i + 1; k++) {
                h = gather_sum<kNP>(gran + (long long)k * G, G, err, par, abortw);
                if (threadIdx.x == 0) st_plain(xslot(k), (unsigned long long)__double_as_longlong(h));
            }
            return;
        }
        xcd_elect3(elect, seq, red, xcc);
    }
    if constexpr (XG == 2) xcd_elect(elect, seq, red, xcc);
    const long long stride = (long long)G * kBlock;
    const long long u0 = ub * (long long)kBlock + threadIdx.x;
    // diagnostics (GG_MGS_TRACE): per step the start, h known, partial formed,
    // partial published -- row 0 unit-block 0, row 1 the reducer of XCD 0
    const int trow = !trace ? -1 : ub == 0 ? 0 : (red && xcc == 0 && XG == 2) ? 1 : -1;
    auto stamp = [&](int k, int ph) {
        if (trow >= 0 && threadIdx.x == 0)
            trace[((long long)trow * (i + 2) + k) * 4 + ph] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    double2 w[J], vk[J], vn[J];
    [[maybe_unused]] double2 vl[PF == 2 ? J : 1];             // PF 2: the third basis buffer
    bool val[J];                                              // unit holds a real row (UnitMap)
#pragma unroll
    for (int j = 0; j < J; j++) {
        const long long u = u0 + j * stride;
        val[j] = u < units && unit_real(um, u);
        if (val[j]) {
            w[j] = ld2(w_in, u);
            vk[j] = ld2(V, u);
        }
    }
    auto load_v = [&](int q, double2 *dst) {                  // basis vector q, streamed
        const double *vp = V + (long long)q * ldv;
#pragma unroll
        for (int j = 0; j < J; j++)
            if (val[j]) dst[j] = ld2_nt(vp, u0 + j * stride);
    };
    if constexpr (PF == 2) {
        if (i >= 1) load_v(1, vn);                            // v_1, behind w and v_0
    }
    int par = 0;                                              // block_sum_pp's LDS row
    auto publish = [&](int k, double acc) {
        acc = block_sum_pp(acc, par);
        if (threadIdx.x == 0) st_agent(gran + (long long)k * G + ub, (unsigned long long)__double_as_longlong(acc));
    };
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < J; j++)
        if (val[j]) {
            acc += w[j].x * vk[j].x;
            acc += w[j].y * vk[j].y;
        }
    publish(0, acc);                                          // <w, v_0>
    // step k: h_k, w -= h_k v_k, the partial of the next dot (v_{k+1}, or the
    // norm), published.  cur = v_k, nxt = v_{k+1} (loaded), lnd = the buffer
    // v_{k+2} lands in (PF 2; the three rotate, no register copies -- a copy of
    // a landing buffer would wait for its loads)
    auto step = [&](int k, double2 *cur, double2 *nxt, double2 *lnd) -> bool {
        stamp(k, 0);
        if constexpr (PF == 1) {
            if (k < i) load_v(k + 1, nxt);                    // v_{k+1}, in flight during the sum
        }
        double h;
        if (k == 0) {
            if (XG >= 2 ? !gather_xcd_first<kNP>(gran, xslot(0), G, red, ds, par, h)
                        : !gather_h_first<false, kNP>(gran, hg, G, ds, par, h))
                return false;
        } else if constexpr (XG >= 2) {
            h = gather_xcd<kNP>(gran + (long long)k * G, xslot(k), k, G, red, err, par, abortw);
        } else {
            h = gather_h<false, kNP>(gran + (long long)k * G, hg + k, k, G, err, par, abortw);
        }
        if constexpr (PF == 0) {
            __builtin_amdgcn_sched_barrier(0);
            if (k < i) load_v(k + 1, nxt);                    // v_{k+1} after the sum
        }
        if constexpr (PF == 2) {
            // v_{k+2} issued after this step's polls, which so find no basis
            // loads of their own in front of them (v_{k+1} went out a step ago)
            __builtin_amdgcn_sched_barrier(0);
            if (k + 2 <= i) load_v(k + 2, lnd);
        }
        stamp(k, 1);
        if (ub == 0 && threadIdx.x == 0) H[k + i * (m + 1)] = h;
        const double a = -h;
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (val[j]) {
                w[j].x = a * cur[j].x + w[j].x;
                w[j].y = a * cur[j].y + w[j].y;
                const double2 o = (k < i) ? nxt[j] : w[j];    // next dot: v_{k+1}, or the norm
                acc += w[j].x * o.x;
                acc += w[j].y * o.y;
            }
        }
        stamp(k, 2);
        publish(k + 1, acc);
        stamp(k, 3);
        return true;
    };
    if constexpr (PF == 2) {
        for (int k = 0; k <= i; k += 3) {
            if (!step(k, vk, vn, vl)) return;
            if (k + 1 > i) break;
            step(k + 1, vn, vl, vk);
            if (k + 2 > i) break;
            step(k + 2, vl, vk, vn);
        }
    } else {
        for (int k = 0; k <= i; k += 2) {
            if (!step(k, vk, vn, nullptr)) return;
            if (k + 1 > i) break;
            step(k + 1, vn, vk, nullptr);
        }
    }
    stamp(i + 1, 0);
    const double hn = sqrt(XG >= 2 ? gather_xcd<kNP>(gran + (long long)(i + 1) * G, xslot(i + 1), i + 1, G, red, err, par,
                                                abortw)
                                   : gather_h<false, kNP>(gran + (long long)(i + 1) * G, hg + i + 1, i + 1, G, err, par,
                                                     abortw));
    stamp(i + 1, 1);
    if (ub == 0 && threadIdx.x == 0) {                       // as k_arnoldi_finalize
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
        if (resid < ds->tol) {
            ds->conv_i = i;
            ds->done = DONE_INNER;
        }
    }
    const double inv = (hn != 0.0) ? 1.0 / hn : 0.0;
    double *vout = V + (long long)(i + 1) * ldv;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const long long u = u0 + j * stride;
        if (val[j]) {
            double2 a = w[j];
            a.x = inv * a.x;
            a.y = inv * a.y;
            st2(vout, u, a);
            if (mout) {
                const double2 c = ld2(msc, u);
                st2(mout, u, make_double2(a.x * c.x, a.y * c.y));
            }
        } else if (mout && u < units) {
            // padding: k_mul's product of the slot as it stands (never written here)
            const double2 a = ld2(vout, u), c = ld2(msc, u);
            st2(mout, u, make_double2(a.x * c.x, a.y * c.y));
        }
        if (fill && u < units) {
            if (2 * u < nfill) fill[2 * u] = kSentinel;
            if (2 * u + 1 < nfill) fill[2 * u + 1] = kSentinel;
        }
    }
}

// ---- two scenarios per launch (the many-RHS batch, batch.hip) ----------------
// k_arnoldi_persist's default form (XCD-local reducers, v_{k+1} streamed during
// the gather) for two scenarios at once: scenario q's buffers q * zs bytes after
// scenario 0's; per step the two rows are gathered together -- every granule of
// both loaded at once, the pending ones re-polled, then each row summed in the
// same q order (gather_row_sum + block_sum_pp: the same bits) -- so the two
// scenarios share the step's hand-off latency instead of paying it in two
// launches.  A gated scenario (converged) is skipped inside the launch.
template <int J>
__device__ __forceinline__ void gather2_xcd(const unsigned long long *row0, const unsigned long long *row1,
                                            unsigned long long *slot0, unsigned long long *slot1, int G, bool red,
                                            const bool (&act)[2], int *err, int &par, int limit,
                                            const int *abort0, const int *abort1, double (&h)[2], int &miss)
{
    constexpr int NP = kGatherPer;
    __shared__ double hb2[2][2];
    if (red) {
        unsigned long long a[2][NP];
        const unsigned long long *rows[2] = {row0, row1};
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int r = 0; r < NP; r++) {
                const int k = threadIdx.x + r * kBlock;
                a[q][r] = (act[q] && k < G) ? ld_agent(rows[q] + k) : 0ull;
            }
        int spins = 0;
        while (true) {
            bool pend = false;
#pragma unroll
            for (int q = 0; q < 2; q++)
#pragma unroll
                for (int r = 0; r < NP; r++) pend |= a[q][r] == kSentinel;
            if (!pend) break;
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int q = 0; q < 2; q++)
#pragma unroll
                for (int r = 0; r < NP; r++)
                    if (a[q][r] == kSentinel) a[q][r] = ld_agent(rows[q] + threadIdx.x + r * kBlock);
            if ((spins & 255) == 255 && ((act[0] && (ld_agent_int(abort0) & DONE_ABORT)) ||
                                         (act[1] && (ld_agent_int(abort1) & DONE_ABORT)))) {
                miss = 1;
                break;
            }
            if (++spins > limit) {
                miss = 1;
                break;
            }
        }
        unsigned long long *slots[2] = {slot0, slot1};
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (!act[q]) continue;                                    // (block-uniform)
            h[q] = block_sum_pp(gather_row_sum<NP>(a[q], G), par);
            if (threadIdx.x == 0) st_plain(slots[q], (unsigned long long)__double_as_longlong(h[q]));
        }
        return;
    }
    // the XCD's other blocks: thread q polls scenario q's slot
    if (threadIdx.x < 2 && act[threadIdx.x]) {
        const unsigned long long *sl = threadIdx.x ? slot1 : slot0;
        unsigned long long v = ld_agent(sl);
        int spins = 0;
        while (v == kSentinel) {
            __builtin_amdgcn_s_sleep(1);
            v = ld_agent(sl);
            const int *ab = threadIdx.x ? abort1 : abort0;
            if ((spins & 255) == 255 && (ld_agent_int(ab) & DONE_ABORT)) {
                miss = 1;
                break;
            }
            if (++spins > limit) {
                miss = 1;
                break;
            }
        }
        hb2[par & 1][threadIdx.x] = __longlong_as_double((long long)v);
    }
    __syncthreads();
    h[0] = hb2[par & 1][0];
    h[1] = hb2[par & 1][1];
    par ^= 1;
}

// three blocks per CU (168 VGPRs at J = 4, 22 spilled): C5's grid of 532
// blocks co-resident (2 per CU at 192 VGPRs would hold 512) -- C5 with 8
// scenarios 10,606 -> 11,255 it/s, MGS 54.3 -> 45.5 us per pair of scenarios
// (profiles/r06/r06x_c5_pair.txt)
template <int J>
__global__ __launch_bounds__(kBlock, 3) void k_arnoldi_persist2(Gate g, long long zs, int i, int m, DevState *ds,
                                                             const double *__restrict__ w_in,
                                                             double *__restrict__ V, long long ldv, double *H,
                                                             double *cs, double *sn, double *s, double *hist,
                                                             unsigned long long *gran, long long units, int *err,
                                                             unsigned long long *xb, unsigned long long *elect,
                                                             unsigned long long seq, UnitMap um)
{
    bool act[2];
    DevState *dsq[2] = {ds, zp(ds, zs, 1)};
    __shared__ int sab[2];
    if (threadIdx.x < 2) sab[threadIdx.x] = ld_agent_int(&dsq[threadIdx.x]->done) & DONE_ABORT;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; q++) act[q] = !gated_z(g, zs, q) && !sab[q];
    if (!act[0] && !act[1]) return;
    const int G = gridDim.x;
    const int ub = (int)blockIdx.x;
    bool red = true;
    unsigned xcc = 0;
    xcd_elect(elect, seq, red, xcc);
    const long long stride = (long long)G * kBlock;
    const long long u0 = ub * (long long)kBlock + threadIdx.x;
    const double *wq[2] = {w_in, zp(w_in, zs, 1)};
    double *Vq[2] = {V, zp(V, zs, 1)};
    unsigned long long *gq[2] = {gran, zp(gran, zs, 1)};
    unsigned long long *xq[2] = {xb, zp(xb, zs, 1)};
    const int *abw[2] = {&dsq[0]->done, &dsq[1]->done};
    auto xslot = [&](int q, int k) { return xq[q] + ((long long)k * kXcds + xcc) * kXcdSlot; };
    double2 w[2][J], vk[2][J], vn[2][J];
    bool val[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const long long u = u0 + j * stride;
        val[j] = u < units && unit_real(um, u);
#pragma unroll
        for (int q = 0; q < 2; q++)
            if (val[j] && act[q]) {
                w[q][j] = ld2(wq[q], u);
                vk[q][j] = ld2(Vq[q], u);
            }
    }
    int par = 0;
    // both scenarios' partials of one step, each with block_sum_pp's tree
    auto publish = [&](int k, double (&acc)[2]) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (!act[q]) continue;
            const double a = block_sum_pp(acc[q], par);
            if (threadIdx.x == 0) st_agent(gq[q] + (long long)k * G + ub, (unsigned long long)__double_as_longlong(a));
        }
    };
    {
        double acc[2] = {0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int j = 0; j < J; j++)
                if (val[j] && act[q]) {
                    acc[q] += w[q][j].x * vk[q][j].x;
                    acc[q] += w[q][j].y * vk[q][j].y;
                }
        publish(0, acc);                                          // <w, v_0>
    }
    auto step = [&](int k, double2 (&cur)[2][J], double2 (&nxt)[2][J]) -> bool {
        if (k < i) {                                              // v_{k+1}, in flight during the gather
#pragma unroll
            for (int q = 0; q < 2; q++) {
                if (!act[q]) continue;
                const double *vp = Vq[q] + (long long)(k + 1) * ldv;
#pragma unroll
                for (int j = 0; j < J; j++)
                    if (val[j]) nxt[q][j] = ld2_nt(vp, u0 + j * stride);
            }
        }
        double h[2] = {0.0, 0.0};
        int miss = 0;
        gather2_xcd<J>(gq[0] + (long long)k * G, gq[1] + (long long)k * G, xslot(0, k), xslot(1, k), G, red, act,
                       err, par, k == 0 ? kResidSpin : kSpinLimit, abw[0], abw[1], h, miss);
        if (k == 0) {
            // the launch's first all-gather bounds the co-residency wait
            if (__syncthreads_or(miss)) {
                if (threadIdx.x < 2 && act[threadIdx.x]) set_abort(dsq[threadIdx.x]);
                return false;
            }
        } else if (miss && !(ld_agent_int(abw[0]) & DONE_ABORT) && !(ld_agent_int(abw[1]) & DONE_ABORT)) {
            atomicOr(err, 1);                                     // a wait timed out
        }
        double acc[2] = {0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (!act[q]) continue;
            if (ub == 0 && threadIdx.x == 0) zp(H, zs, q)[k + i * (m + 1)] = h[q];
            const double a = -h[q];
#pragma unroll
            for (int j = 0; j < J; j++) {
                if (val[j]) {
                    w[q][j].x = a * cur[q][j].x + w[q][j].x;
                    w[q][j].y = a * cur[q][j].y + w[q][j].y;
                    const double2 o = (k < i) ? nxt[q][j] : w[q][j];
                    acc[q] += w[q][j].x * o.x;
                    acc[q] += w[q][j].y * o.y;
                }
            }
        }
        publish(k + 1, acc);
        return true;
    };
    for (int k = 0; k <= i; k += 2) {
        if (!step(k, vk, vn)) return;
        if (k + 1 > i) break;
        step(k + 1, vn, vk);
    }
    double hn[2] = {0.0, 0.0};
    {
        int miss = 0;
        gather2_xcd<J>(gq[0] + (long long)(i + 1) * G, gq[1] + (long long)(i + 1) * G, xslot(0, i + 1),
                       xslot(1, i + 1), G, red, act, err, par, kSpinLimit, abw[0], abw[1], hn, miss);
        if (miss && !(ld_agent_int(abw[0]) & DONE_ABORT) && !(ld_agent_int(abw[1]) & DONE_ABORT)) atomicOr(err, 1);
    }
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if (!act[q]) continue;
        const double hq = sqrt(hn[q]);
        if (ub == 0 && threadIdx.x == 0) {                        // as k_arnoldi_finalize
            DevState *d = dsq[q];
            const int ld = m + 1;
            double *Hc = zp(H, zs, q) + i * ld;
            double *csq = zp(cs, zs, q), *snq = zp(sn, zs, q), *sq = zp(s, zs, q);
            Hc[i + 1] = hq;
            for (int k = 0; k < i; k++) apply_rot(Hc[k], Hc[k + 1], csq[k], snq[k]);
            double c, sv;
            gen_rot(Hc[i], Hc[i + 1], c, sv);
            csq[i] = c;
            snq[i] = sv;
            apply_rot(Hc[i], Hc[i + 1], c, sv);
            apply_rot(sq[i], sq[i + 1], c, sv);
            const double resid = fabs(sq[i + 1]) / d->normb;
            zp(hist, zs, q)[d->hist_len + i] = resid;
            d->resid = resid;
            if (resid < d->tol) {
                d->conv_i = i;
                d->done = DONE_INNER;
            }
        }
        const double inv = (hq != 0.0) ? 1.0 / hq : 0.0;
        double *vout = Vq[q] + (long long)(i + 1) * ldv;
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (val[j]) {
                double2 a = w[q][j];
                a.x = inv * a.x;
                a.y = inv * a.y;
                st2(vout, u0 + j * stride, a);
            }
        }
    }
}

// k_arnoldi_wide -- the same inner iteration for vectors too long for
// k_arnoldi_persist's registers (C4: 11.6M slots): only w stays on chip (kWideJR
// units per thread in registers, kWideJL in LDS), v_k and v_{k+1} are streamed
// (non-temporal) at every step, kWideD units ahead of their use -- 16 B per
// slot and step against the per-step kernels' 32 (w read and written).  Same
// reduction tree as k_dot / k_mgs_step (G blocks of 256 threads, grid-stride
// units, per thread ascending j, block_sum, G partials summed in sum_partials
// order), so it is bit-identical to the per-step path.  Needs every block
// co-resident (host: kWideG blocks, two per CU).
// kWideJS of a thread's units of v_{k+1} are kept in LDS from step k, where they
// are streamed for the next dot, to step k+1, where they are v_k (and v_0 from
// the first dot to step 0): that share of the basis is read from HBM once per
// step instead of twice (LDS: 2 blocks x (kWideJL + kWideJS) x 256 x 16 B)
#ifndef GG_WIDE_STASH
#define GG_WIDE_STASH 14
#endif
constexpr int kWideJR = 40, kWideJL = 5, kWideD = 8, kWideJS = GG_WIDE_STASH;
#ifndef GG_WIDE_NEXT_NT
#define GG_WIDE_NEXT_NT 0
#endif
__global__ __launch_bounds__(kBlock, 2) void k_arnoldi_wide(Gate g, int i, int m, DevState *ds,
                                                            const double *__restrict__ w_in,
                                                            double *__restrict__ V, long long ldv,
                                                            double *H, double *cs, double *sn,
                                                            double *s, double *hist,
                                                            unsigned long long *gran, unsigned long long *hg,
                                                            long long units, int *err, UnitMap um)
{
    constexpr int J = kWideJR + kWideJL;
    if (gated(g)) return;
    if (block_aborted(ds)) return;                            // co-residency (gather_first)
    const int *abortw = &ds->done;
    __shared__ double2 wl[kWideJL * kBlock];
    __shared__ double2 vst[(kWideJS > 0 ? kWideJS : 1) * kBlock];   // v_{k+1} (then v_k) of units j < kWideJS
    const int G = gridDim.x;
    const int stride = G * kBlock;                      // units (vectors < 2^31 units: host check)
    const int u0 = blockIdx.x * kBlock + threadIdx.x;
    // this thread's units u0 + j stride, j < nval
    const int nval = units > u0 ? (int)((units - u0 + stride - 1) / stride) : 0;
    // (no padding skip here: the validity mask costs this kernel its registers
    // -- 148 VGPRs spilled -- at 256 VGPRs; um is unused)
    (void)um;
    auto ok = [&](int j) { return j < nval; };
    double2 wr[kWideJR];
    auto wget = [&](int j) -> double2 { return j < kWideJR ? wr[j] : wl[(j - kWideJR) * kBlock + threadIdx.x]; };
    auto wset = [&](int j, double2 v) {
        if (j < kWideJR) wr[j] = v;
        else wl[(j - kWideJR) * kBlock + threadIdx.x] = v;
    };
    int gpar = 0;                                       // block_sum_pp's LDS row
    auto publish = [&](int k, double acc) {
        acc = block_sum_pp(acc, gpar);
        if (threadIdx.x == 0) st_agent(gran + (long long)k * G + blockIdx.x, (unsigned long long)__double_as_longlong(acc));
    };
    // streaming ring: slot j % kWideD holds unit j's v_k (and v_{k+1}).  The
    // unit offsets are recomputed in every step from a laundered base (not
    // hoisted: 45 live offsets would not fit beside w)
    double2 pk[kWideD], pn[kWideD];
    // v_{k+1} is read again as v_k in the next step: GG_WIDE_NEXT_NT=0 reads it
    // with the default policy (it may stay in the Infinity Cache for that
    // second read), 1 streams it non-temporally like v_k's last read
    // stash: v_k's units j < kWideJS come from LDS (written one step earlier)
    auto fetch = [&](int j, int ub, const double2 *vkp, const double2 *vnp, bool stash) {
        if (j < J && ok(j)) {
            if (stash && j < kWideJS) {
                pk[j % kWideD] = vst[j * kBlock + threadIdx.x];
            } else {
                const dbl2v a = __builtin_nontemporal_load(reinterpret_cast<const dbl2v *>(vkp) + ub + j * stride);
                pk[j % kWideD] = make_double2(a.x, a.y);
            }
            if (vnp) {
                if constexpr (GG_WIDE_NEXT_NT) {
                    const dbl2v c = __builtin_nontemporal_load(reinterpret_cast<const dbl2v *>(vnp) + ub + j * stride);
                    pn[j % kWideD] = make_double2(c.x, c.y);
                } else {
                    pn[j % kWideD] = vnp[ub + j * stride];
                }
            }
        }
    };
    auto vec = [&](const double *p) { return reinterpret_cast<const double2 *>(p); };
    double acc = 0.0;
    {
        int ub = u0;
        asm volatile("" : "+v"(ub));
#pragma unroll
        for (int j = 0; j < kWideD; j++) fetch(j, ub, vec(V), nullptr, false);
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (ok(j)) {
                const double2 wv = vec(w_in)[ub + j * stride];
                wset(j, wv);
                const double2 v0 = pk[j % kWideD];
                acc += wv.x * v0.x;
                acc += wv.y * v0.y;
                if (j < kWideJS) vst[j * kBlock + threadIdx.x] = v0;     // v_0 again at step 0
            }
            fetch(j + kWideD, ub, vec(V), nullptr, false);
        }
    }
    publish(0, acc);                                          // <w, v_0>
    for (int k = 0; k <= i; k++) {
        const double2 *vkp = vec(V + (long long)k * ldv);
        const double2 *vnp = (k < i) ? vec(V + (long long)(k + 1) * ldv) : nullptr;
        int ub = u0;
        asm volatile("" : "+v"(ub));
#pragma unroll
        for (int j = 0; j < kWideD; j++) fetch(j, ub, vkp, vnp, true);    // in flight during the sum
        double h;
        if (k == 0) {
            if (!gather_h_first<true>(gran, hg, G, ds, gpar, h)) return;
        } else {
            h = gather_h<true>(gran + (long long)k * G, hg + k, k, G, err, gpar, abortw);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) H[k + i * (m + 1)] = h;
        const double a = -h;
        acc = 0.0;
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (ok(j)) {
                double2 wv = wget(j);
                const double2 vk = pk[j % kWideD];
                wv.x = a * vk.x + wv.x;
                wv.y = a * vk.y + wv.y;
                wset(j, wv);
                const double2 o = vnp ? pn[j % kWideD] : wv;    // next dot: v_{k+1}, or the norm
                acc += wv.x * o.x;
                acc += wv.y * o.y;
                if (vnp && j < kWideJS) vst[j * kBlock + threadIdx.x] = o;   // v_k of the next step
            }
            fetch(j + kWideD, ub, vkp, vnp, true);
        }
        publish(k + 1, acc);
    }
    const double hn = sqrt(gather_h<true>(gran + (long long)(i + 1) * G, hg + i + 1, i + 1, G, err, gpar, abortw));
    if (blockIdx.x == 0 && threadIdx.x == 0) {               // as k_arnoldi_finalize
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
        if (resid < ds->tol) {
            ds->conv_i = i;
            ds->done = DONE_INNER;
        }
    }
    const double inv = (hn != 0.0) ? 1.0 / hn : 0.0;
    double2 *vout = reinterpret_cast<double2 *>(V + (long long)(i + 1) * ldv);
#pragma unroll
    for (int j = 0; j < J; j++) {
        if (ok(j)) {
            double2 a = wget(j);
            a.x = inv * a.x;
            a.y = inv * a.y;
            vout[u0 + j * stride] = a;
        }
    }
}

// y = H(0:k,0:k)^-1 s(0:k)  (Update, src/gmres.cu:93-116); k = conv_i or nit-1.
// One wave: lane j keeps y[j] and row j of H in registers; for i = k..0 lane i
// divides, the value is broadcast, lanes j < i subtract -- per element the same
// operations in the same order as the serial back-substitution.
constexpr int kMaxRestart = 64;
__global__ __launch_bounds__(64) void k_update_y(Gate g, int m, DevState *ds, const double *H,
                                                 const double *s, double *y, long long zs = 0)
{
    if (gated_z(g, zs, blockIdx.y)) return;
    ds = zp(ds, zs, blockIdx.y);
    H = zp(H, zs, blockIdx.y);
    s = zp(s, zs, blockIdx.y);
    y = zp(y, zs, blockIdx.y);
    const int lane = threadIdx.x;
    const int k = (ds->done & DONE_INNER) ? ds->conv_i : ds->nit - 1;
    if (lane == 0) ds->upd_k = k;
    const int ld = m + 1;
    double yj = lane <= k ? s[lane] : 0.0;
    double hrow[kMaxRestart];
#pragma unroll
    for (int i = 0; i < kMaxRestart; i++) hrow[i] = (lane <= k && i <= k) ? H[lane + i * ld] : 0.0;
#pragma unroll
    for (int i = kMaxRestart - 1; i >= 0; i--) {
        if (i > k) continue;                              // uniform
        if (lane == i) yj = yj / hrow[i];
        const double yi = __shfl(yj, i, 64);
        if (lane < i) yj = yj - hrow[i] * yi;
    }
    if (lane <= k) y[lane] = yj;
}

// the same for restarts above kMaxRestart: one thread, serial
__global__ void k_update_y_serial(Gate g, int m, DevState *ds, const double *H, const double *s,
                                  double *y, long long zs = 0)
{
    if (gated_z(g, zs, blockIdx.y)) return;
    ds = zp(ds, zs, blockIdx.y);
    H = zp(H, zs, blockIdx.y);
    s = zp(s, zs, blockIdx.y);
    y = zp(y, zs, blockIdx.y);
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
                                                     long long units, UnitMap um, long long zs = 0)
{
    if (gated_z(g, zs, blockIdx.y)) return;
    ds = zp(ds, zs, blockIdx.y);
    y = zp(y, zs, blockIdx.y);
    V = zp(V, zs, blockIdx.y);
    acc = zp(acc, zs, blockIdx.y);
    const int k = ds->upd_k;
    for (long long u = blockIdx.x * (long long)kBlock + threadIdx.x; u < units;
         u += (long long)gridDim.x * kBlock) {
        if (!unit_real(um, u)) continue;                      // padding: +0 stays +0
        double2 a = ld2(acc, u);
        // eight basis vectors' loads in flight at a time, added in ascending j
        for (int j0 = 0; j0 <= k; j0 += 8) {
            double2 vv[8];
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (j0 + q <= k) vv[q] = ld2_nt(V + (j0 + q) * ldv, u);
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (j0 + q <= k) {
                    const double yj = y[j0 + q];
                    a.x = a.x + vv[q].x * yj;
                    a.y = a.y + vv[q].y * yj;
                }
        }
        st2(acc, u, a);
    }
}

// beta = ||r|| after a restart; history; j += nit
__global__ void k_end_cycle(const double *part, int G, DevState *ds, double *hist, long long zs = 0)
{
    part = zp(part, zs, blockIdx.y);
    ds = zp(ds, zs, blockIdx.y);
    hist = zp(hist, zs, blockIdx.y);
    if (ds->done) {
        // the cycle that converged inside has applied its update: a cycle
        // enqueued behind it must not apply it again
        if (threadIdx.x == 0 && (ds->done & DONE_INNER)) ds->done |= DONE_FINAL;
        return;
    }
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
#ifndef GG_REDUCE_UPT
#define GG_REDUCE_UPT 4
#endif
int reduce_grid(long long units)
{
    // vectors too long for k_arnoldi_persist's registers at 1024 blocks (more
    // than 8 units per thread) reduce over kWideG blocks, two per CU, so that
    // k_arnoldi_wide can keep w on chip with the same tree
    if (units > (long long)1024 * kBlock * 8) return kWideG;
    long long g = (units + kBlock * GG_REDUCE_UPT - 1) / (kBlock * GG_REDUCE_UPT);   // >= 2*UPT elements / thread
    if (g < 1) g = 1;
    if (g > 1024) g = 1024;
    return (int)g;
}

void launch_fill_u64(unsigned long long *p, long long n, unsigned long long v, hipStream_t st)
{
    k_fill_u64<<<blocks_for(n, kBlock, 4096), kBlock, 0, st>>>(p, n, v);
}
void launch_transient_step(int n, int nsrc, const int *kind, const int *dptr, const double *data, int it,
                           double h, double *u, const int *src_ptr, const int *src_idx, const double *cdiag,
                           const double *x, double *w, hipStream_t st)
{
    if (nsrc > 0) k_sources<<<(nsrc + kBlock - 1) / kBlock, kBlock, 0, st>>>(nsrc, kind, dptr, data, it, h, u);
    if (n > 0)
        k_transient_rhs<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(n, src_ptr, src_idx, u, cdiag, x, w);
}
void launch_transient_step_csr(int n, int nsrc, const int *kind, const int *dptr, const double *data, int it,
                               double h, double *u, const int *bp, const int *bi, const double *bv,
                               const int *rp, const int *ri, const double *rv, const double *x, double *w,
                               hipStream_t st)
{
    if (nsrc > 0) k_sources<<<(nsrc + kBlock - 1) / kBlock, kBlock, 0, st>>>(nsrc, kind, dptr, data, it, h, u);
    if (n > 0)
        k_transient_rhs_csr<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(n, bp, bi, bv, u, rp, ri, rv, x, w);
}

void launch_taps(int ntap, const int *tap, const double *x, double *mx, double *mn, double *sm, int mode,
                 double npts, hipStream_t st)
{
    if (ntap > 0) k_taps<<<(ntap + kBlock - 1) / kBlock, kBlock, 0, st>>>(ntap, tap, x, mx, mn, sm, mode, npts);
}
void launch_gather_ports(int nport, const int *port, const double *x, double *out, hipStream_t st)
{
    if (nport > 0) k_gather_ports<<<(nport + kBlock - 1) / kBlock, kBlock, 0, st>>>(nport, port, x, out);
}

int trsv_flow_max_blocks()
{
    int dev = 0, per = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    int per2 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_trsv_flow<false>, kBlock, 0) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per2, k_trsv_flow<true>, kBlock, 0) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return std::min(per, per2) * cus;
}
int ilu0_columns_max_blocks()
{
    int dev = 0, per = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_ilu0_columns, kBlock, 0) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return per * cus;
}
void launch_ilu0_columns(int n, const int *cp, const int *ri, const double *cv0, double *cv, int *level,
                         int *done, int *err, int blocks, hipStream_t st)
{
    k_ilu0_columns<<<blocks, kBlock, 0, st>>>(n, cp, ri, cv0, cv, level, done, err);
}
int iluk_wave_max_blocks()
{
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_iluk_wave, kBlock, 0) != hipSuccess) return 0;
    return cus * per;
}
int iluk_wave_cap() { return kIlukCap; }
void launch_iluk_scatter(int n, const int *arp, const int *aci, const double *av, const long long *prow,
                         const int *pcol, double *val, hipStream_t st)
{
    k_iluk_scatter<<<blocks_for(n, kBlock, 8192), kBlock, 0, st>>>(n, arp, aci, av, prow, pcol, val);
}
void launch_iluk_wave(int n, const long long *prow, const int *nl, const int *pcol, double *val, double *dinv,
                      int *done, const int *rows_short, int nshort, const int *rows_long, int nlong,
                      int long_blocks, int *scratch, int *err, int blocks, hipStream_t st)
{
    k_iluk_wave<<<blocks, kBlock, 0, st>>>(n, prow, nl, pcol, val, dinv, done, rows_short, nshort, rows_long,
                                           nlong, long_blocks, scratch, err);
}
void launch_gather(const double *in, const long long *idx, double *out, long long n, hipStream_t st,
                   double *fill0, double *fill1, long long nfill)
{
    if (!fill0 || !fill1) nfill = 0;
    k_gather<<<blocks_for(std::max(n, nfill), kBlock, 8192), kBlock, 0, st>>>(
        in, idx, out, n, reinterpret_cast<unsigned long long *>(fill0), reinterpret_cast<unsigned long long *>(fill1),
        nfill);
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
void launch_sub_seq(Gate g, const DevCsr &C, const double *x, const double *in, double *out,
                    hipStream_t st, double *fill0, double *fill1, int nfill)
{
    const int n = std::max(C.n, nfill);
    if (n == 0) return;
    k_sub_seq<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(
        g, C.n, C.rp.p, C.ci.p, C.v.p, x, in, out, reinterpret_cast<unsigned long long *>(fill0),
        reinterpret_cast<unsigned long long *>(fill1), nfill);
}

void launch_sep_flow(Gate g, int ntask, const int4 *tasks, const int *rows, const SepFlow &f, int *err, hipStream_t st)
{
    if (ntask <= 0) return;
    // one block per CU at most (every waiting lane polls; all co-resident), a wave per task
    static const int cap = [] {
        int dev = 0, c = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_sep_flow, kBlock, 0) != hipSuccess) per = 0;
        return per > 0 ? c : 0;
    }();
    GG_REQUIRE(cap > 0, GG_EHIP, "k_sep_flow cannot be resident");
    const long long need = ((long long)ntask + kBlock / 64 - 1) / (kBlock / 64);
    const int blocks = (int)std::min<long long>(cap, need);
    k_sep_flow<<<blocks, kBlock, 0, st>>>(g, ntask, tasks, rows, f, err);
}
void launch_allgather_local(const ShardPtrs &b, int P, long long off, long long cnt, hipStream_t st)
{
    if (P <= 1 || cnt == 0) return;
    k_allgather_local<<<blocks_for(P * cnt, kBlock, 8192), kBlock, 0, st>>>(b, P, off, cnt);
}
void launch_ipc_allgather(const IpcPeers &pp, int me, int P, double *buf, long long cnt,
                          unsigned long long seq, long long capd, int *err, hipStream_t st)
{
    // every rank must pick the same block count for the same cnt
    const int nb = (int)std::min<long long>(kIpcXB, std::max<long long>(1, (cnt + 2047) / 2048));
    k_ipc_allgather<<<nb, kBlock, 0, st>>>(pp, me, P, buf, cnt, seq, capd, err, nullptr, nullptr, nullptr, nullptr,
                                           0);
}
void launch_ipc_gather_allgather(const IpcPeers &pp, int me, int P, const double *x, const long long *gidx,
                                 double *buf, long long cnt, unsigned long long seq, long long capd, int *err,
                                 double *f0, double *f1, long long nf, hipStream_t st)
{
    // the block count depends on cnt only, as launch_ipc_allgather's (every rank the same)
    const int nb = (int)std::min<long long>(kIpcXB, std::max<long long>(1, (cnt + 2047) / 2048));
    if (!f0 || !f1) nf = 0;
    k_ipc_allgather<<<nb, kBlock, 0, st>>>(pp, me, P, buf, cnt, seq, capd, err, x, gidx,
                                           reinterpret_cast<unsigned long long *>(f0),
                                           reinterpret_cast<unsigned long long *>(f1), nf);
}
bool launch_dd_spmv_x(Gate g, const DdSpmvCall &c, hipStream_t st)
{
    const DevCsr &AI = *c.AI, &AS = *c.AS;
    if (AI.panel || AS.panel || c.P < 2 || c.P > kMaxShards) return false;
    DdSpmvX a{};
    a.pp = c.pp;
    a.me = c.me;
    a.P = c.P;
    a.loop = c.loop ? 1 : 0;
    a.halo = c.halo;
    a.cnt = c.cnt;
    a.capd = c.capd;
    a.seq = c.seq;
    a.err = c.err;
    a.gidx = c.gidx;
    a.arrived = c.arrived;
    // the exchange's block count depends on cnt only (every rank the same, as
    // launch_ipc_gather_allgather's); loopback: k_gather_allgather_local's span
    a.nbx = c.loop ? (int)std::min<long long>(kIpcXB, std::max<long long>(1, ((long long)c.P * c.cnt + 2047) / 2048))
                   : (int)std::min<long long>(kIpcXB, std::max<long long>(1, (c.cnt + 2047) / 2048));
    a.target = c.epoch * (unsigned long long)a.nbx;
    auto rows = [](const DevCsr &A, int &sell, int &n, int &nb, const int *&ptr, const int *&rp, const int *&ci,
                   const double *&v) {
        sell = A.sell ? 1 : 0;
        n = A.n;
        if (A.sell) {
            nb = A.nslice;
            ptr = A.sptr.p;
            rp = nullptr;
            ci = A.sci.p;
            v = A.sv.p;
            return (A.nslice + kBlock / 64 - 1) / (kBlock / 64);
        }
        nb = A.nblk;
        ptr = A.blk.p;
        rp = A.rp.p;
        ci = A.ci.p;
        v = A.v.p;
        return A.nblk;
    };
    a.nbi = AI.nblk == 0 ? 0 : rows(AI, a.i_sell, a.i_n, a.i_nb, a.i_ptr, a.i_rp, a.i_ci, a.i_v);
    a.nbs = AS.nblk == 0 ? 0 : rows(AS, a.s_sell, a.s_n, a.s_nb, a.s_ptr, a.s_rp, a.s_ci, a.s_v);
    a.x = c.x;
    a.b = c.b;
    a.y = c.y;
    a.S0 = c.S0;
    const int grid = a.nbx + a.nbi + a.nbs;
    if (c.resid) k_dd_spmv_x<true><<<grid, kBlock, 0, st>>>(g, a);
    else k_dd_spmv_x<false><<<grid, kBlock, 0, st>>>(g, a);
    return true;
}
void launch_gather_allgather_local(const ShardPtrs &b, const IdxPtrs &gi, int P, long long off, long long cnt,
                                   const FillPtrs &fl, long long nf, hipStream_t st)
{
    if (P * cnt == 0 && nf == 0) return;
    k_gather_allgather_local<<<blocks_for(std::max(P * cnt, nf), kBlock, 8192), kBlock, 0, st>>>(b, gi, P, off, cnt,
                                                                                             fl, nf);
}
void launch_scatter_idx(const double *in, const long long *src, const long long *dst, double *out,
                        long long n, hipStream_t st)
{
    if (n == 0) return;
    k_scatter_idx<<<blocks_for(n, kBlock, 8192), kBlock, 0, st>>>(in, src, dst, out, n);
}

void launch_fingerprint(const void *p, long long nw, unsigned long long *out, hipStream_t st)
{
    if (nw <= 0) return;
    k_fingerprint<<<blocks_for(nw, kBlock, 2048), kBlock, 0, st>>>(static_cast<const unsigned *>(p), nw, out);
}
void launch_f64_to_f32(Gate g, const double *in, float *out, int n, hipStream_t st)
{
    k_f64_to_f32<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, out, n);
}
void launch_f32_to_f64(Gate g, const float *in, double *out, int n, hipStream_t st)
{
    k_f32_to_f64<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, out, n);
}
void launch_mul(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st)
{
    k_mul<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, out, n);
}
void launch_div(Gate g, const double *in, const double *s, double *out, int n, hipStream_t st)
{
    k_div<<<blocks_for(n, kBlock, 1 << 30), kBlock, 0, st>>>(g, in, s, out, n);
}

void launch_spmv(Gate g, const DevCsr &A, const double *x, const double *b, double *y, bool resid,
                 hipStream_t st, const double *ydiv)
{
    if (A.nblk == 0) return;
    if (A.panel && A.rtile && !resid && !ydiv && x != y) {
        // row tiles: one launch, each block its rows' segments panel by panel
        k_spmv_rtile<<<A.rtile, kBlock, 0, st>>>(g, A.rt_sub.p, A.pblk.p, A.seg_row.p, A.seg_ptr.p, A.pci.p, A.pv.p, x,
                                                  y, A.zero_rows.p, A.nzero);
        return;
    }
    if (A.panel && !resid && !ydiv && x != y) {
        // column panels: one launch per panel over its segment blocks
        for (int p = 0; p < A.npanel; p++) {
            const int nb = A.pan_blk_h[p + 1] - A.pan_blk_h[p];
            if (nb > 0)
                k_spmv_panel<<<nb, kBlock, 0, st>>>(g, A.pblk.p + A.pan_blk_h[p], A.seg_row.p, A.seg_ptr.p, A.pci.p,
                                                     A.pv.p, x, y, A.zero_rows.p, p == 0 ? A.nzero : 0);
        }
        return;
    }
#define GG_SPMV(R, D)                                                                                  \
    do {                                                                                               \
        if (A.sell)                                                                                    \
            k_spmv_sell<R, D><<<(A.nslice + kBlock / 64 - 1) / (kBlock / 64), kBlock, 0, st>>>(        \
                g, A.n, A.nslice, A.sptr.p, A.sci.p, A.sv.p, x, b, y, ydiv, nullptr);                  \
        else                                                                                           \
            k_spmv_stream<R, D><<<A.nblk, kBlock, 0, st>>>(g, A.blk.p, A.rp.p, A.ci.p, A.v.p, x, b, y, \
                                                          ydiv);                                       \
    } while (0)
    if (ydiv) {
        if (resid) GG_SPMV(true, true);
        else GG_SPMV(false, true);
    } else {
        if (resid) GG_SPMV(true, false);
        else GG_SPMV(false, false);
    }
#undef GG_SPMV
}

bool launch_spmv_xdiv(Gate g, const DevCsr &A, const double *x, const double *xdiv, double *y, hipStream_t st,
                      const double *ydiv, double *fill, int nfill)
{
    if (!A.sell || !ydiv) return false;
    // the caller relies on the fill having happened (DevTri::prefilled): when
    // it cannot ride on the SpMV's lanes it gets a launch of its own
    if (fill && (A.nblk == 0 || nfill > A.nslice * 64)) {
        k_fill_gated<<<blocks_for(nfill, kBlock, 8192), kBlock, 0, st>>>(
            g, reinterpret_cast<unsigned long long *>(fill), nfill, kSentinel);
        fill = nullptr;
    }
    if (A.nblk == 0) return true;
    if (!fill) nfill = 0;
    k_spmv_sell<false, true, true><<<(A.nslice + kBlock / 64 - 1) / (kBlock / 64), kBlock, 0, st>>>(
        g, A.n, A.nslice, A.sptr.p, A.sci.p, A.sv.p, x, nullptr, y, ydiv, xdiv,
        reinterpret_cast<unsigned long long *>(fill), fill ? nfill : 0);
    return true;
}

template <bool FWD, int DIV>
int wave3d_max_blocks()
{
    static int cached = -1;
    if (cached < 0) {
        int dev = 0, per = 0, cus = 0;
        (void)hipGetDevice(&dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_trsv_wave2d<FWD, DIV, false, true>,
                                                         WaveCfg<DIV, true>::THREADS, 0) != hipSuccess)
            per = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cached = std::max(1, per * cus);
    }
    return cached;
}

template <bool FWD, int DIV>
int tile3d_max_blocks()
{
    static int cached = -1;
    if (cached < 0) {
        int dev = 0, per = 0, cus = 0;
        (void)hipGetDevice(&dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_trsv_tile3d<FWD, DIV>, TileCfg<DIV>::THREADS, 0) !=
            hipSuccess)
            per = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cached = std::max(1, per * cus);
    }
    return cached;
}

int tile_batch_steps() { return GG_TILE_BATCH; }

// tests: GG_TILE_GRID = workgroups of the tile solve (beyond what can be
// resident: the task queue must still drain it)
// the tile solve's mode: static (0) unless the triangle fell back to the
// queue (1); GG_TILE_QUEUE=1 forces the queue (tests, A/B)
static int tile_dyn(const DevTri &T)
{
    const char *e = std::getenv("GG_TILE_QUEUE");
    return (T.tile_queue || (e && e[0] == '1')) ? 1 : 0;
}
static int tile_grid_override(int g)
{
    const char *e = std::getenv("GG_TILE_GRID");
    return e && atoi(e) > 0 ? atoi(e) : g;
}
// tests: GG_PERSIST_TEST_LDS = dynamic LDS bytes added to the persistent
// orthogonalization launches, so that fewer blocks fit than the grid needs
// (the co-residency abort and the per-step rerun, kernels.hip gather_first)
static size_t persist_test_lds()
{
    const char *e = std::getenv("GG_PERSIST_TEST_LDS");
    return e ? (size_t)std::max(0, atoi(e)) : 0;
}

int wave_batch_steps(int div, bool d3, int skew)
{
    // WD_MUL streams as many arrays as WD_HW (y in d's place): the same batches
    const bool hw = div == WD_HW || div == WD_MUL;
    if (d3) return div == WD_UNIT ? WaveCfg<WD_UNIT, true>::B : hw ? WaveCfg<WD_HW, true>::B
                                                                   : WaveCfg<WD_RCP, true>::B;
    if (skew == 2)
        return div == WD_UNIT ? WaveCfg<WD_UNIT, false, 2>::B : hw ? WaveCfg<WD_HW, false, 2>::B
                                                                   : WaveCfg<WD_RCP, false, 2>::B;
    if (skew == 3)
        return div == WD_UNIT ? WaveCfg<WD_UNIT, false, 3>::B : hw ? WaveCfg<WD_HW, false, 3>::B
                                                                   : WaveCfg<WD_RCP, false, 3>::B;
    if (div == WD_UFMA) return WaveCfg<WD_UFMA>::B;
    if (div == WD_SFMA) return WaveCfg<WD_SFMA>::B;
    return div == WD_UNIT ? WaveCfg<WD_UNIT>::B : hw ? WaveCfg<WD_HW>::B : WaveCfg<WD_RCP>::B;
}

bool fused_spmv_ok(const DevTri &T, const DevCsr &A)
{
    const Wave2D &w = T.wl;
    return T.kind == DevTri::WAVE2D && T.lower && !T.tail && w.ok && !w.tile && w.nz == 1 && w.skew == 1 && !T.trace &&
           (T.eff_div() == WD_UFMA || T.eff_div() == WD_SFMA) && A.sell && w.T % kFsGroup == 0 &&
           (long long)A.nslice >= (long long)w.nbands * w.T && (long long)A.n >= (long long)w.nbands * w.T * 64;
}

void launch_trsv_spmv(Gate g, DevTri &T, const DevCsr &A, const double *v, double *w, double *x, int *err,
                      hipStream_t st, const double *ydiv, const double *xdiv)
{
    const Wave2D &wl = T.wl;
    const size_t nflag = (size_t)wl.nbands * (wl.T / kFsGroup);
    if (T.fcnt.n < nflag) {
        T.fcnt.alloc(nflag);
        GG_HIP(hipMemsetAsync(T.fcnt.p, 0, nflag * sizeof(unsigned long long), st));
    }
    // every CU the bands leave free computes b (the SpMV blocks wait on nothing)
    static const int cus = [] {
        int dev = 0, c = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c;
    }();
    const int ns = std::max(64, cus - wl.nbands);
    FusedSpmv fs;
    fs.sptr = A.sptr.p;
    fs.sci = A.sci.p;
    fs.sv = A.sv.p;
    fs.v = v;
    fs.w = w;
    fs.cnt = T.fcnt.p;
    fs.ydiv = ydiv;
    fs.xdiv = xdiv;
    fs.n = A.n;
    fs.ns = ns;
    if (T.eff_div() == WD_UFMA)
        k_trsv_wave2d_spmv<WD_UFMA><<<wl.nbands + ns, WaveCfg<WD_UFMA>::THREADS, 0, st>>>(
            g, wl.T, wl.nbands, T.c1.p, T.c2.p, nullptr, nullptr, x, T.bnd.p, err, wl.P2, fs);
    else   // the split engine's non-unit L, coefficients and b pre-scaled by RN(1/d)
        k_trsv_wave2d_spmv<WD_SFMA><<<wl.nbands + ns, WaveCfg<WD_SFMA>::THREADS, 0, st>>>(
            g, wl.T, wl.nbands, T.c1s.p, T.c2s.p, T.rw.p, nullptr, x, T.bnd.p, err, wl.P2, fs);
}

static void launch_trsv_one(Gate g, DevTri &T, const double *b, double *x, int *err, hipStream_t st);

void launch_trsv(Gate g, DevTri &T, const double *b, double *x, int *err, hipStream_t st)
{
    if (!T.tail) {
        launch_trsv_one(g, T, b, x, err, st);
        return;
    }
    // bordered grid: tail, coupling, grid (forward); grid, tail (backward)
    const int e = T.eff_div();
    const bool fm = e == WD_UFMA || e == WD_SFMA;
    // the tail rows divide as the grid's do (GG_DIV_FMA: the fused-order copy)
    DevTri &tl = fm ? *T.tail_fma : *T.tail;
    tl.fast = 0;
    tl.mul = e == WD_MUL;
    if (tl.lev_ptr_d.p) {
        // a small tail: one workgroup for the tail and the coupling
        auto tail_small = [&](bool coup) {
            k_tail_small<<<1, 1024, 0, st>>>(g, (int)tl.lev_ptr.size() - 1, tl.lev_ptr_d.p, tl.lev_rows.p,
                                             tl.off.rp.p, tl.off.ci.p, tl.off.v.p, tl.d.p,
                                             (tl.mul || tl.fmrow) ? tl.rw.p : nullptr, tl.fmrow ? 1 : 0, b, x,
                                             coup ? T.ncoup : 0, T.cslot.p, T.crp.p, T.cci.p, T.cv.p,
                                             const_cast<double *>(b), fm ? 1 : 0);
        };
        if (T.lower) {
            tail_small(true);
            launch_trsv_one(g, T, b + T.bofs, x + T.bofs, err, st);
        } else {
            launch_trsv_one(g, T, b + T.bofs, x + T.bofs, err, st);
            tail_small(false);
        }
        return;
    }
    if (T.lower) {
        launch_trsv_one(g, tl, b, x, err, st);
        if (T.ncoup)
            k_border_sub<<<(T.ncoup + kBlock - 1) / kBlock, kBlock, 0, st>>>(
                g, T.ncoup, T.cslot.p, T.crp.p, T.cci.p, T.cv.p, x, const_cast<double *>(b), fm ? 1 : 0);
        launch_trsv_one(g, T, b + T.bofs, x + T.bofs, err, st);
    } else {
        launch_trsv_one(g, T, b + T.bofs, x + T.bofs, err, st);
        launch_trsv_one(g, tl, b, x, err, st);
    }
}

static void launch_trsv_one(Gate g, DevTri &T, const double *b, double *x, int *err, hipStream_t st)
{
    if (T.kind == DevTri::LEVEL) {
        const int nlev = (int)T.lev_ptr.size() - 1;
        static const int flow_blocks = trsv_flow_max_blocks();
        const char *lv = getenv("GG_TRSV_LEVELS");         // 1: one launch per level
        const bool per_level = lv && atoi(lv) != 0;
        const int nrows = T.lev_ptr[nlev];
        if (!per_level && b != x && flow_blocks > 0 && nlev > 1 && nrows > 0) {
            // few resident waves: every waiting lane polls, so the grid is
            // capped at GG_FLOW_BPC blocks per CU (default 1)
            static const int cus = [] {
                int dev = 0, c = 0;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
                return c;
            }();
            // one block per CU where the levels are narrow (every waiting lane
            // polls; more pollers slow the hand-offs), up to occupancy where a
            // level holds more tasks than 4 waves per CU can take (C3: 3,100
            // tasks per level, 0.66 ms per solve at 8 blocks per CU vs 2.1 ms at 1)
            const char *bpc_s = getenv("GG_FLOW_BPC");
            const long long per_level = (T.ntask + nlev - 1) / std::max(nlev, 1);
            const long long wave_slots = 4LL * std::max(cus, 1);          // 4 waves per block, 1 block per CU
            // (the randomly permuted PG split, 1,100 tasks per level: 2 blocks per
            // CU 84 / 102 us for L / U against 95 / 127 at 4 and 102 / 131 at 8,
            // profiles/r04/r04s_pgr_bpc*.json -- so the extra factor 2 only beyond
            // two waves per slot)
            const long long wpl = (per_level + wave_slots - 1) / wave_slots;
            const int bpc = bpc_s ? std::max(1, atoi(bpc_s))
                                  : per_level <= wave_slots ? 1
                                  : (int)std::min<long long>(8, per_level > 2 * wave_slots ? 2 * wpl : wpl);
            const long long need = ((long long)T.ntask + kBlock / 64 - 1) / (kBlock / 64);   // a wave per task
            const int blocks = (int)std::min<long long>(std::min<long long>(flow_blocks, (long long)bpc * std::max(cus, 1)), need);
            if (!T.prefilled)
                k_fill_gated<<<blocks_for(nrows, kBlock, 8192), kBlock, 0, st>>>(
                    g, reinterpret_cast<unsigned long long *>(x), nrows, kSentinel);
            if (T.ell)
                k_trsv_flow<true><<<blocks, kBlock, 0, st>>>(g, T.ntask, T.tasks.p, T.lev_rows.p, T.off.rp.p,
                                                             T.off.ci.p, T.off.v.p, T.d.p, b, x, err,
                                                             (T.mul || T.fmrow) ? T.rw.p : nullptr, T.fmrow ? 1 : 0,
                                                             T.eci.p, T.ev.p);
            else
                k_trsv_flow<false><<<blocks, kBlock, 0, st>>>(g, T.ntask, T.tasks.p, T.lev_rows.p, T.off.rp.p,
                                                              T.off.ci.p, T.off.v.p, T.d.p, b, x, err,
                                                              (T.mul || T.fmrow) ? T.rw.p : nullptr, T.fmrow ? 1 : 0,
                                                              nullptr, nullptr);
            return;
        }
        for (int l = 0; l < nlev; l++) {
            const int cnt = T.lev_ptr[l + 1] - T.lev_ptr[l];
            if (cnt == 0) continue;
            k_trsv_level<<<(cnt + kBlock - 1) / kBlock, kBlock, 0, st>>>(
                g, cnt, T.lev_rows.p + T.lev_ptr[l], T.off.rp.p, T.off.ci.p, T.off.v.p, T.d.p, b, x,
                (T.mul || T.fmrow) ? T.rw.p : nullptr, T.fmrow ? 1 : 0);
        }
    } else if (T.kind == DevTri::WAVE2D) {
        const Wave2D &w = T.wl;
        const int div = T.eff_div();
        // WD_MUL / WD_SFMA stream y = RN(1/d) in d's place
        const double *dv = (div == WD_UNIT || div == WD_UFMA) ? nullptr
                         : (div == WD_MUL || div == WD_SFMA) ? T.rw.p : T.dw.p;
        const double *rv = div == WD_RCP ? T.rw.p : nullptr;
        if ((div == WD_UFMA || div == WD_SFMA) && !w.tile) {
            // GG_DIV_FMA on a 2D grid (build_tri admits unskewed ones in canonical order)
            dim3 grid(w.nbands * (T.lower ? 1 : GG_WAVE_XCD));
            const double *k1 = div == WD_SFMA ? T.c1s.p : T.c1.p, *k2 = div == WD_SFMA ? T.c2s.p : T.c2.p;
            if (w.skew > 1) {
                // ILU(k) grids (skewed lanes): the fills pre-scaled with U's coefficients
                const double *f1 = div == WD_SFMA ? T.ce1s.p : T.ce1.p, *f2 = div == WD_SFMA ? T.ce2s.p : T.ce2.p;
#define GG_FMA_SKEW_LAUNCH(FWD, DIV, S)                                                            \
    k_trsv_wave2d<FWD, DIV, false, false, S, false><<<grid, WaveCfg<DIV, false, S>::THREADS, 0, st>>>( \
        g, w.T, w.nbands, b, k1, k2, dv, rv, x, T.bnd.p, err, nullptr, 1, w.P2, nullptr, nullptr, f1, f2)
                if (T.lower && div == WD_UFMA) {
                    if (w.skew == 2) GG_FMA_SKEW_LAUNCH(true, WD_UFMA, 2);
                    else GG_FMA_SKEW_LAUNCH(true, WD_UFMA, 3);
                } else if (!T.lower && div == WD_SFMA) {
                    if (w.skew == 2) GG_FMA_SKEW_LAUNCH(false, WD_SFMA, 2);
                    else GG_FMA_SKEW_LAUNCH(false, WD_SFMA, 3);
                } else if (T.lower && div == WD_SFMA) {
                    if (w.skew == 2) GG_FMA_SKEW_LAUNCH(true, WD_SFMA, 2);
                    else GG_FMA_SKEW_LAUNCH(true, WD_SFMA, 3);
                } else {
                    std::abort();   // build_tri: no unit upper triangle
                }
#undef GG_FMA_SKEW_LAUNCH
                return;
            }
#define GG_FMA_LAUNCH(FWD, DIV, TR)                                                                \
    k_trsv_wave2d<FWD, DIV, TR><<<grid, WaveCfg<DIV>::THREADS, 0, st>>>(                           \
        g, w.T, w.nbands, b, k1, k2, dv, rv, x, T.bnd.p, err, T.trace, 1, w.P2, nullptr, nullptr,   \
        nullptr, nullptr)
            // (T.il needs no instantiation of its own: the fused rows take the
            // in-line term first in either canonical order)
            if (T.lower && div == WD_UFMA) {
                if (T.trace) GG_FMA_LAUNCH(true, WD_UFMA, true);
                else GG_FMA_LAUNCH(true, WD_UFMA, false);
            } else if (!T.lower && div == WD_SFMA) {
                if (T.trace) GG_FMA_LAUNCH(false, WD_SFMA, true);
                else GG_FMA_LAUNCH(false, WD_SFMA, false);
            } else if (T.lower && div == WD_SFMA) {
                GG_FMA_LAUNCH(true, WD_SFMA, false);      // the split engine's non-unit L
            } else
#undef GG_FMA_LAUNCH
                std::abort();   // build_tri: no unit upper triangle
        } else if (w.tile) {
            // 3D tiles: persistent, every workgroup co-resident (tiles wait on tiles)
            const int ntask = w.nbands;
            const bool sc = div == WD_SFMA;     // GG_DIV_FMA's U: coefficients pre-scaled by RN(1/d)
            const double *k1 = sc ? T.c1s.p : T.c1.p, *k2 = sc ? T.c2s.p : T.c2.p, *k0 = sc ? T.c0s.p : T.c0.p;
#define GG_TILE_LAUNCH(FWD, DIV)                                                                   \
    do {                                                                                           \
        const int grid = std::min(std::min(ntask, tile_grid_override(tile3d_max_blocks<FWD, DIV>())), \
                                  kTileDummyBlocks);                                                     \
        if (T.trace)                                                                               \
            k_trsv_tile3d<FWD, DIV, true><<<grid, TileCfg<DIV>::THREADS, 0, st>>>(                 \
                g, w.T, w.NJ, w.NK, T.order.p, b, k1, k2, dv, rv, k0, x, T.bnd.p, err,              \
                T.trace, tile_dyn(T));                                                             \
        else                                                                                       \
            k_trsv_tile3d<FWD, DIV><<<grid, TileCfg<DIV>::THREADS, 0, st>>>(                       \
                g, w.T, w.NJ, w.NK, T.order.p, b, k1, k2, dv, rv, k0, x, T.bnd.p, err,              \
                nullptr, tile_dyn(T));                                                             \
    } while (0)
            if (div == WD_UFMA || div == WD_SFMA) {
                // GG_DIV_FMA (build_tri admits the unit L and a non-unit U)
                if (T.lower && div == WD_UFMA) GG_TILE_LAUNCH(true, WD_UFMA);
                else if (!T.lower && div == WD_SFMA) GG_TILE_LAUNCH(false, WD_SFMA);
                else std::abort();
            } else if (T.lower) {
                if (div == WD_UNIT) GG_TILE_LAUNCH(true, WD_UNIT);
                else if (div == WD_HW) GG_TILE_LAUNCH(true, WD_HW);
                else if (div == WD_MUL) GG_TILE_LAUNCH(true, WD_MUL);
                else GG_TILE_LAUNCH(true, WD_RCP);
            } else {
                if (div == WD_UNIT) GG_TILE_LAUNCH(false, WD_UNIT);
                else if (div == WD_HW) GG_TILE_LAUNCH(false, WD_HW);
                else if (div == WD_MUL) GG_TILE_LAUNCH(false, WD_MUL);
                else GG_TILE_LAUNCH(false, WD_RCP);
            }
#undef GG_TILE_LAUNCH
        } else if (w.nz == 1) {
            dim3 grid(w.nbands * (T.lower ? 1 : GG_WAVE_XCD));
#define GG_WAVE_LAUNCH_S(FWD, DIV, S, IL)                                                          \
    k_trsv_wave2d<FWD, DIV, false, false, S, IL><<<grid, WaveCfg<DIV, false, S>::THREADS, 0, st>>>( \
        g, w.T, w.nbands, b, T.c1.p, T.c2.p, dv, rv, x, T.bnd.p, err, nullptr, 1, w.P2, nullptr,   \
        nullptr, T.ce1.p, T.ce2.p)
#define GG_WAVE_LAUNCH(FWD, DIV)                                                                   \
    do {                                                                                           \
        if (T.trace && w.skew == 1 && !T.il)                                                       \
            k_trsv_wave2d<FWD, DIV, true><<<grid, WaveCfg<DIV>::THREADS, 0, st>>>(                 \
                g, w.T, w.nbands, b, T.c1.p, T.c2.p, dv, rv, x, T.bnd.p, err, T.trace, 1, w.P2,     \
                nullptr, nullptr, nullptr, nullptr);                                               \
        else if (T.il)                                                                             \
            GG_WAVE_LAUNCH_S(FWD, DIV, 1, true);                                                   \
        else if (w.skew == 1)                                                                      \
            GG_WAVE_LAUNCH_S(FWD, DIV, 1, false);                                                  \
        else if (w.skew == 2)                                                                      \
            GG_WAVE_LAUNCH_S(FWD, DIV, 2, false);                                                  \
        else                                                                                       \
            GG_WAVE_LAUNCH_S(FWD, DIV, 3, false);                                                  \
    } while (0)
            if (T.lower) {
                if (div == WD_UNIT) GG_WAVE_LAUNCH(true, WD_UNIT);
                else if (div == WD_HW) GG_WAVE_LAUNCH(true, WD_HW);
                else if (div == WD_MUL) GG_WAVE_LAUNCH(true, WD_MUL);
                else GG_WAVE_LAUNCH(true, WD_RCP);
            } else {
                if (div == WD_UNIT) GG_WAVE_LAUNCH(false, WD_UNIT);
                else if (div == WD_HW) GG_WAVE_LAUNCH(false, WD_HW);
                else if (div == WD_MUL) GG_WAVE_LAUNCH(false, WD_MUL);
                else GG_WAVE_LAUNCH(false, WD_RCP);
            }
#undef GG_WAVE_LAUNCH
#undef GG_WAVE_LAUNCH_S
        } else {
            // 3D: persistent, every workgroup co-resident (tasks wait on tasks)
            const int ntask = w.nz * w.nbands;
#define GG_WAVE_LAUNCH3(FWD, DIV)                                                                  \
    do {                                                                                           \
        const int grid = std::min(std::min(ntask, wave3d_max_blocks<FWD, DIV>()), kTileDummyBlocks); \
        k_trsv_wave2d<FWD, DIV, false, true><<<grid, WaveCfg<DIV, true>::THREADS, 0, st>>>(        \
            g, w.T, w.nbands, b, T.c1.p, T.c2.p, dv, rv, x, T.bnd.p, err, nullptr, w.nz, w.P2,      \
            T.c0.p, T.prog.p, nullptr, nullptr);                                                   \
    } while (0)
            if (T.lower) {
                if (div == WD_UNIT) GG_WAVE_LAUNCH3(true, WD_UNIT);
                else if (div == WD_HW) GG_WAVE_LAUNCH3(true, WD_HW);
                else if (div == WD_MUL) GG_WAVE_LAUNCH3(true, WD_MUL);
                else GG_WAVE_LAUNCH3(true, WD_RCP);
            } else {
                if (div == WD_UNIT) GG_WAVE_LAUNCH3(false, WD_UNIT);
                else if (div == WD_HW) GG_WAVE_LAUNCH3(false, WD_HW);
                else if (div == WD_MUL) GG_WAVE_LAUNCH3(false, WD_MUL);
                else GG_WAVE_LAUNCH3(false, WD_RCP);
            }
#undef GG_WAVE_LAUNCH3
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
    launch_mgs_step_r(g, i, k, m, w, vk, vnext, part_in, G, part_out, H, G, Ppad, Ppad, st);
}
void launch_mgs_step_r(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, int nparts_in, double *part_out, double *H, int G,
                       long long Ppad, long long Pdot, hipStream_t st)
{
    if (vnext == w)
        k_mgs_step<true><<<G, kBlock, 0, st>>>(g, i, k, m, w, vk, nullptr, part_in, part_out, H,
                                                nparts_in, Ppad / 2, Pdot / 2);
    else
        k_mgs_step<false><<<G, kBlock, 0, st>>>(g, i, k, m, w, vk, vnext, part_in, part_out, H,
                                                 nparts_in, Ppad / 2, Pdot / 2);
}
void launch_multidot(Gate g, const double *w, const double *V, long long ldv, int nk, double *part, int G,
                     long long Pdot, hipStream_t st)
{
    dim3 grid(G, (nk + kCgsKC - 1) / kCgsKC);
    k_multidot<<<grid, kBlock, 0, st>>>(g, w, V, ldv, nk, part, G, Pdot / 2);
}
void launch_cgs_reduce(Gate g, const double *part, int P, int G, long long cnt, int nk, double *h, double *H,
                       int i, int m, bool add, hipStream_t st)
{
    k_cgs_reduce<<<nk, kBlock, 0, st>>>(g, part, P, G, cnt, h, H, i, m, add ? 1 : 0);
}
void launch_cgs_update(Gate g, double *w, const double *V, long long ldv, const double *h, int nk, int G,
                       long long Ppad, long long Pdot, double *part_norm, hipStream_t st)
{
    if (part_norm)
        k_cgs_update<true><<<G, kBlock, 0, st>>>(g, w, V, ldv, h, nk, Ppad / 2, Pdot / 2, part_norm);
    else
        k_cgs_update<false><<<G, kBlock, 0, st>>>(g, w, V, ldv, h, nk, Ppad / 2, Pdot / 2, nullptr);
}
bool launch_cgs_update_dot(Gate g, double *w, const double *V, long long ldv, const double *h, int nk, int G,
                           long long Ppad, long long Pdot, double *part, hipStream_t st)
{
    if (nk > kCgsFuseMax) return false;
    k_cgs_update_dot<<<G, kBlock, 0, st>>>(g, w, V, ldv, h, nk, Ppad / 2, Pdot / 2, part, G);
    return true;
}
void launch_arnoldi_finalize(Gate g, int i, int m, DevState *ds, const double *part, int G,
                             const double *w, double *vnext, double *H, double *cs, double *sn,
                             double *s, double *hist, long long Ppad, hipStream_t st)
{
    launch_arnoldi_finalize_r(g, i, m, ds, part, G, G, w, vnext, H, cs, sn, s, hist, Ppad, st);
}
void launch_arnoldi_finalize_r(Gate g, int i, int m, DevState *ds, const double *part, int nparts_in,
                               int G, const double *w, double *vnext, double *H, double *cs,
                               double *sn, double *s, double *hist, long long Ppad, hipStream_t st)
{
    k_arnoldi_finalize<<<G, kBlock, 0, st>>>(g, i, m, ds, part, nparts_in, w, vnext, H, cs, sn, s,
                                              hist, Ppad / 2);
}
size_t xch_area_bytes(int P, long long capd)
{
    return sizeof(double) * ((size_t)kMaxShards * kIpcXB + 2ull * P * capd + (size_t)kMaxShards * kIpcXF);
}
void launch_multidot_x(Gate g, const double *w, const double *V, long long ldv, int nk, double *part, int G,
                       long long Pdot, const Xch &x, unsigned long long seq, hipStream_t st)
{
    // (the caller checks nk <= kCgsXMax, G <= kIpcXF, nk * G <= x.capd)
    k_multidot_x<<<dim3(G, (nk + kCgsKC - 1) / kCgsKC), kBlock, 0, st>>>(g, w, V, ldv, nk, part, G, Pdot / 2, x, seq);
}
void launch_cgs_update_x(Gate g, double *w, const double *V, long long ldv, int nk, int G, long long Ppad,
                         long long Pdot, const double *part_in, unsigned long long sin, double *H, int i, int m,
                         bool add, double *part_out, double *norm_out, const Xch &x, unsigned long long sout,
                         hipStream_t st)
{
    if (part_out)
        k_cgs_update_x<true><<<G, kBlock, 0, st>>>(g, w, V, ldv, nk, Ppad / 2, Pdot / 2, G, part_in, sin, H, i, m,
                                                    add ? 1 : 0, part_out, x, sout, add ? 0 : kCgsKC);
    else
        k_cgs_update_x<false><<<G, kBlock, 0, st>>>(g, w, V, ldv, nk, Ppad / 2, Pdot / 2, G, part_in, sin, H, i,
                                                     m, add ? 1 : 0, norm_out, x, sout, add ? 0 : kCgsKC);
}
void launch_dot_x(Gate g, const double *a, const double *b, double *part, int G, long long Pdot, const Xch &x,
                  unsigned long long seq, hipStream_t st)
{
    k_dot_x<<<G, kBlock, 0, st>>>(g, a, b, part, Pdot / 2, x, seq);
}
void launch_mgs_step_x(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, unsigned long long sin, double *part_out, double *H, int G,
                       long long Ppad, long long Pdot, const Xch &x, unsigned long long sout, hipStream_t st)
{
    if (!vnext)
        k_mgs_step_x<true><<<G, kBlock, 0, st>>>(g, i, k, m, w, vk, nullptr, part_in, sin, part_out, H, G, Ppad / 2,
                                                  Pdot / 2, x, sout);
    else
        k_mgs_step_x<false><<<G, kBlock, 0, st>>>(g, i, k, m, w, vk, vnext, part_in, sin, part_out, H, G, Ppad / 2,
                                                   Pdot / 2, x, sout);
}
void launch_arnoldi_finalize_x(Gate g, int i, int m, DevState *ds, const double *part_in, unsigned long long sin,
                               int G, const double *w, double *vnext, double *H, double *cs, double *sn,
                               double *s, double *hist, long long Ppad, const Xch &x, hipStream_t st)
{
    k_arnoldi_finalize_x<<<G, kBlock, 0, st>>>(g, i, m, ds, part_in, sin, G, w, vnext, H, cs, sn, s, hist,
                                                Ppad / 2, x);
}
#ifndef GG_MGS_GATHER_DEFAULT
#define GG_MGS_GATHER_DEFAULT 2
#endif
constexpr int kMgsGatherDefault = GG_MGS_GATHER_DEFAULT;

int arnoldi_persist_units(int G, long long Ppad)
{
    const long long units = Ppad / 2, per = (long long)G * kBlock;
    const int J = (int)((units + per - 1) / per);
    return J <= 1 ? 1 : J <= 2 ? 2 : J <= 4 ? 4 : J <= 8 ? 8 : 0;
}

// the k_arnoldi_persist instantiation for J units per thread under the
// current GG_MGS_GATHER / GG_MGS_PREFETCH (one choice for the occupancy query
// and the launch: ADVICE r4)
using PersistFn = void (*)(Gate, int, int, DevState *, const double *, double *, long long, double *, double *,
                           double *, double *, double *, unsigned long long *, unsigned long long *, long long, int *,
                           unsigned long long *, unsigned long long *, unsigned long long, UnitMap, long long *,
                           const double *, double *, unsigned long long *, long long);
template <int XG, int PF>
PersistFn persist_fn_j(int J)
{
    if constexpr (PF == 2) {
        return J == 1 ? k_arnoldi_persist<1, XG, PF> : J == 2 ? k_arnoldi_persist<2, XG, PF>
                                                               : k_arnoldi_persist<4, XG, PF>;
    } else {
        return J == 1   ? k_arnoldi_persist<1, XG, PF>
               : J == 2 ? k_arnoldi_persist<2, XG, PF>
               : J == 4 ? k_arnoldi_persist<4, XG, PF>
                        : k_arnoldi_persist<8, XG, PF>;
    }
}
PersistFn persist_fn(int J)
{
    const int xg = mgs_gather_form();
    const int pf = mgs_prefetch();
    if (xg == 2 && pf == 2 && J <= 4) return persist_fn_j<2, 2>(J);
    if (xg == 3 && pf) return persist_fn_j<3, 1>(J);
    if (xg >= 2) return pf ? persist_fn_j<2, 1>(J) : persist_fn_j<2, 0>(J);
    return pf ? persist_fn_j<0, 1>(J) : persist_fn_j<0, 0>(J);
}

// blocks of the J-unit instantiation that can be resident at once
int arnoldi_persist_max_blocks(int J)
{
    int dev = 0, cus = 0, per = 0;
    if (J != 1 && J != 2 && J != 4 && J != 8) return 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    // the instantiation launch_arnoldi_persist launches
    const void *f = reinterpret_cast<const void *>(persist_fn(J));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, kBlock, 0) != hipSuccess) return 0;
    return cus * per;
}

// k_arnoldi_wide: usable when G = kWideG blocks of kWideJR + kWideJL units per
// thread cover the vectors and every block is co-resident
bool arnoldi_wide_ok(int G, long long Ppad)
{
    static int maxb = -1;
    if (maxb < 0) {
        int dev = 0, cus = 0, per = 0;
        maxb = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_arnoldi_wide, kBlock, 0) == hipSuccess)
            maxb = cus * per;
    }
    const long long units = Ppad / 2;
    return G == kWideG && G <= maxb && units <= (long long)G * kBlock * (kWideJR + kWideJL) && units < (1LL << 31);
}

void launch_arnoldi_wide(Gate g, int i, int m, DevState *ds, const double *w, double *V, long long ldv,
                         double *H, double *cs, double *sn, double *s, double *hist,
                         unsigned long long *gran, unsigned long long *hg, int G, long long Ppad, int *err,
                         const UnitMap &um, hipStream_t st)
{
    k_arnoldi_wide<<<G, kBlock, persist_test_lds(), st>>>(g, i, m, ds, w, V, ldv, H, cs, sn, s, hist, gran, hg,
                                                          Ppad / 2, err, um);
}

#ifndef GG_MGS_PREFETCH_DEFAULT
#define GG_MGS_PREFETCH_DEFAULT 1
#endif
int mgs_prefetch()
{
    // 1: v_{k+1} streamed during step k's gather, 0: after it, 2: v_{k+2}
    // issued after step k's gather (prefetch distance 2, J <= 4)
    const char *e = std::getenv("GG_MGS_PREFETCH");
    return e ? std::min(std::max(atoi(e), 0), 2) : GG_MGS_PREFETCH_DEFAULT;
}
int mgs_gather_form()
{
    // 0: every block gathers, 2: XCD-local reducers elected among the blocks,
    // 3: XCD-local reducer-only blocks (kXcds extra blocks)
    const char *e = std::getenv("GG_MGS_GATHER");
    return e ? (atoi(e) == 2 ? 2 : atoi(e) == 3 ? 3 : 0) : kMgsGatherDefault;
}

void launch_arnoldi_persist(Gate g, int i, int m, DevState *ds, const double *w, double *V,
                            long long ldv, double *H, double *cs, double *sn, double *s,
                            double *hist, unsigned long long *gran, unsigned long long *hg, int G, long long Ppad,
                            int *err, unsigned long long *xb, unsigned long long *elect, unsigned long long seq,
                            const UnitMap &um, hipStream_t st, long long *trace, const double *msc, double *mout,
                            double *fill, long long nfill)
{
    const int J = arnoldi_persist_units(G, Ppad);
    GG_REQUIRE(persist_np(J) == 0 || G <= persist_np(J) * kBlock, GG_EINVAL,
               "k_arnoldi_persist: grid beyond the all-gather's reach");
    const PersistFn f = persist_fn(J);
    const int extra = (mgs_gather_form() == 3 && mgs_prefetch()) ? kXcds : 0;   // reducer-only blocks
    f<<<G + extra, kBlock, persist_test_lds(), st>>>(g, i, m, ds, w, V, ldv, H, cs, sn, s, hist, gran, hg, Ppad / 2,
                                                     err, xb, elect, seq, um, trace, msc, mout,
                                                     reinterpret_cast<unsigned long long *>(fill), fill ? nfill : 0);
}

// the two-scenario persistent orthogonalization (k_arnoldi_persist2): 0 when
// the vectors take no J or the grid cannot be co-resident
int arnoldi_persist2_units(int G, long long Ppad)
{
    const int J = arnoldi_persist_units(G, Ppad);
    if (J != 1 && J != 2 && J != 4) return 0;
    static int cached[5] = {-1, -1, -1, -1, -1};
    if (cached[J] < 0) {
        int dev = 0, cus = 0, per = 0;
        const void *f = J == 1 ? reinterpret_cast<const void *>(k_arnoldi_persist2<1>)
                        : J == 2 ? reinterpret_cast<const void *>(k_arnoldi_persist2<2>)
                                 : reinterpret_cast<const void *>(k_arnoldi_persist2<4>);
        cached[J] = (hipGetDevice(&dev) == hipSuccess &&
                     hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                     hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, kBlock, 0) == hipSuccess)
                        ? cus * per
                        : 0;
    }
    return G <= cached[J] ? J : 0;
}
void launch_arnoldi_persist2(Gate g, long long zs, int i, int m, DevState *ds, const double *w, double *V,
                             long long ldv, double *H, double *cs, double *sn, double *s, double *hist,
                             unsigned long long *gran, int G, long long Ppad, int *err, unsigned long long *xb,
                             unsigned long long *elect, unsigned long long seq, const UnitMap &um, hipStream_t st)
{
    const int J = arnoldi_persist_units(G, Ppad);
    GG_REQUIRE(J == 1 || J == 2 || J == 4, GG_EINVAL, "k_arnoldi_persist2: vectors too long");
    GG_REQUIRE(G <= kGatherPer * kBlock, GG_EINVAL, "k_arnoldi_persist2: grid beyond the all-gather's reach");
#define GG_P2(JJ)                                                                                             \
    k_arnoldi_persist2<JJ><<<G, kBlock, persist_test_lds(), st>>>(g, zs, i, m, ds, w, V, ldv, H, cs, sn, s, hist, \
                                                                  gran, Ppad / 2, err, xb, elect, seq, um)
    if (J == 1) GG_P2(1);
    else if (J == 2) GG_P2(2);
    else GG_P2(4);
#undef GG_P2
}

void launch_update(Gate g, int m, DevState *ds, const double *H, const double *s, double *ysmall,
                   const double *V, long long ldv, double *acc, int G, long long Ppad, hipStream_t st,
                   const UnitMap &um)
{
    if (m <= kMaxRestart) k_update_y<<<1, 64, 0, st>>>(g, m, ds, H, s, ysmall);
    else k_update_y_serial<<<1, 64, 0, st>>>(g, m, ds, H, s, ysmall);
    k_update_x<<<G, kBlock, 0, st>>>(g, ds, ysmall, V, ldv, acc, Ppad / 2, um);
}
void launch_end_cycle(const double *part, int G, DevState *ds, double *hist, hipStream_t st)
{
    k_end_cycle<<<1, kBlock, 0, st>>>(part, G, ds, hist);
}

}  // namespace gg

// ================================================= batched (many-RHS) launchers
// nsc scenarios per launch; scenario q's per-scenario buffers q * zs bytes after
// scenario 0's (solver.hip / batch.hip: one arena per scenario).  The same
// kernels as the single-scenario launchers with blockIdx.y = scenario: the
// same per-scenario arithmetic, bit for bit.
namespace gg {

void launch_fill_u64_b(unsigned long long *p, long long n, unsigned long long v, int nsc, long long zs,
                       hipStream_t st)
{
    k_fill_u64<<<dim3(blocks_for(n, kBlock, 4096), nsc), kBlock, 0, st>>>(p, n, v, zs);
}
void launch_gather_b(const double *in, long long zin, const long long *idx, double *out, long long zout,
                     long long n, int nsc, hipStream_t st)
{
    k_gather_b<<<dim3(blocks_for(n, kBlock, 4096), nsc), kBlock, 0, st>>>(in, zin, idx, out, zout, n);
}
void launch_init_state_b(DevState *ds, long long zs, int nsc, double tol, int max_iter, int m, hipStream_t st)
{
    k_init_state_b<<<(nsc + 63) / 64, 64, 0, st>>>(ds, zs, nsc, tol, max_iter, m);
}
void launch_pack_states_b(const DevState *ds, long long zs, int nsc, DevState *out, const int *err, hipStream_t st)
{
    k_pack_states_b<<<(nsc + 64) / 64, 64, 0, st>>>(ds, zs, nsc, out, err);
}
void launch_transient_step_b(int n, int nsc, int maxsrc, const int *soff, const int *kind, const int *dptr,
                             const double *data, int it, double h, double *u, const int *sptr, const int *sidx,
                             const double *cdiag, const double *x, double *w, long long ldx, hipStream_t st)
{
    if (maxsrc > 0) k_sources_b<<<dim3((maxsrc + kBlock - 1) / kBlock, nsc), kBlock, 0, st>>>(soff, kind, dptr, data, it, h, u);
    if (n > 0) k_transient_rhs_b<<<dim3((n + kBlock - 1) / kBlock, nsc), kBlock, 0, st>>>(n, sptr, sidx, u, cdiag, x, w, ldx);
}
void launch_gather_ports_b(int nport, const int *port, const double *x, long long ldx, double *out, long long ldo,
                           int nsc, hipStream_t st)
{
    if (nport > 0)
        k_gather_ports_b<<<dim3((nport + kBlock - 1) / kBlock, nsc), kBlock, 0, st>>>(nport, port, x, ldx, out, ldo);
}
void launch_spmv_b(Gate g, const DevCsr &A, const double *x, const double *b, double *y, bool resid, int nsc,
                   long long zs, hipStream_t st)
{
    if (A.nblk == 0) return;
    if (!A.sell) {
        // CSR-stream (no sliced copy): one launch per scenario, the same kernel
        for (int q = 0; q < nsc; q++) {
            const long long o = (long long)q * zs;
            auto at = [o](auto *p) { return p ? reinterpret_cast<decltype(p)>(reinterpret_cast<char *>(const_cast<void *>(static_cast<const void *>(p))) + o) : p; };
            Gate gq = g;
            gq.done = at(g.done);
            gq.nit = at(g.nit);
            launch_spmv(gq, A, at(x), resid ? at(b) : nullptr, at(y), resid, st);
        }
        return;
    }
    const int blocks = (A.nslice + kBlock / 64 - 1) / (kBlock / 64);
    // up to 8 scenarios per launch (A's entries read once for all of them)
    for (int q0 = 0; q0 < nsc; q0 += kBatchSpmv) {
        const int c = std::min(kBatchSpmv, nsc - q0);
        const long long o = (long long)q0 * zs;
        auto at = [o](auto *p) { return p ? reinterpret_cast<decltype(p)>(reinterpret_cast<char *>(const_cast<void *>(static_cast<const void *>(p))) + o) : p; };
        Gate gq = g;
        gq.done = at(g.done);
        gq.nit = at(g.nit);
        if (resid)
            k_spmv_sell_b<true, kBatchSpmv><<<blocks, kBlock, 0, st>>>(gq, zs, c, A.n, A.nslice, A.sptr.p, A.sci.p,
                                                                       A.sv.p, at(x), at(b), at(y));
        else
            k_spmv_sell_b<false, kBatchSpmv><<<blocks, kBlock, 0, st>>>(gq, zs, c, A.n, A.nslice, A.sptr.p, A.sci.p,
                                                                        A.sv.p, at(x), nullptr, at(y));
    }
}
bool trsv_batchable(const DevTri &T)
{
    const Wave2D &w = T.wl;
    if (T.kind != DevTri::WAVE2D || T.tail || !w.ok || w.tile || w.nz != 1 || w.skew != 1 || T.il || T.trace)
        return false;
    const int e = T.eff_div();
    return T.lower ? (e == WD_UNIT || e == WD_UFMA) : (e == WD_HW || e == WD_RCP || e == WD_MUL || e == WD_SFMA);
}
// the batched wavefront's workgroup map (trsv_wave2d_body's zmap), default 1:
// band b of every scenario on one XCD, so the scenarios share its coefficient
// streams in the L2 -- C5 with 8 scenarios (one box, rocprofv3 FETCH_SIZE,
// profiles/r06/c5_batch_pmc.txt): U 236 -> 83 MB, L 177 -> 75 MB per launch,
// 10,500 -> 10,751 it/s; 0: a scenario's bands on one XCD
int batch_zmap()
{
    static const int z = [] {
        const char *e = std::getenv("GG_BATCH_ZMAP");
        return e ? std::atoi(e) : 1;
    }();
    return z;
}
void launch_trsv_b(Gate g, DevTri &T, const double *b, double *x, unsigned long long *bnd, int *err, int nsc,
                   long long zs, hipStream_t st)
{
    GG_REQUIRE(trsv_batchable(T), GG_EINVAL, "batched triangular solve: 2D wavefront, canonical order only");
    const Wave2D &w = T.wl;
    const int e = T.eff_div();
    const int zmap = batch_zmap();
    const dim3 grid(w.nbands * nsc);
    const double *k1 = e == WD_SFMA ? T.c1s.p : T.c1.p, *k2 = e == WD_SFMA ? T.c2s.p : T.c2.p;
    const double *dv = (e == WD_UNIT || e == WD_UFMA) ? nullptr : (e == WD_MUL || e == WD_SFMA) ? T.rw.p : T.dw.p;
    const double *rv = e == WD_RCP ? T.rw.p : nullptr;
    static const bool s1single = [] {
        const char *e = std::getenv("GG_BATCH_S1_SINGLE");     // diagnostics: one scenario on the single kernel
        return e && e[0] == '1';
    }();
    if (nsc == 1 && s1single) {
        DevTri &T2 = T;
        unsigned long long *keep = T2.bnd.p;
        T2.bnd.p = bnd;
        launch_trsv(g, T2, b, x, err, st);
        T2.bnd.p = keep;
        return;
    }
#define GG_BT(FWD, DIV)                                                                                     \
    k_trsv_wave2d_batch<FWD, DIV><<<grid, WaveCfg<DIV>::THREADS, 0, st>>>(g, w.T, w.nbands, b, k1, k2, dv, rv, \
                                                                          x, bnd, err, w.P2, nsc, zs, zmap)
    if (T.lower) {
        if (e == WD_UFMA) GG_BT(true, WD_UFMA);
        else GG_BT(true, WD_UNIT);
    } else {
        if (e == WD_SFMA) GG_BT(false, WD_SFMA);
        else if (e == WD_MUL) GG_BT(false, WD_MUL);
        else if (e == WD_RCP) GG_BT(false, WD_RCP);
        else GG_BT(false, WD_HW);
    }
#undef GG_BT
}
long long trsv_b_granules(const DevTri &T)
{
    // hand-off granules, then per band workgroup 64 zero + 64 write-only dummies, + 64
    return T.wl.ngran() + 128LL * T.wl.nbands + 64;
}
void launch_dot_b(Gate g, const double *a, const double *b, double *part, int G, long long Ppad, int nsc,
                  long long zs, hipStream_t st)
{
    k_dot<<<dim3(G, nsc), kBlock, 0, st>>>(g, a, b, part, Ppad / 2, zs);
}
void launch_set_normb_b(const double *part, int G, DevState *ds, int nsc, long long zs, hipStream_t st)
{
    k_set_normb<<<dim3(1, nsc), kBlock, 0, st>>>(part, G, ds, zs);
}
void launch_init_beta_b(const double *part, int G, DevState *ds, double *hist, int nsc, long long zs, hipStream_t st)
{
    k_init_beta<<<dim3(1, nsc), kBlock, 0, st>>>(part, G, ds, hist, zs);
}
void launch_init_cycle_b(DevState *ds, const double *r, double *v0, double *s, int G, long long Ppad, int nsc,
                         long long zs, hipStream_t st)
{
    k_init_cycle<<<dim3(G, nsc), kBlock, 0, st>>>(ds, r, v0, s, Ppad / 2, zs);
}
void launch_mgs_step_b(Gate g, int i, int k, int m, double *w, const double *vk, const double *vnext,
                       const double *part_in, double *part_out, double *H, int G, long long Ppad, int nsc,
                       long long zs, hipStream_t st)
{
    if (vnext == w)
        k_mgs_step<true><<<dim3(G, nsc), kBlock, 0, st>>>(g, i, k, m, w, vk, nullptr, part_in, part_out, H, G,
                                                          Ppad / 2, Ppad / 2, zs);
    else
        k_mgs_step<false><<<dim3(G, nsc), kBlock, 0, st>>>(g, i, k, m, w, vk, vnext, part_in, part_out, H, G,
                                                           Ppad / 2, Ppad / 2, zs);
}
void launch_arnoldi_finalize_b(Gate g, int i, int m, DevState *ds, const double *part, int G, const double *w,
                               double *vnext, double *H, double *cs, double *sn, double *s, double *hist,
                               long long Ppad, int nsc, long long zs, hipStream_t st)
{
    k_arnoldi_finalize<<<dim3(G, nsc), kBlock, 0, st>>>(g, i, m, ds, part, G, w, vnext, H, cs, sn, s, hist,
                                                        Ppad / 2, zs);
}
void launch_update_b(Gate g, int m, DevState *ds, const double *H, const double *s, double *ysmall, const double *V,
                     long long ldv, double *acc, int G, long long Ppad, const UnitMap &um, int nsc, long long zs,
                     hipStream_t st)
{
    if (m <= kMaxRestart) k_update_y<<<dim3(1, nsc), 64, 0, st>>>(g, m, ds, H, s, ysmall, zs);
    else k_update_y_serial<<<dim3(1, nsc), 64, 0, st>>>(g, m, ds, H, s, ysmall, zs);
    k_update_x<<<dim3(G, nsc), kBlock, 0, st>>>(g, ds, ysmall, V, ldv, acc, Ppad / 2, um, zs);
}
void launch_end_cycle_b(const double *part, int G, DevState *ds, double *hist, int nsc, long long zs, hipStream_t st)
{
    k_end_cycle<<<dim3(1, nsc), kBlock, 0, st>>>(part, G, ds, hist, zs);
}

}  // namespace gg
