// Micro-benchmark of the wavefront compute wave's batch loop (one wave, LDS
// operands prefilled, no loaders): which part of a batch costs what.
// Diagnostics only (not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_old(double v, double old)
{
    int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

constexpr int PBN = 4;       // pairs per batch
constexpr int NB = 64;       // batches timed
// FLAGS: 1 refill reads, 2 xbuf write, 4 bv reads at top, 8 barrier, 16 lgkmcnt(0) before barrier
template <int A, bool RCP, int FLAGS, int GUARD>
__global__ void k_ring(double *out, long long *cyc)
{
    constexpr int PB = PBN * 64;
    constexpr int SLOT = A * PB;
    constexpr int R = 4;
    __shared__ double2 lds[R * SLOT + 64 + 2 * PB];
    const int lane = threadIdx.x;
    for (int i = lane; i < R * SLOT + 64 + 2 * PB; i += 64)
        lds[i] = make_double2(1.0 + 1e-3 * (i & 15), 0.5 + 1e-3 * (i & 7));
    __syncthreads();
    double *bring = reinterpret_cast<double *>(lds + R * SLOT);
    double2 *xbuf = lds + R * SLOT + 64;
    double2 rg[PBN][A];
#pragma unroll
    for (int kk = 0; kk < PBN; kk++)
#pragma unroll
        for (int a = 0; a < A; a++) rg[kk][a] = lds[a * PB + kk * 64 + lane];
    double2 bv[PBN];
#pragma unroll
    for (int kk = 0; kk < PBN; kk++) bv[kk] = make_double2(0.25, 0.5);
    double xp = 0.0;
    bool bad = false;
    long long t0, t1;
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int bi = 0; bi < NB; bi++) {
        if (FLAGS & 16) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (FLAGS & 8) asm volatile("s_barrier" ::: "memory");
        if (FLAGS & 4) {
            const double2 *br = reinterpret_cast<const double2 *>(bring + (bi & 1) * 64);
#pragma unroll
            for (int kk = 0; kk < PBN; kk++) bv[kk] = br[kk];
        }
        const double2 *sn = lds + ((bi + 1) % R) * SLOT + lane;
        double xv[2 * PBN];
#pragma unroll
        for (int kk = 0; kk < PBN; kk++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const bool sx = h == 0;
                const double bb = sx ? rg[kk][0].x : rg[kk][0].y;
                const double e1 = sx ? rg[kk][1].x : rg[kk][1].y;
                const double e2 = sx ? rg[kk][2].x : rg[kk][2].y;
                const double old = h ? bv[kk].y : bv[kk].x;
                const double xs = dpp_old<0x138>(xp, old);
                double acc = bb - e1 * xs;
                acc = acc - e2 * xp;
                if constexpr (RCP) {
                    const double d = sx ? rg[kk][3].x : rg[kk][3].y;
                    const double y = sx ? rg[kk][4].x : rg[kk][4].y;
                    if (GUARD == 1) bad |= (unsigned)(__builtin_amdgcn_frexp_exp(acc) + 900) > 1800u;
                    const double q0 = acc * y;
                    // class mask: 0x3 NaN, 0x4|0x200 +-inf, 0x10|0x80 +-subnormal
                    if (GUARD == 2) bad |= __builtin_amdgcn_class(q0 * 0x1p-130, 0x3 | 0x4 | 0x200 | 0x10 | 0x80);
                    const double q1 = __builtin_fma(-__builtin_fma(q0, d, -acc), y, q0);
                    acc = __builtin_fma(-__builtin_fma(q1, d, -acc), y, q1);
                }
                xp = acc;
                xv[2 * kk + h] = acc;
            }
            if (FLAGS & 2) xbuf[(bi & 1) * PB + kk * 64 + lane] = make_double2(xv[2 * kk], xv[2 * kk + 1]);
            if (FLAGS & 1) {
#pragma unroll
                for (int a = 0; a < A; a++) rg[kk][a] = sn[a * PB + kk * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    { int f = __builtin_amdgcn_readfirstlane(__double2hiint(xp));
      asm volatile("; use %0" ::"s"(f)); }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[lane] = xp + (bad ? 1.0 : 0.0);
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int A, bool RCP, int FLAGS, int GUARD = 1>
void run(double *dout, long long *dc, const char *name)
{
    long long h = 0;
    for (int r = 0; r < 3; r++) k_ring<A, RCP, FLAGS, GUARD><<<1, 64>>>(dout, dc);
    (void)hipMemcpy(&h, dc, sizeof h, hipMemcpyDeviceToHost);
    printf("%-6s flags %2d : %7.1f cycles/step\n", name, FLAGS, (double)h / (NB * 2 * PBN));
}

int main()
{
    double *dout;
    long long *dc;
    (void)hipMalloc(&dout, 64 * sizeof(double));
    (void)hipMalloc(&dc, sizeof(long long));
#define BOTH(F) run<3, false, F>(dout, dc, "unit"); run<5, true, F>(dout, dc, "rcp");
    BOTH(0) BOTH(1) BOTH(2) BOTH(3) BOTH(4) BOTH(7) BOTH(15) BOTH(31)
    run<5, true, 0, 0>(dout, dc, "rcp-noguard");
    run<5, true, 0, 2>(dout, dc, "rcp-classguard");
    run<5, true, 31, 0>(dout, dc, "rcp-noguard");
    run<5, true, 31, 2>(dout, dc, "rcp-classguard");
    return 0;
}
