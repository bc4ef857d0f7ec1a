// Micro-benchmark: dependent-chain latency (cycles) of fp64 VALU ops and DPP on
// gfx950, one wave.  Diagnostics only (not part of the library).
// Build as the library: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off lat_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_old(double v, double old)
{
    int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double dpp_zero_rowshr(double v)
{
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x111, 0xf, 0xf, true);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x111, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// the same shift with bound_ctrl (out-of-range lanes read 0) and the edge lane's
// value selected afterwards: no `old` operand tied into the DPP move
template <int CTRL, int EDGE>
__device__ __forceinline__ double dpp_sel(double v, double old)
{
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
    const double t = __hiloint2double(hi, lo);
    return (threadIdx.x & 63) == EDGE ? old : t;
}

constexpr int N = 256;

__global__ void k_probe(const double *in, double *out, long long *cyc)
{
    const int l = threadIdx.x;
    double a = in[l], b = in[64 + l], c = in[128 + l], d = in[192 + l];
    double x;
    long long t0, t1;
#define TIMED(slot, body)                                                      \
    x = a;                                                                     \
    __builtin_amdgcn_s_waitcnt(0);                                             \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");  \
    asm volatile("; def %0" : "+v"(x));                                        \
    _Pragma("unroll") for (int i = 0; i < N; i++) { body; }                    \
    { int f = __builtin_amdgcn_readfirstlane(__double2hiint(x));               \
      asm volatile("; use %0" ::"s"(f)); }                                     \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");  \
    out[slot * 64 + l] = x;                                                    \
    if (l == 0) cyc[slot] = t1 - t0;
    TIMED(0, x = x + b)
    TIMED(1, x = x * b)
    TIMED(2, x = __builtin_fma(x, b, c))
    TIMED(3, x = (c - b * x) - d * x)
    TIMED(4, x = (c - b * dpp_old<0x138>(x, d)) - d * x)
    TIMED(5, x = x / b)
    TIMED(6, { double q = x * c; double r = __builtin_fma(-q, b, x); x = __builtin_fma(r, c, q); })
    TIMED(7, x = dpp_old<0x138>(x, d))
    TIMED(8, { double y = (c - b * dpp_old<0x138>(x, d)) - d * x; x = y / a; })
    TIMED(9, { double y = (c - b * dpp_old<0x138>(x, d)) - d * x; double q = y * c; double r = __builtin_fma(-q, a, y); x = __builtin_fma(r, c, q); })
    TIMED(10, { x = x + b; a = a + c; })
    TIMED(11, x = __builtin_amdgcn_rcp(x))
    TIMED(12, x = dpp_old<0x111>(x, d))
    TIMED(13, x = dpp_old<0x142>(x, d))
    TIMED(14, x = dpp_old<0x1B>(x, d))
    TIMED(15, x = (c - b * dpp_old<0x111>(x, d)) - d * x)
    TIMED(16, x = dpp_old<0x13C>(x, d))
    TIMED(17, x = dpp_zero_rowshr(x) + b)
    TIMED(18, x = __shfl_up(x, 1, 64) + b)
    // the wavefront U step exactly (k_trsv_wave2d WD_RCP): DPP, mul, two subs,
    // q0 = acc*y and the two FMA corrections
    TIMED(19, { double acc = (c - b * dpp_old<0x130>(x, d)) - d * x; double q0 = acc * c;
                double q1 = __builtin_fma(-__builtin_fma(q0, a, -acc), c, q0);
                x = __builtin_fma(-__builtin_fma(q1, a, -acc), c, q1); })
    TIMED(20, x = (dpp_sel<0x138, 0>(x, d)))
    TIMED(21, x = (c - b * dpp_sel<0x138, 0>(x, d)) - d * x)
    TIMED(22, { double acc = (c - b * dpp_sel<0x130, 63>(x, d)) - d * x; double q0 = acc * c;
                double q1 = __builtin_fma(-__builtin_fma(q0, a, -acc), c, q0);
                x = __builtin_fma(-__builtin_fma(q1, a, -acc), c, q1); })
    // the wavefront U step with GG_DIV_RCP (k_trsv_wave2d WD_MUL): DPP, mul, two subs, one mul
    TIMED(23, x = ((c - b * dpp_old<0x130>(x, d)) - d * x) * a)
    // GG_DIV_FMA (k_trsv_wave2d WD_UFMA / WD_SFMA): in-line term fused first, then
    // the line term fused after the DPP move (U: b and coefficients pre-scaled)
    TIMED(24, x = __builtin_fma(-b, dpp_old<0x138>(x, d), __builtin_fma(-d, x, c)))
    TIMED(25, x = __builtin_fma(-b, dpp_old<0x130>(x, d), __builtin_fma(-d, x, c * a)))
}

// shader clock vs the constant 100 MHz real-time counter over a long chain
__global__ void k_clock(const double *in, double *out, long long *cyc)
{
    const int l = threadIdx.x;
    double x = in[l], b = in[64 + l];
    long long t0, t1, r0, r1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
    for (int i = 0; i < (1 << 20); i++) x = x * b;
    { int f = __builtin_amdgcn_readfirstlane(__double2hiint(x)); asm volatile("; use %0" ::"s"(f)); }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
    out[l] = x;
    if (l == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

// same dependent step chain, wave 0 only, other waves of the block parked
template <int MODE>
__global__ void k_probe_block(const double *in, double *out, long long *cyc)
{
    const int l = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    __shared__ double pad[MODE == 2 ? 18000 : 1];
    if (w > 0) {
        if (MODE == 1 || MODE == 2) __syncthreads();
        else __builtin_amdgcn_s_sleep(127);
        return;
    }
    double a = in[l], b = in[64 + l], c = in[128 + l], d = in[192 + l];
    pad[0] = a;
    double x = a;
    long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile("; def %0" : "+v"(x));
#pragma unroll
    for (int i = 0; i < N; i++) x = (c - b * dpp_old<0x138>(x, d)) - d * x;
    { int f = __builtin_amdgcn_readfirstlane(__double2hiint(x));
      asm volatile("; use %0" ::"s"(f)); }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[l] = x + pad[0];
    if (l == 0) cyc[0] = t1 - t0;
    if (MODE == 1 || MODE == 2) __syncthreads();
}

int main()
{
    double h[256];
    for (int i = 0; i < 256; i++) h[i] = 1.0 + 1e-3 * i;
    double *din, *dout;
    long long *dc, hc[32] = {0};   // 26 probes
    hipMalloc(&din, sizeof h);
    hipMalloc(&dout, 32 * 64 * sizeof(double));
    hipMalloc(&dc, sizeof hc);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) k_probe<<<1, 64>>>(din, dout, dc);
    hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    const char *names[] = {"add", "mul", "fma", "step(no dpp)", "step(dpp)", "div", "markstein div",
                           "dpp only", "step+div", "step+markstein", "add x2 indep", "rcp",
                           "row_shr:1", "row_bcast:15", "quad_perm", "step(row_shr)", "wave_ror:1",
                           "row_shr+add", "shfl_up+add", "U step (WD_RCP)",
                           "wave_shr sel", "step(wave_shr sel)", "U step (sel)", "U step (WD_MUL)",
                           "L step (UFMA)", "U step (SFMA)"};
    for (int i = 0; i < 26; i++) printf("%-16s %7.2f cycles/iter\n", names[i], (double)hc[i] / N);
    for (int nw : {1, 5, 7}) {
        for (int mode = 0; mode < 3; mode++) {
            for (int rep = 0; rep < 3; rep++) {
                if (mode == 0) k_probe_block<0><<<1, 64 * nw>>>(din, dout, dc);
                if (mode == 1) k_probe_block<1><<<1, 64 * nw>>>(din, dout, dc);
                if (mode == 2) k_probe_block<2><<<1, 64 * nw>>>(din, dout, dc);
            }
            hipMemcpy(hc, dc, sizeof(long long), hipMemcpyDeviceToHost);
            printf("block waves %d mode %d: step(dpp) %7.2f cycles/iter\n", nw, mode, (double)hc[0] / N);
        }
    }
    for (int nb : {16, 256}) {
        for (int rep = 0; rep < 3; rep++) k_probe_block<2><<<nb, 64 * 5>>>(din, dout, dc);
        hipMemcpy(hc, dc, sizeof(long long), hipMemcpyDeviceToHost);
        printf("grid %d blocks x 5 waves, mode 2: step(dpp) %7.2f cycles/iter\n", nb, (double)hc[0] / N);
    }
    for (int rep = 0; rep < 2; rep++) k_clock<<<1, 64>>>(din, dout, dc);
    hipMemcpy(hc, dc, 2 * sizeof(long long), hipMemcpyDeviceToHost);
    printf("shader clock %.3f GHz (s_memtime / s_memrealtime at 100 MHz, one wave)\n",
           (double)hc[0] / (double)hc[1] * 0.1);
    return 0;
}
