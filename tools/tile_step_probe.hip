// Micro-benchmark: dependent-chain cycles per step of the 3D tile wavefront's
// recurrence (kernels.hip k_trsv_tile3d) on gfx950, one wave: the plane shift
// (permlane swaps + selects), the line shift (DPP row_shr:1) and the full unit-L
// step, against the 2D step.  Diagnostics only (not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/tile_step_probe.hip -o tools/tile_step_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_old(double v, double old)
{
    int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ unsigned bfi(unsigned m, unsigned a, unsigned b) { return (a & m) | (b & ~m); }
struct RowMasks { unsigned m0, m1, m3, mhi; };
// two-register swaps (as the library kernel)
__device__ __forceinline__ double plane_shift2(double x, double kb, const RowMasks &rm)
{
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const unsigned klo = (unsigned)__double2loint(kb), khi = (unsigned)__double2hiint(kb);
    const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const auto l32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    unsigned rlo = bfi(rm.mhi, bfi(rm.m3, l32[0], l16[1]), bfi(rm.m1, l16[0], klo));
    unsigned rhi = bfi(rm.mhi, bfi(rm.m3, h32[0], h16[1]), bfi(rm.m1, h16[0], khi));
    return __hiloint2double((int)rhi, (int)rlo);
}
// lane-16 move through ds_bpermute (LDS crossbar)
__device__ __forceinline__ double plane_bperm(double x, double kb, int srcaddr, bool first)
{
    int lo = __builtin_amdgcn_ds_bpermute(srcaddr, __double2loint(x));
    int hi = __builtin_amdgcn_ds_bpermute(srcaddr, __double2hiint(x));
    const double t = __hiloint2double(hi, lo);
    return first ? kb : t;
}

constexpr int N = 256;

__global__ void k_probe(const double *in, double *out, long long *cyc)
{
    const int l = threadIdx.x;
    const int row = l >> 4;
    const RowMasks rm{row == 0 ? ~0u : 0u, row == 1 ? ~0u : 0u, row == 3 ? ~0u : 0u, row >= 2 ? ~0u : 0u};
    const int rowmap[4] = {0, 1, 3, 2};
    const int src = ((l & 15) + 16 * rowmap[(row + 3) & 3]) * 4;
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
    TIMED(0, x = (c - b * dpp_old<0x138>(x, d)) - d * x)                                     // 2D step
    TIMED(1, x = plane_shift2(x, d, rm))                                                    // plane shift
    TIMED(2, x = dpp_old<0x111>(x, d))                                                      // line shift
    TIMED(3, x = ((c - b * plane_shift2(x, d, rm)) - a * dpp_old<0x111>(x, d)) - d * x)     // tile step
    TIMED(4, x = plane_bperm(x, d, src, row == 0))                                          // bpermute shift
    TIMED(5, x = ((c - b * plane_bperm(x, d, src, row == 0)) - a * dpp_old<0x111>(x, d)) - d * x)
}

int main()
{
    double h[256];
    for (int i = 0; i < 256; i++) h[i] = 0.25 + 1e-3 * i;
    double *din, *dout;
    long long *dc, hc[16];
    if (hipMalloc(&din, sizeof(h)) || hipMalloc(&dout, 16 * 64 * sizeof(double)) || hipMalloc(&dc, sizeof(hc)))
        return 1;
    if (hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice)) return 1;
    const char *nm[6] = {"2D step (wave_shr DPP, mul, 2 sub)", "plane shift (permlane swaps + selects)",
                         "line shift (DPP row_shr:1)", "tile step (plane + line + in-line)",
                         "plane shift via ds_bpermute", "tile step with ds_bpermute"};
    for (int rep = 0; rep < 3; rep++) {
        k_probe<<<1, 64>>>(din, dout, dc);
        if (hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost)) return 1;
    }
    for (int k = 0; k < 6; k++) printf("%-45s %6.1f cycles/step\n", nm[k], (double)hc[k] / N);
    return 0;
}
