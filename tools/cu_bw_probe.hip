// Micro-benchmark: how many GB/s ONE CU can stream from data resident in the
// Infinity Cache when only K CUs of the chip are streaming (the wavefront
// triangular solve's situation: 16 workgroups, each reading its band's arrays).
// Diagnostics only (not part of the library).
//
//   mode 0: W waves, global_load_dwordx4 into registers, D loads in flight per lane
//   mode 1: W waves, LDS-DMA (global_load_lds_dwordx4) into a per-wave ring, counted vmcnt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__host__ __device__ constexpr int vm_wait(int n)
{
    return (n & 15) | (7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14);
}

// block b streams chunk b: `bytes` bytes, split over its W waves (wave w takes
// 1 KiB pieces w, w+W, ...)
template <int D>
__global__ void k_reg(const double2 *src, long long pieces, double *out, long long *cyc)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
    const double2 *base = src + (long long)blockIdx.x * pieces * 64 + lane;
    long long t0 = 0;
    if (threadIdx.x == 0) t0 = (long long)__builtin_amdgcn_s_memrealtime();
    double acc = 0.0;
    double2 r[D];
    long long p = wave;
#pragma unroll
    for (int d = 0; d < D; d++) r[d] = base[(p + (long long)d * W) * 64];
    for (; p + (long long)D * W < pieces; p += (long long)D * W) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            acc += r[d].x + r[d].y;
            r[d] = base[(p + (long long)(d + D) * W) * 64];
        }
    }
#pragma unroll
    for (int d = 0; d < D; d++) acc += r[d].x + r[d].y;
    __syncthreads();
    if (threadIdx.x == 0) cyc[blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime() - t0;
    if (acc == 12345.678) out[0] = acc;
}

// LDS-DMA: each wave keeps RING 1-KiB pieces in flight into its own LDS ring
template <int RING>
__global__ void k_dma(const double2 *src, long long pieces, double *out, long long *cyc)
{
    extern __shared__ double2 lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, W = blockDim.x >> 6;
    const double2 *base = src + (long long)blockIdx.x * pieces * 64 + lane;
    double2 *ring = lds + wave * RING * 64;
    long long t0 = 0;
    if (threadIdx.x == 0) t0 = (long long)__builtin_amdgcn_s_memrealtime();
    const long long mine = (pieces - wave + W - 1) / W;
    long long k = 0;
    for (; k < RING && k < mine; k++)
        __builtin_amdgcn_global_load_lds((gbl_void_t *)(base + (wave + k * W) * 64),
                                         (lds_void_t *)(ring + (k % RING) * 64), 16, 0, 0);
    double acc = 0.0;
    for (long long j = 0; j < mine; j++) {
        if (k - j == RING) __builtin_amdgcn_s_waitcnt(vm_wait(RING - 1));
        else __builtin_amdgcn_s_waitcnt(vm_wait(0));
        acc += ring[(j % RING) * 64 + lane].x;
        if (k < mine) {
            __builtin_amdgcn_global_load_lds((gbl_void_t *)(base + (wave + k * W) * 64),
                                             (lds_void_t *)(ring + (k % RING) * 64), 16, 0, 0);
            k++;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) cyc[blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime() - t0;
    if (acc == 12345.678) out[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main()
{
    const long long chunk = 4ll << 20;                  // bytes per block
    const int maxK = 32;
    const long long pieces = chunk / 1024;
    double2 *src; double *out; long long *cyc;
    CK(hipMalloc(&src, chunk * maxK));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&cyc, 8 * 1024));
    CK(hipMemset(src, 0, chunk * maxK));
    CK(hipFuncSetAttribute((const void *)k_dma<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void *)k_dma<40>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    std::vector<long long> hc(maxK);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto report = [&](const char *name, int K, int W, auto launch) {
        for (int rep = 0; rep < 3; rep++) launch();      // warm (MALL-resident)
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipGetLastError());
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(hc.data(), cyc, 8 * K, hipMemcpyDeviceToHost));
        double mx = 0, mn = 1e30;
        for (int i = 0; i < K; i++) { mx = hc[i] > mx ? hc[i] : mx; mn = hc[i] < mn ? hc[i] : mn; }
        // s_memrealtime: 100 MHz
        printf("%-10s K=%2d W=%2d  launch %.1f us  per-CU GB/s: min %.1f max %.1f\n", name, K, W, ms * 1e3,
               chunk / (mx * 10.0), chunk / (mn * 10.0));
        return 0;
    };
    for (int K : {8, 16, 32}) {
        for (int W : {1, 2, 4, 8}) {
            report("reg D=4", K, W, [&] { hipLaunchKernelGGL(k_reg<4>, dim3(K), dim3(64 * W), 0, 0, src, pieces, out, cyc); });
            report("reg D=8", K, W, [&] { hipLaunchKernelGGL(k_reg<8>, dim3(K), dim3(64 * W), 0, 0, src, pieces, out, cyc); });
            report("dma R=16", K, W, [&] { hipLaunchKernelGGL(k_dma<16>, dim3(K), dim3(64 * W), W * 16 * 1024, 0, src, pieces, out, cyc); });
            if (W * 40 <= 128) report("dma R=40", K, W, [&] { hipLaunchKernelGGL(k_dma<40>, dim3(K), dim3(64 * W), W * 40 * 1024, 0, src, pieces, out, cyc); });
        }
    }
    return 0;
}
