// stage_probe.hip -- diagnostics (not part of the library): what exporting a
// wavefront step's values costs the recurrence wave on gfx950.
//
// The recurrence is the GG_DIV_FMA unit-L step of k_trsv_wave2d:
//   x = fma(-b, dpp_shr1(x), fma(-d, x, c))
// run for N steps by NC identical waves of one workgroup (the redundant compute
// waves of GG_WAVE_NC), each exporting the step pairs p with p % NC == its index
// (ST 1: ds_write_b128 into LDS, ST 2: global_store_dwordx4, ST 0: nothing),
// optionally reading 3 double2 operands per pair from LDS kWaveLook = 3 pairs
// ahead (RD), like the kernel's compute wave.  Cycles per step from s_memtime
// of wave 0.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off stage_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp_old(double v, double old)
{
    int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

constexpr int N = 512;              // steps (256 pairs)
constexpr int RING = 16;            // export slots (pairs) in LDS
constexpr int LOOK = 3;

template <int ST, int RD, int NC>
__global__ void k_stage(const double *in, double *out, double2 *gx, long long *cyc)
{
    __shared__ double2 ex[RING * 64];
    __shared__ double2 rd[3 * 16 * 64];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int k = w; k < 3 * 16; k += blockDim.x / 64) rd[k * 64 + l] = make_double2(in[l], in[64 + l]);
    __syncthreads();
    if (w >= NC) {
        __syncthreads();
        return;
    }
    const double b = in[l], c = in[64 + l], d = in[128 + l];
    double x = in[192 + l];
    double2 rg[LOOK + 1][3];
    if constexpr (RD) {
#pragma unroll
        for (int q = 0; q < LOOK; q++)
#pragma unroll
            for (int a = 0; a < 3; a++) rg[q][a] = rd[(a * 16 + q) * 64 + l];
    }
    long long t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
#pragma unroll LOOK + 1
    for (int p = 0; p < N / 2; p++) {
        double bb = b, cc = c;
        if constexpr (RD) {
            // operands of this pair (read LOOK pairs ago), the pair LOOK ahead issued now
            const int slot = p % (LOOK + 1);
            bb = rg[slot][0].x + rg[slot][1].y * 0.0;
            cc = rg[slot][2].x;
            const int q = (p + LOOK) & 15;
#pragma unroll
            for (int a = 0; a < 3; a++) rg[(p + LOOK) % (LOOK + 1)][a] = rd[(a * 16 + q) * 64 + l];
        }
        const double x0 = __builtin_fma(-bb, dpp_old<0x138>(x, d), __builtin_fma(-d, x, cc));
        const double x1 = __builtin_fma(-bb, dpp_old<0x138>(x0, d), __builtin_fma(-d, x0, cc));
        if (p % NC == w) {
            if constexpr (ST == 1) ex[(p & (RING - 1)) * 64 + l] = make_double2(x0, x1);
            if constexpr (ST == 2) gx[((long long)p * 64 + l)] = make_double2(x0, x1);
        }
        x = x1;
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        int f = __builtin_amdgcn_readfirstlane(__double2hiint(x));
        asm volatile("; use %0" ::"s"(f));
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[threadIdx.x] = x + ex[l].x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    __syncthreads();
}

template <int ST, int RD, int NC>
void run(const double *din, double *dout, double2 *gx, long long *dc, int waves)
{
    long long h = 0;
    for (int rep = 0; rep < 3; rep++) k_stage<ST, RD, NC><<<1, 64 * waves>>>(din, dout, gx, dc);
    (void)hipMemcpy(&h, dc, sizeof h, hipMemcpyDeviceToHost);
    printf("  export %-6s reads %-3s compute waves %d (block %d waves): %7.2f cycles/step\n",
           ST == 0 ? "none" : ST == 1 ? "LDS" : "global", RD ? "yes" : "no", NC, waves, (double)h / N);
}

int main()
{
    double h[256];
    for (int i = 0; i < 256; i++) h[i] = 1.0 + 1e-3 * i;
    double *din, *dout;
    double2 *gx;
    long long *dc;
    (void)hipMalloc(&din, sizeof h);
    (void)hipMalloc(&dout, 8192 * sizeof(double));
    (void)hipMalloc(&gx, (size_t)N * 64 * sizeof(double2));
    (void)hipMalloc(&dc, 8 * sizeof(long long));
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    for (int waves : {1, 4, 5}) {
        printf("-- block of %d waves\n", waves);
        run<0, 0, 1>(din, dout, gx, dc, waves);
        run<1, 0, 1>(din, dout, gx, dc, waves);
        run<2, 0, 1>(din, dout, gx, dc, waves);
        run<0, 1, 1>(din, dout, gx, dc, waves);
        run<1, 1, 1>(din, dout, gx, dc, waves);
        run<2, 1, 1>(din, dout, gx, dc, waves);
        if (waves >= 2) {
            run<1, 0, 2>(din, dout, gx, dc, waves);
            run<2, 0, 2>(din, dout, gx, dc, waves);
            run<1, 1, 2>(din, dout, gx, dc, waves);
            run<2, 1, 2>(din, dout, gx, dc, waves);
        }
        if (waves >= 4) {
            run<1, 1, 4>(din, dout, gx, dc, waves);
            run<2, 1, 4>(din, dout, gx, dc, waves);
        }
    }
    return 0;
}
