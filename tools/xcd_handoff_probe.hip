// Hand-off latency between two workgroups, same XCD vs different XCDs, by
// store flavour (diagnostics only, not part of the library):
//   st 0: agent-scope (sc1) store -- the line leaves the XCD's L2 (what the
//         wavefront kernels' granules use today)
//   st 1: plain store -- the line stays in the producer XCD's L2, so a
//         same-XCD consumer's sc1 (L1-bypassing) poll is served by L2; NOT
//         visible cross-XCD without a release (the probe then times out)
// Ping-pong between block 0 and block `peer` (blocks b and b + 8 usually share
// an XCD; the XCC ids are read with s_getreg and reported), lane 0 of wave 0;
// waves 1..3 of both blocks optionally stream a large buffer (the loader's
// load on the endpoint CUs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/xcd_handoff_probe.hip -o tools/xcd_handoff_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#pragma clang diagnostic ignored "-Wunused-result"

__device__ __forceinline__ unsigned xcc_id()
{
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int ST>
__device__ __forceinline__ void st_flag(unsigned long long *p, unsigned long long v)
{
    if constexpr (ST == 0) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    }
}

typedef double d4v __attribute__((ext_vector_type(4)));
constexpr int kIters = 2000;
constexpr long long kLimit = 200000;      // polls before giving up (cross-XCD plain stores)

template <int ST>
__global__ __launch_bounds__(256) void k_pingpong(unsigned long long *flags, int peer, int stream,
                                                  const double4 *buf, long long nbuf, long long *out,
                                                  unsigned *xcc, double *sink)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
    const bool player = blockIdx.x == 0 || (int)blockIdx.x == peer;
    if (!player) return;
    __shared__ int done;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (wave > 0) {
        // streaming waves (the loader's traffic on this CU), until the ping-pong ends
        double acc = 0.0;
        if (stream) {
            long long i = ((long long)blockIdx.x * 3 + wave - 1) * 64 * 64 + lane;
            while (!__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const d4v v = __builtin_nontemporal_load(reinterpret_cast<const d4v *>(buf) + ((i + k * 64) % nbuf));
                    acc += v.x + v.w;
                }
                i += 8 * 64 * 7;
            }
        }
        if (acc == 12345.0) sink[0] = acc;
        return;
    }
    if (lane != 0) return;
    unsigned long long *ping = flags, *pong = flags + 64;      // separate 512-B lines
    long long t0 = 0, t1 = 0, bad = 0;
    if (blockIdx.x == 0) {
        t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (int k = 1; k <= kIters; k++) {
            st_flag<ST>(ping, k);
            long long spins = 0;
            while (ld_sc1(pong) != (unsigned long long)k) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kLimit) { bad = 1; break; }
            }
            if (bad) break;
        }
        t1 = (long long)__builtin_amdgcn_s_memrealtime();
        out[0] = t1 - t0;
        out[1] = bad;
    } else {
        for (int k = 1; k <= kIters; k++) {
            long long spins = 0;
            while (ld_sc1(ping) != (unsigned long long)k) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kLimit) { bad = 1; break; }
            }
            if (bad) break;
            st_flag<ST>(pong, k);
        }
        out[2] = bad;
    }
    __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

int main()
{
    const long long nbuf = (512LL << 20) / sizeof(double4);     // 512 MiB: beyond the Infinity Cache
    double4 *buf;
    unsigned long long *flags;
    long long *out;
    unsigned *xcc;
    double *sink;
    hipMalloc(&buf, nbuf * sizeof(double4));
    hipMemset(buf, 0, nbuf * sizeof(double4));
    hipMalloc(&flags, 128 * sizeof(unsigned long long));
    hipMalloc(&out, 4 * sizeof(long long));
    hipMalloc(&xcc, 64 * sizeof(unsigned));
    hipMalloc(&sink, sizeof(double));
    std::printf("one-way hand-off latency (ns), block 0 <-> peer, %d round trips\n", kIters);
    std::printf("%-6s %-6s %-7s %-10s %-10s %s\n", "peer", "store", "stream", "xcc(0,p)", "ns/hop", "status");
    for (int peer : {8, 16, 1, 3}) {
        for (int st : {0, 1}) {
            for (int stream : {0, 1}) {
                hipMemset(flags, 0, 128 * sizeof(unsigned long long));
                hipMemset(out, 0, 4 * sizeof(long long));
                if (st == 0)
                    k_pingpong<0><<<64, 256>>>(flags, peer, stream, buf, nbuf, out, xcc, sink);
                else
                    k_pingpong<1><<<64, 256>>>(flags, peer, stream, buf, nbuf, out, xcc, sink);
                if (hipDeviceSynchronize() != hipSuccess) {
                    std::printf("launch failed\n");
                    return 1;
                }
                long long o[4];
                unsigned x[64];
                hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
                hipMemcpy(x, xcc, sizeof x, hipMemcpyDeviceToHost);
                const double ns = o[0] * 10.0 / (2.0 * kIters);      // s_memrealtime: 100 MHz
                std::printf("%-6d %-6s %-7d %u,%-8u %-10.1f %s\n", peer, st ? "plain" : "sc1", stream, x[0], x[peer], ns,
                            (o[1] || o[2]) ? "TIMED OUT (not visible)" : "ok");
            }
        }
    }
    return 0;
}
