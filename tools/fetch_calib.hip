// fetch_calib: calibrate rocprofv3's FETCH_SIZE (TCC_EA0_RDREQ x 64 B) against
// known byte counts for the access patterns the solver's kernels use.
// MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a 16-B/lane coalesced stream;
// other widths are uncalibrated.  Each kernel below reads a known number of
// bytes (and, for the gathers, a known number of distinct 64-B / 128-B lines)
// from a table far larger than the 256 MiB Infinity Cache, so every byte comes
// from HBM.  Run:
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d OUT -o run -- tools/fetch_calib
// then compare each kernel's FETCH_SIZE (KiB) with the bytes printed here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr long long kTable = 3LL << 30;        // 3 GiB table (12x the Infinity Cache)

// coalesced stream, W bytes per lane per load
template <class T>
__global__ void k_stream(const T *__restrict__ p, long long n, double *sink)
{
    double acc = 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const T v = p[i];
        acc += (double)reinterpret_cast<const unsigned char *>(&v)[0];
    }
    if (acc == -1.0) sink[0] = acc;
}

// 8-B gathers at random 128-B-aligned addresses (one load per distinct line):
// SC1 = agent-scope (sc1) loads, as the flow solve's polls
template <bool SC1>
__global__ void k_gather(const unsigned long long *__restrict__ p, const long long *__restrict__ idx, long long n,
                         double *sink)
{
    unsigned long long acc = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long *a = p + idx[i];
        acc += SC1 ? __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *a;
    }
    if (acc == 1ull) sink[0] = (double)acc;
}

// two dependent 8-B loads per random 128-B line, the second OFF bytes after
// the first and issued once the first has returned (so a 128-B fill serves it
// from L2, a 64-B fill does not when OFF = 64); launched with few enough
// threads that the lines in flight fit the L2s
template <int OFF>
__global__ void k_gather2(const unsigned long long *__restrict__ p, const long long *__restrict__ idx, long long n,
                          double *sink)
{
    unsigned long long acc = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long *a = p + idx[i];
        const unsigned long long v0 = *a;
        acc += v0 + a[OFF / 8 + (v0 == 12345ull)];       // address depends on v0: issued after it returns
    }
    if (acc == 1ull) sink[0] = (double)acc;
}

// distinct random lines: index i -> line (i * prime) mod nlines, 16 words per line
__global__ void k_make_idx(long long *idx, long long n, long long nlines, long long mult)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        idx[i] = ((i * mult) % nlines) * 16;     // 16 x 8 B = one 128-B line
}

int main()
{
    char *buf;
    long long *idx;
    double *sink;
    CK(hipMalloc(&buf, kTable));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(buf, 1, kTable));
    const long long ng = 4LL << 20;               // 4 Mi gathers (32 MiB of index, streamed)
    CK(hipMalloc(&idx, ng * 8));
    const long long nlines = kTable / 128;
    k_make_idx<<<4096, 256>>>(idx, ng, nlines, 2654435761LL % nlines);
    CK(hipDeviceSynchronize());
    const long long bytes = 1LL << 30;            // 1 GiB per stream
    // flush the Infinity Cache between kernels: stream the rest of the table
    auto flush = [&] {
        k_stream<uint4><<<8192, 256>>>(reinterpret_cast<const uint4 *>(buf + bytes), (kTable - bytes) / 16, sink);
    };
    flush();
    k_stream<uint4><<<8192, 256>>>(reinterpret_cast<const uint4 *>(buf), bytes / 16, sink);
    flush();
    k_stream<unsigned long long><<<8192, 256>>>(reinterpret_cast<const unsigned long long *>(buf), bytes / 8, sink);
    flush();
    k_stream<unsigned int><<<8192, 256>>>(reinterpret_cast<const unsigned int *>(buf), bytes / 4, sink);
    flush();
    k_gather<false><<<4096, 256>>>(reinterpret_cast<const unsigned long long *>(buf), idx, ng, sink);
    flush();
    k_gather<true><<<4096, 256>>>(reinterpret_cast<const unsigned long long *>(buf), idx, ng, sink);
    flush();
    // 256 x 256 threads: 8 MiB of lines in flight, within the L2s
    k_gather2<8><<<256, 256>>>(reinterpret_cast<const unsigned long long *>(buf), idx, ng, sink);
    flush();
    k_gather2<64><<<256, 256>>>(reinterpret_cast<const unsigned long long *>(buf), idx, ng, sink);
    CK(hipDeviceSynchronize());
    printf("k_stream<uint4>: %lld bytes\n", bytes);
    printf("k_stream<unsigned long long>: %lld bytes\n", bytes);
    printf("k_stream<unsigned int>: %lld bytes\n", bytes);
    printf("k_gather<false>: %lld gathers of 8 B at distinct 128-B lines (+ %lld B of index stream)\n", ng, ng * 8);
    printf("k_gather<true>: %lld gathers of 8 B at distinct 128-B lines (+ %lld B of index stream)\n", ng, ng * 8);
    printf("k_gather2<8> / <64>: %lld lines, two dependent 8-B loads each, 8 / 64 B apart\n", ng);
    printf("flush kernels (k_stream<uint4> with n = %lld): %lld bytes each\n", (kTable - bytes) / 16, kTable - bytes);
    return 0;
}
