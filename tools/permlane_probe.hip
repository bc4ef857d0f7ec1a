// permlane_probe.hip -- checks the lane semantics of gfx950's v_permlane16_swap /
// v_permlane32_swap as the 3D tile wavefront (kernels.hip k_trsv_tile3d) uses them.
// Build: hipcc --offload-arch=gfx950 -O2 tools/permlane_probe.hip -o tools/permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned *out)
{
    const unsigned l = threadIdx.x;
    const unsigned a = 1000 + l, b = 2000 + l;
    auto p16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    auto p32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[l] = p16[0];
    out[64 + l] = p16[1];
    out[128 + l] = p32[0];
    out[192 + l] = p32[1];
    // one register as both operands (a row-pair / half swap in place?)
    unsigned c = 3000 + l, d = 4000 + l;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0" : "+v"(c));
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0" : "+v"(d));
    out[256 + l] = c;
    out[320 + l] = d;
}

int main()
{
    unsigned *d, h[384];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *nm[6] = {"p16.vdst", "p16.src", "p32.vdst", "p32.src", "p16 self", "p32 self"};
    for (int q = 0; q < 6; q++) {
        printf("%s:", nm[q]);
        for (int l = 0; l < 64; l += 8) printf(" [%d]=%u", l, h[q * 64 + l]);
        printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
