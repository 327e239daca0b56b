// Debug: semantics of v_permlane16_swap_b32 / v_permlane32_swap_b32 on gfx950 (which lanes move).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__global__ void k(unsigned *o) {
    const unsigned l = threadIdx.x;
    u32x2 r = __builtin_amdgcn_permlane16_swap(1000 + l, 2000 + l, false, false);
    o[l] = r.x; o[64 + l] = r.y;
    u32x2 s = __builtin_amdgcn_permlane32_swap(1000 + l, 2000 + l, false, false);
    o[128 + l] = s.x; o[192 + l] = s.y;
}
int main() {
    unsigned *d, h[256];
    hipMalloc(&d, 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    for (int t = 0; t < 4; ++t) {
        printf("%s %s:", t < 2 ? "p16" : "p32", t % 2 ? "y" : "x");
        for (int l = 0; l < 64; l += 4) printf(" %u", h[t * 64 + l]);
        printf("\n");
    }
    return 0;
}
