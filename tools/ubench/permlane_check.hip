// Semantics check of v_permlane32_swap_b32 (__builtin_amdgcn_permlane32_swap)
// on gfx950: lane l passes old = l, src = 100 + l; prints both results for
// lanes 0, 31, 32, 63.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out) {
    const unsigned l = threadIdx.x;
    const auto r = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
    out[2 * l] = r[0];
    out[2 * l + 1] = r[1];
}

int main() {
    unsigned* d;
    (void)hipMalloc(&d, 128 * sizeof(unsigned));
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
    unsigned h[128];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l : {0, 1, 31, 32, 33, 63})
        printf("lane %2d: first %3u second %3u\n", l, h[2 * l], h[2 * l + 1]);
    (void)hipFree(d);
    return 0;
}
