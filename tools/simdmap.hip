// tools/simdmap.hip — diagnostics: which SIMD each wave of a workgroup runs on (HW_ID register).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/simdmap tools/simdmap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(uint32_t *out) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = hw;
}

int main() {
    uint32_t *d, h[64 * 16];
    hipMalloc(&d, sizeof(h));
    for (int threads : {256, 512}) {
        hipMemset(d, 0xff, sizeof(h));
        hipLaunchKernelGGL(k, dim3(4), dim3(threads), 0, 0, d);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        for (int b = 0; b < 4; b++) {
            printf("threads=%d block=%d:", threads, b);
            for (int w = 0; w < threads / 64; w++) {
                const uint32_t v = h[b * 16 + w];
                printf(" w%d:simd%u/wave%u/cu%u", w, (v >> 4) & 3, v & 15, (v >> 8) & 15);
            }
            printf("\n");
        }
    }
    return 0;
}
