// tools/mulrate.hip — microbenchmark (diagnostics): cycles per instruction of 32-bit integer multiply
// vs add / alignbit on gfx950, for a lone wave (latency and issue) and for a full chip (throughput).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mulrate tools/mulrate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP, int CHAINS>
__global__ void k(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) v[c] = seed + threadIdx.x * 7 + c;
    const long long t0 = clock64();
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#pragma unroll
            for (int c = 0; c < CHAINS; c++) {
                if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed | 1));
                if (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "v"(seed));
                if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 17" : "+v"(v[c]));
                if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[c]) : "v"(seed | 1));
            }
        }
    }
    const long long t1 = clock64();
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0x100000] = (uint32_t)(t1 - t0);
}

template <int OP, int CHAINS>
void run(const char *name, uint32_t *d, int blocks, int threads) {
    const uint32_t iters = 4096;
    hipLaunchKernelGGL((k<OP, CHAINS>), dim3(blocks), dim3(threads), 0, 0, d, iters, 12345u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<OP, CHAINS>), dim3(blocks), dim3(threads), 0, 0, d, iters, 12345u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint32_t cyc = 0;
    hipMemcpy(&cyc, d + 0x100000, 4, hipMemcpyDeviceToHost);
    const double n_inst = (double)iters * 8 * CHAINS;                 // per wave
    const double waves = (double)blocks * threads / 64;
    printf("%-14s chains=%d blocks=%5d thr=%4d: %7.2f cyc/inst (wave0 clock)  chip %8.1f G wave-inst/s\n", name, CHAINS,
           blocks, threads, cyc / n_inst, n_inst * waves / (ms * 1e-3) / 1e9);
}

int main() {
    uint32_t *d;
    hipMalloc(&d, (0x100000 + 64) * 4 + 256 * 1024 * 64 * 4);
    // lone wave: dependent chain (latency) and 8 independent chains (issue)
    run<0, 1>("mul_lo_u32", d, 1, 64);
    run<0, 8>("mul_lo_u32", d, 1, 64);
    run<1, 1>("add_u32", d, 1, 64);
    run<1, 8>("add_u32", d, 1, 64);
    run<2, 1>("alignbit", d, 1, 64);
    run<2, 8>("alignbit", d, 1, 64);
    run<3, 1>("mul_u32_u24", d, 1, 64);
    run<3, 8>("mul_u32_u24", d, 1, 64);
    // full chip: 256 CUs x 4 SIMDs x 4 waves
    run<0, 8>("mul_lo_u32", d, 1024, 256);
    run<1, 8>("add_u32", d, 1024, 256);
    run<3, 8>("mul_u32_u24", d, 1024, 256);
    return 0;
}
