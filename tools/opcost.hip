// tools/opcost.hip — microbenchmark (diagnostics): throughput of the integer VALU operations the FarmHash chain,
// premix and formatter use, per SIMD, on a full chip. Each lane runs 8 independent dependency chains of one
// instruction (inline asm, so the opcode is exactly the one named); 1 or 4 waves per SIMD. Prints ns per
// wave-instruction per SIMD (time x SIMDs / wave-instructions) and the equivalent cycles at 2.4 GHz.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/opcost tools/opcost.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CH8(BODY) BODY(0) BODY(1) BODY(2) BODY(3) BODY(4) BODY(5) BODY(6) BODY(7)

template <int OP>
__global__ void k_op(uint32_t *out, uint32_t iters, uint32_t seed) {
    uint32_t x[8], y = seed * 3u + threadIdx.x, z = seed ^ 0x9e3779b9u;
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = seed + threadIdx.x * 7u + i;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
#define B(i)                                                                                                  \
    if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));                                  \
    if (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y));                                  \
    if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 19" : "+v"(x[i]));                                  \
    if (OP == 3) asm volatile("v_lshl_add_u32 %0, %0, 2, %0" : "+v"(x[i]));                                   \
    if (OP == 4) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));                     \
    if (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));                     \
    if (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));                               \
    if (OP == 7) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(y));                              \
    if (OP == 8) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));                  \
    if (OP == 9) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y));                         \
    if (OP == 10) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));               \
    if (OP == 11) asm volatile("v_lshlrev_b32 %0, 2, %0" : "+v"(x[i]));                                       \
    if (OP == 12) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));                     \
    if (OP == 13) asm volatile("v_add_u32 %0, 0x1234567, %0" : "+v"(x[i]));                                   \
    if (OP == 14) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));                              \
    if (OP == 15) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y));                              \
    if (OP == 16) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(x[i]) : "v"(x[i]));
            CH8(B)
#undef B
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static const char *names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_lshl_add_u32", "v_add3_u32", "v_perm_b32",
                              "v_mul_lo_u32", "v_mul_u32_u24", "v_mad_u32_u24", "v_cndmask_b32", "v_alignbyte_b32",
                              "v_lshlrev_b32", "v_or3_b32", "v_add_u32 (literal)", "v_mul_hi_u32", "v_pk_add_u16",
                              "v_mov_b32_dpp"};

template <int OP>
void run(uint32_t *d, int sms) {
    const uint32_t iters = 4096;
    double res[2];
    for (int w = 0; w < 2; w++) {
        const int thr = w == 0 ? 64 : 256;
        const int blocks = sms * 4;            // one workgroup per SIMD
        hipLaunchKernelGGL((k_op<OP>), dim3(blocks), dim3(thr), 0, 0, d, 16u, 7u);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL((k_op<OP>), dim3(blocks), dim3(thr), 0, 0, d, iters, 7u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double winst = (double)blocks * (thr / 64) * iters * 32;
        res[w] = ms * 1e6 * (sms * 4) / winst;            // ns per wave-instruction per SIMD
    }
    printf("%-22s 1 wave/SIMD: %6.3f ns (%5.2f cyc@2.4)   4 waves/SIMD: %6.3f ns (%5.2f cyc@2.4)\n", names[OP], res[0],
           res[0] * 2.4, res[1], res[1] * 2.4);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int sms = p.multiProcessorCount;
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, sms, p.clockRate);
    uint32_t *d;
    hipMalloc(&d, (size_t)sms * 4 * 256 * 4);
    run<0>(d, sms); run<1>(d, sms); run<2>(d, sms); run<3>(d, sms); run<4>(d, sms); run<5>(d, sms);
    run<6>(d, sms); run<7>(d, sms); run<8>(d, sms); run<9>(d, sms); run<10>(d, sms); run<11>(d, sms);
    run<12>(d, sms); run<13>(d, sms); run<14>(d, sms); run<15>(d, sms); run<16>(d, sms);
    return 0;
}
