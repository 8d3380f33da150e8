// tools/chain2.hip — microbenchmark (diagnostics): the FarmHash-mk chain of k_csr3 (g/f lanes in one wave, the h lane
// in another on the same SIMD, premixed entries read from LDS six blocks ahead) in two algebraic forms:
//   form 0 (production): r = ror(X ^ M, 19); Xf' = 5 r_f + 5 r_g + PF; Xg' = 5 r_g + Xf' + D   (g/f: 8 VALU, 5 deep)
//                        Xh' = 5 ror(Xh ^ Mh, 19) + KH                                        (h: 4 VALU, 4 deep)
//   form 1: with M' = ror(M, 19) premixed, r = ror(X, 19) ^ M' (the rotation distributes over xor), and
//           Xf' = 5 r_f + 5 r_g + PF, Xg' = (9 r_g + PG) + r_g + 5 r_f with PG = PF + D
//           (g/f: 10 VALU, 4 deep; v_xad_u32 folds an add into the xor); Xh' = 4 r_h + (r_h + KH) (h: 4 VALU, 3 deep)
// Both forms are checked equal block for block (mode 2). One workgroup of 512 threads per CU (waves 0-3 g/f, 4-7 h;
// 768 with four idle waves when STAGER=1), 32-block super steps, each lane reading its own entry.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/chain2 tools/chain2.hip ; run: tools/chain2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

constexpr uint32_t SB = 32, PF = 6, ROWS = 256;

__device__ __forceinline__ void gf0(uint32_t &Xg, uint32_t &Xf, uint32_t mg, uint32_t dd, uint32_t mf, uint32_t pf) {
    uint32_t tg, tf;
    asm volatile("v_xor_b32 %2, %0, %4\n\t"
                 "v_xor_b32 %3, %1, %6\n\t"
                 "v_alignbit_b32 %2, %2, %2, 19\n\t"
                 "v_alignbit_b32 %3, %3, %3, 19\n\t"
                 "v_lshl_add_u32 %2, %2, 2, %2\n\t"
                 "v_lshl_add_u32 %3, %3, 2, %3\n\t"
                 "v_add3_u32 %1, %3, %2, %7\n\t"
                 "v_add3_u32 %0, %2, %1, %5"
                 : "+v"(Xg), "+v"(Xf), "=&v"(tg), "=&v"(tf)
                 : "v"(mg), "v"(dd), "v"(mf), "v"(pf));
}
__device__ __forceinline__ void h0(uint32_t &Xh, uint32_t mh, uint32_t kh) {
    asm volatile("v_xor_b32 %0, %0, %1\n\t"
                 "v_alignbit_b32 %0, %0, %0, 19\n\t"
                 "v_lshl_add_u32 %0, %0, 2, %0\n\t"
                 "v_add_u32 %0, %0, %2"
                 : "+v"(Xh)
                 : "v"(mh), "v"(kh));
}
// form 1: mg, mf = ror(M, 19); pg = PF + D
__device__ __forceinline__ void gf1(uint32_t &Xg, uint32_t &Xf, uint32_t mg, uint32_t pg, uint32_t mf, uint32_t pf) {
    uint32_t ag, af, rg, rf, sg, r5, g5;
    asm volatile("v_alignbit_b32 %2, %0, %0, 19\n\t"          // A_g
                 "v_alignbit_b32 %3, %1, %1, 19\n\t"          // A_f
                 "v_xor_b32 %4, %2, %9\n\t"                   // r_g
                 "v_xor_b32 %5, %3, %11\n\t"                  // r_f
                 "v_xad_u32 %6, %2, %9, %10\n\t"              // S_g = r_g + PG
                 "v_lshl_add_u32 %7, %5, 2, %5\n\t"           // R = 5 r_f
                 "v_lshl_add_u32 %8, %4, 2, %4\n\t"           // G5 = 5 r_g
                 "v_lshl_add_u32 %6, %4, 3, %6\n\t"           // Q = 9 r_g + PG
                 "v_add3_u32 %1, %7, %8, %12\n\t"             // Xf' = R + G5 + PF
                 "v_add3_u32 %0, %6, %4, %7"                  // Xg' = Q + r_g + R
                 : "+v"(Xg), "+v"(Xf), "=&v"(ag), "=&v"(af), "=&v"(rg), "=&v"(rf), "=&v"(sg), "=&v"(r5), "=&v"(g5)
                 : "v"(mg), "v"(pg), "v"(mf), "v"(pf));
}
__device__ __forceinline__ void h1(uint32_t &Xh, uint32_t mh, uint32_t kh) {
    uint32_t a, r;
    asm volatile("v_alignbit_b32 %1, %0, %0, 19\n\t"
                 "v_xor_b32 %2, %1, %3\n\t"
                 "v_xad_u32 %0, %1, %3, %4\n\t"
                 "v_lshl_add_u32 %0, %2, 2, %0"
                 : "+v"(Xh), "=&v"(a), "=&v"(r)
                 : "v"(mh), "v"(kh));
}

__device__ __forceinline__ uint32_t rorh(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }

template <int FORM, int ROLE>
__device__ __forceinline__ uint32_t chain_loop(const char *Eb, uint32_t tid, uint32_t nsup, uint32_t seed) {
    uint32_t X0 = seed + tid, X1 = seed * 3u + tid;
    uint32_t code[SB];
#pragma unroll
    for (int i = 0; i < (int)SB; i++) code[i] = (uint32_t)(i * ROWS + tid) * 16u;
    for (uint32_t t = 0; t < nsup; t++) {
        uint4 va[PF + 1];
#pragma unroll
        for (int i = 0; i < (int)PF; i++) va[i] = *(const uint4 *)(Eb + code[i]);
#pragma unroll
        for (int i = 0; i < (int)SB; i++) {
            if (i + PF < SB) va[(i + PF) % (PF + 1)] = *(const uint4 *)(Eb + code[i + PF]);
            const uint4 A = va[i % (PF + 1)];
            if constexpr (ROLE == 0) {
                if constexpr (FORM == 0) gf0(X0, X1, A.x, A.y, A.z, A.w);
                else gf1(X0, X1, A.x, A.y, A.z, A.w);
            } else {
                if constexpr (FORM == 0) h0(X0, A.x, A.y);
                else h1(X0, A.x, A.y);
            }
        }
    }
    return X0 ^ X1;
}

// LDS: E[SB][ROWS] entries (16 B: {M, aux, M, PF} for g/f, {M, K, -, -} for h), one super step's worth, reused
template <int FORM, int STAGER>
__global__ void __launch_bounds__(ROWS * (2 + STAGER)) kchain(uint32_t *out, uint32_t nsup, uint32_t seed) {
    __shared__ uint4 E[SB][ROWS];
    const uint32_t tid = threadIdx.x & (ROWS - 1), role = threadIdx.x / ROWS;
    for (uint32_t i = threadIdx.x; i < SB * ROWS; i += blockDim.x) {
        const uint32_t x = i * 2654435761u + seed;
        E[i / ROWS][i % ROWS] = make_uint4(x, x ^ 0x5bd1e995u, x * 7u + 1u, x + 0x9e3779b9u);
    }
    __syncthreads();
    const char *Eb = (const char *)&E[0][0];
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t simd = (hw >> 4) & 3u;
    uint32_t r = 0;
    if (role == 0) r = chain_loop<FORM, 0>(Eb, tid, nsup, seed);
    else if (role == 1) r = chain_loop<FORM, 1>(Eb, tid, nsup, seed);
    else r = 0;                                             // idle waves (STAGER=1: resident, nothing to do)
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63u) == 0) out[256 * 768 + blockIdx.x * 16 + (threadIdx.x >> 6)] = simd | (role << 4);
}

// equality of the two forms over random blocks (one lane per sample)
__global__ void kcheck(uint32_t *bad, uint32_t n, uint32_t seed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s = i * 2654435761u + seed;
    auto nx = [&]() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; };
    uint32_t Xg = nx(), Xf = nx(), Xh = nx();
    uint32_t Yg = Xg, Yf = Xf, Yh = Xh;
    for (int k = 0; k < 64; k++) {
        const uint32_t Mg = nx(), Mf = nx(), Mh = nx(), PF = nx(), D = nx(), KH = nx();
        gf0(Xg, Xf, Mg, D, Mf, PF);
        h0(Xh, Mh, KH);
        gf1(Yg, Yf, rorh(Mg, 19), PF + D, rorh(Mf, 19), PF);
        h1(Yh, rorh(Mh, 19), KH);
    }
    if (Xg != Yg || Xf != Yf || Xh != Yh) atomicAdd(bad, 1u);
}

template <int FORM, int STAGER>
double run(uint32_t nsup, uint32_t *out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const dim3 grid(256), blk(ROWS * (2 + STAGER));
    hipLaunchKernelGGL((kchain<FORM, STAGER>), grid, blk, 0, 0, out, nsup, 1u);
    hipEventRecord(a, 0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL((kchain<FORM, STAGER>), grid, blk, 0, 0, out, nsup, (uint32_t)r + 2u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main() {
    uint32_t *out, *bad;
    hipMalloc(&out, 256 * 768 * 4 + 256 * 16 * 4);
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(kcheck, dim3(256), dim3(256), 0, 0, bad, 65536, 7u);
    uint32_t hb = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    const uint32_t nsup = 124500 / SB;                       // one 65,536-member row: 124,500 blocks
    const double f0 = run<0, 0>(nsup, out), f1 = run<1, 0>(nsup, out);
    const double f0s = run<0, 1>(nsup, out), f1s = run<1, 1>(nsup, out);
    // wave -> SIMD of the last run (768 threads): per role, which SIMD; and per CU whether waves w, w+4, w+8 share one
    {
        uint32_t ids[256 * 16];
        hipMemcpy(ids, out + 256 * 768, sizeof ids, hipMemcpyDeviceToHost);
        int same48 = 0, same4 = 0, tot = 0;
        for (int b = 0; b < 256; b++)
            for (int w = 0; w < 4; w++) {
                const uint32_t s0 = ids[b * 16 + w] & 3, s1 = ids[b * 16 + w + 4] & 3, s2 = ids[b * 16 + w + 8] & 3;
                same4 += s0 == s1; same48 += s0 == s1 && s1 == s2; tot++;
            }
        printf("{\"waves_w_w4_same_simd\": %d, \"waves_w_w4_w8_same_simd\": %d, \"pairs\": %d, \"cu0\": [", same4, same48, tot);
        for (int w = 0; w < 12; w++) printf("%s%u", w ? ", " : "", ids[w] & 3);
        printf("]}\n");
    }
    const double blk = (double)nsup * SB;
    printf("{\"forms_equal\": %s, \"blocks\": %.0f, \"form0_ms\": %.3f, \"form1_ms\": %.3f, \"form0_ns_per_block\": %.2f, "
           "\"form1_ns_per_block\": %.2f, \"form0_3waves_ms\": %.3f, \"form1_3waves_ms\": %.3f}\n",
           hb == 0 ? "true" : "false", blk, f0, f1, f0 * 1e6 / blk, f1 * 1e6 / blk, f0s, f1s);
    return hb == 0 ? 0 : 1;
}
