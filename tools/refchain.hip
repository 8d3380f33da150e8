// tools/refchain.hip — microbenchmark (diagnostics): the fast path of a reference-string checksum kernel.
// One wave = 64 rows (lane = row). Every row's string is the reference string S_B shifted by the row's own byte
// shift s (here: a random per-lane constant in [0, SPREAD)). Per super step of 32 blocks the wave
//   (a) stages the next super step's window of S_B in LDS at the four byte alignments (lanes load words, v_alignbyte),
//   (b) streams the next super step's ~24 member words of its row from HBM and compares them with B (the dirty test
//       of the real kernel; never dirty here),
//   (c) runs the FarmHash-mk chain with the M() premixes in the wave over 32 blocks read from the window
//       (5 x ds_read_b32 per block at a per-lane address, PF blocks ahead).
// Prints ms per launch for 65,536 rows (1,024 waves) and for 8,192 rows, with 124,500 blocks per row.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/refchain tools/refchain.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr uint32_t C1 = 0xcc9e2d51u, C2 = 0x1b873593u;
__device__ __forceinline__ uint32_t ror(uint32_t v, int s) { return __builtin_rotateright32(v, s); }
__device__ __forceinline__ uint32_t x5(uint32_t h) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h));
    return r;
}
__device__ __forceinline__ uint32_t fold(uint32_t h, uint32_t mx, uint32_t add) { return x5(ror(h ^ mx, 19)) + 0xe6546b64u + add; }
__device__ __forceinline__ uint32_t M(uint32_t x) { return ror(x * C1, 17) * C2; }
// b + e * c1 as v_mul_lo_u32 + v_add_u32 (the compiler otherwise picks a 64-bit v_mad_u64_u32)
__device__ __forceinline__ uint32_t mad_c1(uint32_t e, uint32_t b) {
    uint32_t r;
    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(e), "v"(C1));
    return r + b;
}

constexpr int SB = 32;                 // blocks per super step
constexpr int PADW = 1024;             // zero words in front of S_B
constexpr int SPREADMAX = 1024;        // bytes
constexpr int WN = (SB * 20 + SPREADMAX + 64) / 4;   // window words per copy

// MODE bit 0: skip the dirty test; bit 1: skip the window staging (reads a stale window); bit 2: block words from
// registers (changing every super step, so the premixes stay in the loop); bit 3: b + e c1 as mul + add; bit 4: a
// scheduling barrier after every block (keeps the reads PF blocks ahead instead of hoisted to the super step's top);
// bit 5: window loads prefetched one super step ahead in registers
template <int PF, int MODE>
__global__ void __launch_bounds__(64) k_ref(const uint32_t *__restrict__ S, uint32_t sw, const uint32_t *__restrict__ rows,
                                            const uint32_t *__restrict__ B, uint32_t N, uint32_t nblk, uint32_t spread,
                                            uint32_t *out) {
    __shared__ uint32_t win[2][4][WN];
    const uint32_t lane = threadIdx.x;
    const uint32_t row = blockIdx.x * 64 + lane;
    const uint32_t s = (row * 2654435761u >> 7) % (spread + 1);
    // wave max of s, rounded up to 4
    uint32_t smax = s;
    for (int o = 32; o > 0; o >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, o, 64));
    const uint32_t SM = (smax + 3) & ~3u;
    const uint32_t delta0 = SM - s;                          // byte offset of block 0 of a super step in the window
    const uint32_t k = delta0 & 3u, w0 = delta0 >> 2;
    const uint32_t *rp = rows + (size_t)row * N;
    const uint32_t T = nblk / SB;
    constexpr int U = (WN + 63) / 64;
    uint32_t plo[U], phi[U];
    auto gload = [&](uint32_t t) {
        const int32_t wb = (int32_t)(160 * t) - (int32_t)(SM >> 2) + PADW;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i0 = min((uint32_t)(wb + (int32_t)(lane + 64 * u)), sw - 2);
            plo[u] = S[i0];
            phi[u] = S[i0 + 1];
        }
    };
    auto lput = [&](uint32_t t) {
        uint32_t *dst = &win[t & 1u][0][0];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = lane + 64 * u;
            if (i < (uint32_t)WN) {
                dst[i] = plo[u];
                dst[WN + i] = __builtin_amdgcn_alignbyte(phi[u], plo[u], 1);
                dst[2 * WN + i] = __builtin_amdgcn_alignbyte(phi[u], plo[u], 2);
                dst[3 * WN + i] = __builtin_amdgcn_alignbyte(phi[u], plo[u], 3);
            }
        }
    };
    auto stage = [&](uint32_t t) {
        // window of super step t: S_B bytes [640 t - SM, ...) = words from (640 t - SM) / 4 (+ PADW)
        if (MODE & 32) {
            lput(t);
            if (t + 1 < nblk / SB) gload(t + 1);
        } else {
            gload(t);
            lput(t);
        }
    };
    uint32_t dirty = 0;
    auto check = [&](uint32_t t) {
        // ~24 member words of the row around super step t, compared with B
        const uint32_t m0 = min(((640u * t) / 39u) & ~3u, N - 24);
        const uint4 *q = (const uint4 *)(rp + m0);
        const uint4 *b = (const uint4 *)(B + m0);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const uint4 x = q[i], y = b[i];
            dirty |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
        }
    };
    uint32_t h = 0x12345u + row, g = 0x777u ^ row, f = 3u * row;
    if (MODE & 32) {
        gload(0);
        lput(0);
        gload(1);
    } else if (!(MODE & 2)) stage(0);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t t = 0; t < T; t++) {
        if (!(MODE & 2) && t + 1 < T) stage(t + 1);
        else if ((MODE & 32) && t + 1 < T) stage(t + 1);
        if (!(MODE & 1)) check(t + 1);
        const uint32_t *base = &win[t & 1u][k][w0];
        uint32_t v[PF][5];
        auto ld = [&](int i) {
#pragma unroll
            for (int j = 0; j < 5; j++) v[i % PF][j] = (MODE & 4) ? (row * 31u + i * 7u + j + t) : base[5 * i + j];
        };
#pragma unroll
        for (int i = 0; i < PF - 1; i++) ld(i);
#pragma unroll
        for (int i = 0; i < SB; i++) {
            if (i + PF - 1 < SB) ld(i + PF - 1);
            const uint32_t a = v[i % PF][0], b = v[i % PF][1], c = v[i % PF][2], d = v[i % PF][3], e = v[i % PF][4];
            const uint32_t hn = fold(h + a, M(d), e);
            uint32_t gn = fold(g + b, M(c), a);
            uint32_t fn = fold(f + c, M((MODE & 8) ? mad_c1(e, b) : b + e * C1), d);
            fn += gn;
            gn += fn;
            h = hn; g = gn; f = fn;
            if (MODE & 16) __builtin_amdgcn_sched_barrier(0);
        }
    }
    out[row] = h ^ g ^ f ^ (dirty ? 1u : 0u);
}

template <int PF, int MODE>
float run(const uint32_t *S, uint32_t sw, const uint32_t *rows, const uint32_t *B, uint32_t N, uint32_t nrows, uint32_t nblk,
          uint32_t spread, uint32_t *out) {
    hipLaunchKernelGGL((k_ref<PF, MODE>), dim3(nrows / 64), dim3(64), 0, 0, S, sw, rows, B, N, 64u, spread, out);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_ref<PF, MODE>), dim3(nrows / 64), dim3(64), 0, 0, S, sw, rows, B, N, nblk, spread, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const uint32_t N = 65536, nblk = 124512;              // 3,891 super steps of 32 blocks
    const uint32_t sw = PADW + nblk * 5 + 4096;
    std::vector<uint32_t> hs(sw);
    for (uint32_t i = 0; i < sw; i++) hs[i] = i < PADW ? 0u : (i * 2654435761u) ^ 0x5bd1e995u;
    uint32_t *S, *rows, *B, *out;
    hipMalloc(&S, sw * 4);
    hipMemcpy(S, hs.data(), sw * 4, hipMemcpyHostToDevice);
    const size_t nr = 65536;
    if (hipMalloc(&rows, nr * N * 4) != hipSuccess) { printf("alloc rows failed\n"); return 1; }
    hipMemset(rows, 0, nr * N * 4);
    hipMalloc(&B, N * 4);
    hipMemset(B, 0, N * 4);
    hipMalloc(&out, nr * 4);
#define R(PF, MODE) run<PF, MODE>(S, sw, rows, B, N, nrows, nblk, spread, out)
    for (uint32_t nrows : {65536u, 8192u}) {
        for (uint32_t spread : {0u, 256u}) {
            printf("rows %6u spread %4u: regs %.3f regs+mul %.3f | nostage %.3f +mul %.3f +mul+sched(PF2 %.3f PF3 %.3f PF4 %.3f)"
                   " | full+mul+sched+pref PF3 %.3f PF4 %.3f, no dirty %.3f\n", nrows, spread,
                   R(3, 7), R(3, 15), R(3, 3), R(3, 11), R(2, 27), R(3, 27), R(4, 27), R(3, 56), R(4, 56), R(3, 57));
            fflush(stdout);
        }
    }
    return 0;
}
