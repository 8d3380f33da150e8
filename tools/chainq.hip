// tools/chainq.hip — microbenchmark (diagnostics): the FarmHash-mk chain in the "carried sum" form, one row per
// lane quad. Each block's h, g and f updates are rewritten over the values fed into the xor
// (Xh = h + a, Xg = g + b, Xf = f + c) so that every constant is folded off the chain:
//   F = 5 * ror(X ^ M, 19)  in every lane (M = M(d), M(c), M(b + e c1) for the h, g, f lanes)
//   Xg' = 2 F_g + F_f + PG,  Xf' = F_f + F_g + PF,  Xh' = F_h + KH
// with PG = 3C + 2a + d + b', PF = 2C + a + d + c', KH = C + e + a' (a', b', c' = the next block's words).
// Lanes of a quad are (g, f, h, 0); the partner term comes through one DPP quad permutation [1, 0, 3, 3],
// so a block is 5 VALU instructions for all three lanes of a row. Also times the single-lane forms of the
// same algebra (8 instructions for g/f, 4 for h) and checks every form against the plain FarmHash block.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/chainq tools/chainq.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

constexpr uint32_t C1 = 0xcc9e2d51u, C2 = 0x1b873593u, CM = 0xe6546b64u;
__host__ __device__ inline uint32_t ror(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }
__host__ __device__ inline uint32_t Mx(uint32_t x) { return ror(x * C1, 17) * C2; }
__device__ __forceinline__ uint32_t x5(uint32_t h) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h));
    return r;
}
__device__ __forceinline__ uint32_t lsh_add(uint32_t x, uint32_t s, uint32_t y) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(s), "v"(y));
    return r;
}

// one block of the quad chain: C++ (the compiler emits a separate v_mov_b32_dpp) or one asm sequence with the
// DPP folded into the add (s_nop 1: the DPP read of a VGPR needs two wait states after its VALU write)
template <bool ASM>
__device__ __forceinline__ void qstep(uint32_t &X, uint32_t m, uint32_t k, uint32_t sh) {
    if (ASM) {
        uint32_t t;
        asm("v_xor_b32 %0, %0, %2\n\t"
            "v_alignbit_b32 %0, %0, %0, 19\n\t"
            "v_lshl_add_u32 %0, %0, 2, %0\n\t"
            "s_nop 1\n\t"
            "v_add_u32_dpp %1, %0, %3 quad_perm:[1,0,3,3] row_mask:0xf bank_mask:0xf\n\t"
            "v_lshl_add_u32 %0, %0, %4, %1"
            : "+v"(X), "=&v"(t) : "v"(m), "v"(k), "v"(sh));
    } else {
        const uint32_t F = x5(__builtin_amdgcn_alignbit(X ^ m, X ^ m, 19));
        const uint32_t P = (uint32_t)__builtin_amdgcn_mov_dpp((int)F, 0xF1, 0xF, 0xF, false);
        X = lsh_add(F, sh, P + k);
    }
}

// per (block, lane) inputs {M, K}; lane role r = lane & 3 (g, f, h, zero)
__host__ __device__ inline void quad_inputs(const uint32_t *w, const uint32_t *wn, uint32_t r, uint32_t &m, uint32_t &k) {
    const uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
    const uint32_t an = wn ? wn[0] : 0u, bn = wn ? wn[1] : 0u, cn = wn ? wn[2] : 0u;
    if (r == 0) { m = Mx(c); k = 3u * CM + 2u * a + d + bn; }
    else if (r == 1) { m = Mx(b + e * C1); k = 2u * CM + a + d + cn; }
    else if (r == 2) { m = Mx(d); k = CM + e + an; }
    else { m = 0; k = 0; }
}

// SRC 0: inputs from registers (a rotating set of 8 blocks); 1: ds_read_b64 per block, 8 blocks ahead;
// 2: ds_read_b128 per two blocks, 8 blocks ahead; 3: as 1 and 4: as 0 with the asm block step. VERIFY: inputs of block j from io[] (nblk <= 64)
template <int SRC>
__global__ void __launch_bounds__(64) kq(uint32_t *out, const uint2 *io, uint32_t nblk, uint32_t seed, int verify) {
    constexpr int NR = 64;                                    // blocks resident in LDS (ring)
    __shared__ uint2 lds[NR * 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t role = lane & 3u;
    uint32_t X = out[64 * blockIdx.x + lane];                 // initial carried values (host-written)
    const uint32_t sh = role == 0 ? 1u : 0u;
    for (int j = 0; j < NR; j++) {
        uint2 v = verify ? io[j * 64 + lane] : make_uint2(seed * (j + 3) + lane * 77, seed ^ (j * 131 + lane));
        if (role == 3) v = make_uint2(0, 0);
        lds[j * 64 + lane] = v;
    }
    __syncthreads();
    uint2 reg[8];
#pragma unroll
    for (int j = 0; j < 8; j++) reg[j] = lds[j * 64 + lane];
    const long long t0 = clock64();
    for (uint32_t b = 0; b < nblk; b += 8) {
        uint2 nx[8];
        if (SRC == 1 || SRC == 3) {
#pragma unroll
            for (int j = 0; j < 8; j++) nx[j] = lds[((b + 8 + j) % NR) * 64 + lane];
        } else if (SRC == 2) {
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const uint4 q = *(const uint4 *)&lds[((((b + 8 + j) % NR) / 2) * 64 + lane) * 2];
                nx[j] = make_uint2(q.x, q.y);
                nx[j + 1] = make_uint2(q.z, q.w);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            qstep<(SRC >= 3)>(X, reg[j].x, reg[j].y, sh);
        }
        if (SRC == 0 || SRC == 4) {
            if (verify) {
#pragma unroll
                for (int j = 0; j < 8; j++) reg[j] = lds[((b + 8 + j) % NR) * 64 + lane];
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++) reg[j].y += X & 1u;       // not hoistable, off the chain
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) reg[j] = nx[j];
        }
    }
    const long long t1 = clock64();
    out[64 * blockIdx.x + lane] = X;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0x100000] = (uint32_t)(t1 - t0);
}

// single-lane carried-sum forms: MODE 0 g/f (8 VALU per block), MODE 1 h (4 VALU per block)
template <int MODE>
__global__ void __launch_bounds__(64) kr(uint32_t *out, uint32_t nblk, uint32_t seed) {
    const uint32_t lane = threadIdx.x;
    uint32_t in[8][4];
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
        for (int i = 0; i < 4; i++) in[j][i] = seed * (j + 3) + i * 77 + lane;
    uint32_t xg = seed + lane, xf = seed ^ lane, xh = seed * 3 + lane;
    const long long t0 = clock64();
    for (uint32_t b = 0; b < nblk; b += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (MODE == 0) {
                const uint32_t T = x5(__builtin_amdgcn_alignbit(xg ^ in[j][0], xg ^ in[j][0], 19));
                const uint32_t S = x5(__builtin_amdgcn_alignbit(xf ^ in[j][1], xf ^ in[j][1], 19));
                xf = S + T + in[j][2];
                xg = xf + T + in[j][3];
            } else {
                xh = x5(__builtin_amdgcn_alignbit(xh ^ in[j][0], xh ^ in[j][0], 19)) + in[j][1];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) in[j][1] += (xg ^ xh) & 1u;
    }
    const long long t1 = clock64();
    out[64 * blockIdx.x + lane] = xg ^ xf ^ xh;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0x100000] = (uint32_t)(t1 - t0);
}

template <typename K>
double timeit(K launch, uint32_t *d, uint32_t nblk, double &cyc) {
    launch(64u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    launch(nblk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint32_t c = 0;
    hipMemcpy(&c, d + 0x100000, 4, hipMemcpyDeviceToHost);
    cyc = (double)c / nblk;
    return ms;
}

struct FHs { uint32_t h, g, f; };
static void ref_block(FHs &s, const uint32_t *w) {
    const uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
    auto mur = [](uint32_t x, uint32_t h) { return ror(h ^ Mx(x), 19) * 5u + CM; };
    s.h += a; s.g += b; s.f += c;
    s.h = mur(d, s.h) + e;
    s.g = mur(c, s.g) + a;
    s.f = mur(b + e * C1, s.f) + d;
    s.f += s.g;
    s.g += s.f;
}

int main() {
    uint32_t *d;
    uint2 *io;
    hipMalloc(&d, (0x100000 + 64) * 4 * 4);
    hipMalloc(&io, 64 * 64 * sizeof(uint2));
    // correctness: 16 rows x 64 blocks through the quad kernel (SRC 0, verify) against the plain block
    {
        const int NB = 64;
        std::vector<uint32_t> w(16 * (NB + 1) * 5);
        srand(7);
        for (auto &x : w) x = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
        std::vector<FHs> st(16);
        std::vector<uint32_t> X0(64);
        std::vector<uint2> in(NB * 64);
        for (int r = 0; r < 16; r++) {
            st[r] = {(uint32_t)rand(), (uint32_t)rand() * 7u, (uint32_t)rand() * 13u};
            const uint32_t *w0 = &w[(r * (NB + 1)) * 5];
            X0[4 * r + 0] = st[r].g + w0[1];
            X0[4 * r + 1] = st[r].f + w0[2];
            X0[4 * r + 2] = st[r].h + w0[0];
            X0[4 * r + 3] = 0;
            for (int j = 0; j < NB; j++)
                for (uint32_t role = 0; role < 4; role++) {
                    uint32_t m, k;
                    quad_inputs(&w[(r * (NB + 1) + j) * 5], j + 1 < NB ? &w[(r * (NB + 1) + j + 1) * 5] : nullptr, role, m, k);
                    in[j * 64 + 4 * r + role] = make_uint2(m, k);
                }
            for (int j = 0; j < NB; j++) ref_block(st[r], &w[(r * (NB + 1) + j) * 5]);
        }
        hipMemcpy(io, in.data(), in.size() * sizeof(uint2), hipMemcpyHostToDevice);
        for (int v = 0; v < 2; v++) {
            hipMemcpy(d, X0.data(), 64 * 4, hipMemcpyHostToDevice);
            if (v == 0) hipLaunchKernelGGL((kq<0>), dim3(1), dim3(64), 0, 0, d, (const uint2 *)io, (uint32_t)NB, 1u, 1);
            else hipLaunchKernelGGL((kq<4>), dim3(1), dim3(64), 0, 0, d, (const uint2 *)io, (uint32_t)NB, 1u, 1);
            std::vector<uint32_t> X(64);
            hipMemcpy(X.data(), d, 64 * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int r = 0; r < 16; r++)
                bad += X[4 * r + 0] != st[r].g || X[4 * r + 1] != st[r].f || X[4 * r + 2] != st[r].h || X[4 * r + 3] != 0;
            printf("quad chain (%s) vs FarmHash block: %s (%d of 16 rows differ)\n", v ? "asm" : "C++", bad ? "MISMATCH" : "bit-exact", bad);
        }
    }
    const uint32_t nb = 131072;
    for (int blocks : {1, 256, 1024, 2048, 4096}) {
        printf("--- %d waves of 64 lanes ---\n", blocks);
        double cyc;
        double ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kq<0>), dim3(blocks), dim3(64), 0, 0, d, (const uint2 *)io, n, 3u, 0); }, d, nb, cyc);
        printf("quad h+g/f (registers)   %7.2f cyc/block | %8.3f ms for %u blocks (%d rows)\n", cyc, ms, nb, blocks * 16);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kq<1>), dim3(blocks), dim3(64), 0, 0, d, (const uint2 *)io, n, 3u, 0); }, d, nb, cyc);
        printf("quad h+g/f (LDS b64)     %7.2f cyc/block | %8.3f ms\n", cyc, ms);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kq<2>), dim3(blocks), dim3(64), 0, 0, d, (const uint2 *)io, n, 3u, 0); }, d, nb, cyc);
        printf("quad h+g/f (LDS b128/2)  %7.2f cyc/block | %8.3f ms\n", cyc, ms);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kq<4>), dim3(blocks), dim3(64), 0, 0, d, (const uint2 *)io, n, 3u, 0); }, d, nb, cyc);
        printf("quad asm (registers)     %7.2f cyc/block | %8.3f ms\n", cyc, ms);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kq<3>), dim3(blocks), dim3(64), 0, 0, d, (const uint2 *)io, n, 3u, 0); }, d, nb, cyc);
        printf("quad asm (LDS b64)       %7.2f cyc/block | %8.3f ms\n", cyc, ms);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kr<0>), dim3(blocks), dim3(64), 0, 0, d, n, 3u); }, d, nb, cyc);
        printf("lane g/f (registers)     %7.2f cyc/block | %8.3f ms (%d rows)\n", cyc, ms, blocks * 64);
        ms = timeit([&](uint32_t n) { hipLaunchKernelGGL((kr<1>), dim3(blocks), dim3(64), 0, 0, d, n, 3u); }, d, nb, cyc);
        printf("lane h (registers)       %7.2f cyc/block | %8.3f ms\n", cyc, ms);
    }
    hipFree(io);
    hipFree(d);
    return 0;
}
