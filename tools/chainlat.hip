// tools/chainlat.hip — microbenchmark (diagnostics): the FarmHash-mk chain bound on gfx950.
// Cycles per 20-byte block of the h and coupled g/f chains of one row per lane, with the data-only work
// (M(x) premixes) either precomputed (chain only) or done in the same wave, and inputs from registers
// or from LDS. Shows the latency floor of a one-row launch and the issue cost per block.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/chainlat tools/chainlat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint32_t C1 = 0xcc9e2d51u, C2 = 0x1b873593u;
__device__ __forceinline__ uint32_t ror(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }
__device__ __forceinline__ uint32_t x5(uint32_t h) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h));
    return r;
}
__device__ __forceinline__ uint32_t fold(uint32_t h, uint32_t mx, uint32_t add) { return x5(ror(h ^ mx, 19)) + 0xe6546b64u + add; }
__device__ __forceinline__ uint32_t M(uint32_t x) { return ror(x * C1, 17) * C2; }

// MODE 0: g/f chain only, premixed inputs in registers
// MODE 1: h + g/f chains, premixed inputs in registers
// MODE 2: h + g/f chains with the M() premixes computed in the wave (registers)
// MODE 3: h + g/f chains, premixed inputs from LDS (ds_read_b128 x2 + b32 per block, lane-contiguous)
// MODE 4: h chain only, premixed
// MODE 5: h + gf, premixed 12-word block records in LDS read by 3 ds_read_b128 (lane stride = 4 mod 64 words:
//         conflict-free), the next 4 blocks' reads issued before the current 4 blocks' arithmetic
// MODE 6: gf only, as 5 (2 ds_read_b128 per block)
template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t nblk, uint32_t seed) {
    __shared__ uint4 lds[64 * 3 * 8];
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t in[8][9];
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
        for (int i = 0; i < 9; i++) in[j][i] = seed * (j + 3) + i * 77 + lane;
    if (MODE == 3 && threadIdx.x < 64) {
        for (int j = 0; j < 8; j++) {
            lds[(lane * 8 + j) * 3 + 0] = make_uint4(in[j][0], in[j][1], in[j][2], in[j][3]);
            lds[(lane * 8 + j) * 3 + 1] = make_uint4(in[j][4], in[j][5], in[j][6], in[j][7]);
            lds[(lane * 8 + j) * 3 + 2] = make_uint4(in[j][8], 0, 0, 0);
        }
    }
    __syncthreads();
    uint32_t h = seed + lane, g = seed ^ lane, f = seed * 3 + lane;
    const long long t0 = clock64();
    for (uint32_t b = 0; b < nblk; b += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint32_t a = in[j][0], bb = in[j][1], c = in[j][2], d = in[j][3], e = in[j][4];
            uint32_t mh = in[j][5], mc = in[j][6], mx = in[j][7];
            if (MODE == 3) {
                const uint4 p = lds[((threadIdx.x & 63) * 8 + j) * 3 + 0];
                const uint4 q = lds[((threadIdx.x & 63) * 8 + j) * 3 + 1];
                a = p.x; bb = p.y; c = p.z; d = p.w; e = q.x; mh = q.y; mc = q.z; mx = q.w;
            }
            if (MODE == 2) {
                mh = M(d); mc = M(c); mx = M(bb + e * C1);
            }
            if (MODE != 0) h = fold(h + a, mh, e);
            if (MODE != 4) {
                const uint32_t gn = fold(g + bb, mc, a);
                uint32_t fn = fold(f + c, mx, d);
                fn += gn;
                g = gn + fn;
                f = fn;
            }
        }
        if (MODE == 2) {   // keep the compiler from hoisting M() out of the loop
#pragma unroll
            for (int j = 0; j < 8; j++) in[j][j & 3] += h;
        }
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = h ^ g ^ f;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0x100000] = (uint32_t)(t1 - t0);
}

template <int MODE>
__global__ void __launch_bounds__(64) k2(uint32_t *out, uint32_t nblk, uint32_t seed) {
    constexpr int NBR = 16, STRIDE = NBR * 12 + 4;          // 16 block records per lane, stride 196 words
    __shared__ uint32_t lds[64 * STRIDE];
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t *my = lds + lane * STRIDE;
    for (int j = 0; j < NBR * 12; j++) my[j] = seed * (j + 3) + lane * 77 + j;
    __syncthreads();
    uint32_t h = seed + lane, g = seed ^ lane, f = seed * 3 + lane;
    uint4 cur[4][3], nxt[4][3];
    auto ld = [&](uint32_t base, uint4 (&x)[4][3]) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 *q = (const uint4 *)(my + ((base + k) % NBR) * 12);
            x[k][0] = q[0];
            x[k][1] = q[1];
            if (MODE == 5) x[k][2] = q[2];
        }
    };
    ld(0, cur);
    const long long t0 = clock64();
    for (uint32_t b = 0; b < nblk; b += 4) {
        ld(b + 4, nxt);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // record: {b, c, Mc, Mx} {C+a, C+d, ., .} {a, Md, C+e, .}
            const uint4 p = cur[k][0], q = cur[k][1], r = cur[k][2];
            if (MODE == 5) h = x5(__builtin_rotateright32((h + r.x) ^ r.y, 19)) + r.z;
            const uint32_t gn = x5(__builtin_rotateright32((g + p.x) ^ p.z, 19)) + q.x;
            uint32_t fn = x5(__builtin_rotateright32((f + p.y) ^ p.w, 19)) + q.y;
            fn += gn;
            g = gn + fn;
            f = fn;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int i = 0; i < 3; i++) cur[k][i] = nxt[k][i];
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = h ^ g ^ f;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0x100000] = (uint32_t)(t1 - t0);
}

template <int MODE>
void run2(const char *name, uint32_t *d, int blocks, uint32_t nblk) {
    hipLaunchKernelGGL((k2<MODE>), dim3(blocks), dim3(64), 0, 0, d, 64u, 12345u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k2<MODE>), dim3(blocks), dim3(64), 0, 0, d, nblk, 12345u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint32_t cyc = 0;
    hipMemcpy(&cyc, d + 0x100000, 4, hipMemcpyDeviceToHost);
    printf("%-22s blocks=%5d thr=  64: wave0 %7.2f cyc/block | %8.3f ms for %u blocks\n", name, blocks, (double)cyc / nblk, ms, nblk);
}

template <int MODE>
void run(const char *name, uint32_t *d, int blocks, int threads, uint32_t nblk) {
    hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(threads), 0, 0, d, 64u, 12345u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<MODE>), dim3(blocks), dim3(threads), 0, 0, d, nblk, 12345u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint32_t cyc = 0;
    hipMemcpy(&cyc, d + 0x100000, 4, hipMemcpyDeviceToHost);
    const double rows = (double)blocks * threads;
    printf("%-22s blocks=%5d thr=%4d: wave0 %7.2f cyc/block | %8.3f ms for %u blocks | %.3e row-blocks/s\n", name, blocks,
           threads, (double)cyc / nblk, ms, nblk, rows * nblk / (ms * 1e-3));
}

int main() {
    uint32_t *d;
    hipMalloc(&d, (0x100000 + 64) * 4 * 16);
    const uint32_t nb = 131072;
    for (int cfg = 0; cfg < 4; cfg++) {
        const int blocks = cfg == 0 ? 1 : cfg == 1 ? 256 : cfg == 2 ? 1024 : 2048;
        const int thr = 64;
        printf("--- %d waves of 64 lanes (rows) ---\n", blocks);
        run<0>("gf chain (premixed)", d, blocks, thr, nb);
        run<4>("h chain (premixed)", d, blocks, thr, nb);
        run<1>("h+gf (premixed)", d, blocks, thr, nb);
        run<2>("h+gf (M in wave)", d, blocks, thr, nb);
        run<3>("h+gf (premixed, LDS)", d, blocks, thr, nb);
        run2<5>("h+gf (LDS b128 recs)", d, blocks, nb);
        run2<6>("gf (LDS b128 recs)", d, blocks, nb);
    }
    hipFree(d);
    return 0;
}
