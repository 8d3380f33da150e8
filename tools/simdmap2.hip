// tools/simdmap2.hip — diagnostics: SIMD placement of the waves of a full grid of multi-wave workgroups
// (HW_ID / XCC_ID of every wave while all of them are resident), as waves per SIMD per CU.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/simdmap2 tools/simdmap2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

template <int LDSW>
__global__ void k(uint32_t *out, uint32_t spin) {
    __shared__ uint32_t pad[LDSW];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    pad[threadIdx.x % LDSW] = hw;
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {}
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        out[2 * (blockIdx.x * 16 + (threadIdx.x >> 6))] = hw;
        out[2 * (blockIdx.x * 16 + (threadIdx.x >> 6)) + 1] = xcc + pad[(threadIdx.x + 1) % LDSW] * 0;
    }
}

void run(int grid, int threads, int ldsw_kind) {
    uint32_t *d;
    hipMalloc(&d, grid * 16 * 8);
    if (ldsw_kind == 0) hipLaunchKernelGGL((k<6000>), dim3(grid), dim3(threads), 0, 0, d, 200000u);
    else hipLaunchKernelGGL((k<1024>), dim3(grid), dim3(threads), 0, 0, d, 200000u);
    std::vector<uint32_t> h(grid * 16 * 2);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::map<uint64_t, std::vector<int>> cu;        // (xcc, se, sh, cu) -> waves per simd
    std::map<int, int> wave_simd[16];
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < threads / 64; w++) {
            const uint32_t v = h[2 * (b * 16 + w)], x = h[2 * (b * 16 + w) + 1] & 15;
            const uint64_t key = ((uint64_t)x << 32) | (((v >> 13) & 7) << 8) | (((v >> 12) & 1) << 4) | ((v >> 8) & 15);
            auto &c = cu[key];
            if (c.empty()) c.assign(4, 0);
            c[(v >> 4) & 3]++;
            wave_simd[w][(v >> 4) & 3]++;
        }
    // role composition of every SIMD: how many wave-0s and wave-1s (formatter / hasher of k_checksum3) share it
    std::map<uint64_t, std::vector<int>> simd_roles;        // (cu key, simd) -> waves per role
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < threads / 64; w++) {
            const uint32_t v = h[2 * (b * 16 + w)], x = h[2 * (b * 16 + w) + 1] & 15;
            const uint64_t key = ((uint64_t)x << 40) | ((uint64_t)((v >> 4) & 3) << 32) | (((v >> 13) & 7) << 8) |
                                 (((v >> 12) & 1) << 4) | ((v >> 8) & 15);
            auto &c = simd_roles[key];
            if (c.empty()) c.assign(threads / 64, 0);
            c[w]++;
        }
    std::map<std::vector<int>, int> rhist;
    for (auto &kv : simd_roles) rhist[kv.second]++;
    printf("   waves of each role per SIMD (wave 0, wave 1, ...) -> SIMDs:\n");
    for (auto &kv : rhist) {
        printf("     [");
        for (size_t i = 0; i < kv.first.size(); i++) printf("%s%d", i ? " " : "", kv.first[i]);
        printf("] x %d\n", kv.second);
    }
    std::map<std::vector<int>, int> hist;
    for (auto &kv : cu) hist[kv.second]++;
    printf("grid %d x %d threads (LDS %s): %zu CUs used; waves per SIMD pattern -> CUs:\n", grid, threads,
           ldsw_kind == 0 ? "24 KB" : "4 KB", cu.size());
    for (auto &kv : hist) printf("   [%d %d %d %d] x %d\n", kv.first[0], kv.first[1], kv.first[2], kv.first[3], kv.second);
    for (int w = 0; w < threads / 64; w++) {
        printf("   wave %d of a workgroup -> simd histogram:", w);
        for (int s = 0; s < 4; s++) printf(" %d", wave_simd[w][s]);
        printf("\n");
    }
    hipFree(d);
}

int main() {
    run(1024, 128, 0);
    run(512, 128, 0);
    run(1024, 128, 1);
    run(768, 320, 0);
    run(4096, 64, 1);
    return 0;
}
