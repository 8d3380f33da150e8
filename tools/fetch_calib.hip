// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on the access patterns of this engine's kernels
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for what it was calibrated on; other widths are not).
// Each pattern moves a known number of bytes, well beyond the 256 MiB Infinity Cache, so the counters see HBM:
//   stream16   : 16 B per lane, coalesced, 2 GiB read (the checksum's row-word stream)
//   stream4    : 4 B per lane, coalesced, 2 GiB read
//   gather4    : one 4-B word per 64-B sector, sectors in a pseudo-random order over 16 GiB (the merges' row-word
//                gathers: one member word of a 256-KB row per change), 256 MiB of sectors touched
//   gather8    : the same with 8-B words (dissemination cells)
//   scatter4   : one 4-B store per 64-B sector, pseudo-random over 16 GiB, 256 MiB of sectors
//   copy16     : 16 B per lane read + 16 B per lane write, 1 GiB each
//   rowstream16: lane = row: every lane streams its own 256-KB region 16 B at a time (the checksum kernels' row-word
//                reads: one wave-instruction touches 64 rows, each row is read front to back), 4 GiB
// usage: rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o run --output-format csv -- ./fetch_calib
//        (then WRITE_SIZE in a second pass). Prints the algorithmic bytes of every kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_stream16(const uint4 *__restrict__ a, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void k_stream4(const uint32_t *__restrict__ a, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// sector s of the k-th access: a bijection of [0, nsec) (odd multiplier mod a power of two)
__device__ __forceinline__ size_t sector_of(size_t k, size_t nsec) { return (k * 0x9E3779B97F4A7C15ull) & (nsec - 1); }

template <typename T>
__global__ void k_gather(const T *__restrict__ a, size_t nsec, size_t count, uint32_t *sink) {
    uint32_t acc = 0;
    constexpr size_t per = 64 / sizeof(T);
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < count; k += (size_t)gridDim.x * blockDim.x) {
        const T v = a[sector_of(k, nsec) * per];
        acc ^= (uint32_t)v;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void k_scatter4(uint32_t *a, size_t nsec, size_t count) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < count; k += (size_t)gridDim.x * blockDim.x)
        a[sector_of(k, nsec) * 16] = (uint32_t)k;
}

// lane l of wave w reads row (w * 64 + l), 256 KB, 16 B per step
__global__ void k_rowstream16(const uint4 *__restrict__ a, size_t rows, uint32_t *sink) {
    const size_t row = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (row >= rows) return;
    const uint4 *p = a + row * (262144 / 16);
    uint32_t acc = 0;
    for (int i = 0; i < 262144 / 16; i += 4) {
        const uint4 v0 = p[i], v1 = p[i + 1], v2 = p[i + 2], v3 = p[i + 3];
        acc ^= v0.x + v1.y + v2.z + v3.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void k_copy16(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
    const size_t big = 16ull << 30, sec = big / 64;
    uint8_t *buf = nullptr, *buf2 = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&buf2, 1ull << 30));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, big));
    CK(hipMemset(buf2, 0, 1ull << 30));
    CK(hipDeviceSynchronize());
    const dim3 g(4096), b(256);
    const size_t n16 = (2ull << 30) / 16, n4 = (2ull << 30) / 4, touches = (256ull << 20) / 64;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const uint4 *)buf, n16, sink);
        hipLaunchKernelGGL(k_stream4, g, b, 0, 0, (const uint32_t *)(buf + (4ull << 30)), n4, sink);
        hipLaunchKernelGGL(k_gather<uint32_t>, g, b, 0, 0, (const uint32_t *)buf, sec, touches, sink);
        hipLaunchKernelGGL(k_gather<unsigned long long>, g, b, 0, 0, (const unsigned long long *)buf, sec, touches, sink);
        hipLaunchKernelGGL(k_scatter4, g, b, 0, 0, (uint32_t *)buf, sec, touches);
        hipLaunchKernelGGL(k_copy16, g, b, 0, 0, (const uint4 *)(buf + (8ull << 30)), (uint4 *)buf2, (1ull << 30) / 16);
        hipLaunchKernelGGL(k_rowstream16, dim3(16384 / 64), dim3(64), 0, 0, (const uint4 *)buf, (size_t)16384, sink);
        CK(hipDeviceSynchronize());
    }
    printf("{\"k_stream16\": {\"read\": %zu}, \"k_stream4\": {\"read\": %zu}, \"k_gather<unsigned int>\": {\"read_words\": %zu, "
           "\"read\": %zu, \"sectors\": %zu}, \"k_gather<unsigned long long>\": {\"read\": %zu, \"sectors\": %zu}, "
           "\"k_scatter4\": {\"write\": %zu, \"sectors\": %zu}, \"k_copy16\": {\"read\": %zu, \"write\": %zu}, "
           "\"k_rowstream16\": {\"read\": %zu}}\n",
           n16 * 16, n4 * 4, touches, touches * 4, touches, touches * 8, touches, touches * 4, touches, 1ull << 30, 1ull << 30,
           (size_t)16384 * 262144);
    hipFree(buf);
    hipFree(buf2);
    hipFree(sink);
    return 0;
}
