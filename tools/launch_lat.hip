// Host cost of a kernel launch onto an idle vs a busy stream (no profiler): tiny kernels launched back to back (the
// queue keeps work), and launched with a host pause after each one long enough for the queue to drain.
// Also with a second stream holding a long-running kernel, as the engine's side stream does.
// build: hipcc -O2 --offload-arch=gfx950 -o tools/launch_lat tools/launch_lat.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_tiny(unsigned *p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }
__global__ void k_spin(unsigned *p, long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) p[1 + blockIdx.x] = 1;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void pause_us(double us) { const double t = now_us(); while (now_us() - t < us) {} }

static void run(const char *what, hipStream_t s, unsigned *p, double pause, int n, int grid) {
    std::vector<double> d(n);
    for (int i = 0; i < n; i++) {
        const double t = now_us();
        hipLaunchKernelGGL(k_tiny, dim3(grid), dim3(256), 0, s, p);
        d[i] = now_us() - t;
        if (pause > 0) pause_us(pause);
    }
    hipStreamSynchronize(s);
    std::sort(d.begin(), d.end());
    double sum = 0;
    for (double x : d) sum += x;
    printf("%-48s launch us: mean %7.1f median %7.1f p90 %7.1f max %7.1f\n", what, sum / n, d[n / 2], d[n * 9 / 10], d[n - 1]);
}

int main() {
    unsigned *p;
    hipMalloc(&p, 4096 * sizeof(unsigned));
    hipStream_t a, b;
    hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    for (int i = 0; i < 50; i++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, a, p);
    hipDeviceSynchronize();
    for (int grid : {1, 256}) {
        char w[96];
        snprintf(w, sizeof w, "grid %d, back to back", grid); run(w, a, p, 0, 400, grid);
        snprintf(w, sizeof w, "grid %d, 30 us host pause after each", grid); run(w, a, p, 30, 400, grid);
        snprintf(w, sizeof w, "grid %d, 100 us host pause after each", grid); run(w, a, p, 100, 400, grid);
        // a long kernel on the second stream (87 workgroups, as a side-stream narrow checksum launch)
        hipLaunchKernelGGL(k_spin, dim3(87), dim3(768), 0, b, p, 2100ll * 1000 * 60);
        snprintf(w, sizeof w, "grid %d, 30 us pause, side stream busy", grid); run(w, a, p, 30, 400, grid);
        hipDeviceSynchronize();
    }
    printf("done\n");
    return 0;
}
