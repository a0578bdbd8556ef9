// Host cost of one kernel launch vs the size of its by-value arguments (MI355X, ROCm 7),
// the GPU held busy behind a spin kernel so the host never waits: hipLaunchKernelGGL and
// hipExtLaunchKernelGGL (with a stop event) of an empty kernel taking 64 B .. 14 KB of
// arguments, plus a bare hipEventRecord and a 16 B hipMemcpyAsync H2D for scale.
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench/launch_cost.hip -o tools/ubench/launch_cost
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

template <int N>
struct Args {
    int v[N / 4];
};
template <int N>
__global__ void k_empty(Args<N> a) {
    if (a.v[0] == 12345 && threadIdx.x == 1000) a.v[N / 4 - 1]++;
}
__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
}
#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                  \
            return 1;                                                           \
        }                                                                       \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int N>
static int bench(hipStream_t s, hipEvent_t ev, int n) {
    Args<N> a{};
    double best_plain = 1e9, best_ext = 1e9;
    for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000000LL);
        double t0 = now_us();
        for (int i = 0; i < n; i++) hipLaunchKernelGGL((k_empty<N>), dim3(1), dim3(64), 0, s, a);
        double t1 = now_us();
        for (int i = 0; i < n; i++)
            hipExtLaunchKernelGGL((k_empty<N>), dim3(1), dim3(64), 0, s, nullptr, ev, 0, a);
        double t2 = now_us();
        CK(hipStreamSynchronize(s));
        best_plain = std::min(best_plain, (t1 - t0) / n);
        best_ext = std::min(best_ext, (t2 - t1) / n);
    }
    std::printf("{\"arg_bytes\": %d, \"launch_us\": %.2f, \"ext_launch_us\": %.2f}\n", N, best_plain, best_ext);
    return 0;
}

int main() {
    hipStream_t s;
    hipEvent_t ev;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int n = 200;
    bench<64>(s, ev, n);
    bench<256>(s, ev, n);
    bench<1024>(s, ev, n);
    bench<4096>(s, ev, n);
    bench<8192>(s, ev, n);
    bench<14336>(s, ev, n);
    double best = 1e9, bestc = 1e9;
    void* d;
    void* h;
    CK(hipMalloc(&d, 4096));
    CK(hipHostMalloc(&h, 4096, hipHostMallocDefault));
    for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000000LL);
        double t0 = now_us();
        for (int i = 0; i < n; i++) hipEventRecord(ev, s);
        double t1 = now_us();
        for (int i = 0; i < n; i++) hipMemcpyAsync(d, h, 2048, hipMemcpyHostToDevice, s);
        double t2 = now_us();
        CK(hipStreamSynchronize(s));
        best = std::min(best, (t1 - t0) / n);
        bestc = std::min(bestc, (t2 - t1) / n);
    }
    std::printf("{\"hipEventRecord_us\": %.2f, \"hipMemcpyAsync_h2d_2KB_pinned_us\": %.2f}\n", best, bestc);
    return 0;
}
