// Probe: latency cost of one per-lane vector load at wave start, from the kernel-argument
// segment vs device memory (the renderer's tile-bin boxes are read this way), for a launch
// shaped like the renderer's (32400 one-wave workgroups, N fp64 FMA per lane).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/vload_src.hip -o tools/ubench/vload_src
#include <hip/hip_runtime.h>
#include <cstdio>
struct Args {
    unsigned long long tab[64];
    const unsigned long long* dtab;
    float* out;
    int W, H, gx;
};
template <int N, int SRC>
__global__ void __launch_bounds__(64) k(Args a) {
    const int t = blockIdx.x;
    const int lane = threadIdx.x & 63;
    unsigned long long v = 0;
    if (SRC == 1) v = a.tab[lane];
    if (SRC == 2) v = a.dtab[lane];
    const int x = (t % a.gx) * 8 + (lane & 7), y = (t / a.gx) * 8 + (lane >> 3);
    double p = x * 1e-3, q = y * 1e-3, u = p + q, w = p - q;
    // a ballot on the loaded value, as the renderer's box compare does
    const unsigned long long m = __ballot((unsigned)(v >> 3) > (unsigned)t);
    p += (double)(m & 1);
    for (int i = 0; i < N; ++i) {
        p = __builtin_fma(p, 1.0000001, 1e-9);
        q = __builtin_fma(q, 0.9999999, 1e-9);
        u = __builtin_fma(u, 1.0000002, 1e-9);
        w = __builtin_fma(w, 0.9999998, 1e-9);
    }
    if (x < a.W && y < a.H) {
        float* o = a.out + 3 * ((size_t)y * a.W + x);
        o[0] = (float)p;
        o[1] = (float)(q + u);
        o[2] = (float)w;
    }
}
template <int N, int S>
float run(Args a, int nt) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<N, S>), dim3(nt), dim3(64), 0, 0, a);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k<N, S>), dim3(nt), dim3(64), 0, 0, a);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms / 20 < best) best = ms / 20;
    }
    return best * 1000;
}
template <int N>
void row(Args a, int nt) {
    printf("N=%3d  none %6.2f  kernarg %6.2f  device %6.2f us\n", N, run<N, 0>(a, nt),
           run<N, 1>(a, nt), run<N, 2>(a, nt));
}
int main() {
    Args a;
    for (int i = 0; i < 64; ++i) a.tab[i] = 1000000ull * i;
    unsigned long long* d;
    hipMalloc(&d, 512);
    hipMemcpy(d, a.tab, 512, hipMemcpyHostToDevice);
    a.dtab = d;
    a.W = 1920;
    a.H = 1080;
    a.gx = 240;
    hipMalloc(&a.out, (size_t)a.W * a.H * 12);
    const int nt = 240 * 135;
    row<16>(a, nt);
    row<64>(a, nt);
    row<128>(a, nt);
    return 0;
}
