// Probe: cost of serial scalar kernel-argument round trips at wave start, for a launch
// shaped like the renderer's (32400 one-wave workgroups, N fp64 FMAs per lane, 12 B/px out).
// Each wave performs R dependent s_loads (the next offset comes from the previous value).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/smem_chain.hip -o tools/ubench/smem_chain
#include <hip/hip_runtime.h>
#include <cstdio>
struct Args {
    int next[64];  // next[i] = i + 1 (kept opaque to the compiler)
    float* out;
    int W, H, gx;
};
template <int N, int R>
__global__ void __launch_bounds__(64) k(Args a) {
    int idx = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) idx = a.next[idx & 63];  // dependent scalar loads
    const int t = blockIdx.x + (idx & 0);                // tie the chain to the work
    const int lane = threadIdx.x & 63;
    const int x = (t % a.gx) * 8 + (lane & 7), y = (t / a.gx) * 8 + (lane >> 3);
    double p = x * 1e-3 + idx, q = y * 1e-3, u = p + q, v = p - q;
    for (int i = 0; i < N; ++i) {
        p = __builtin_fma(p, 1.0000001, 1e-9);
        q = __builtin_fma(q, 0.9999999, 1e-9);
        u = __builtin_fma(u, 1.0000002, 1e-9);
        v = __builtin_fma(v, 0.9999998, 1e-9);
    }
    if (x < a.W && y < a.H) {
        float* o = a.out + 3 * ((size_t)y * a.W + x);
        o[0] = (float)p;
        o[1] = (float)(q + u);
        o[2] = (float)v;
    }
}
template <int N, int R>
float run(Args a, int nt) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<N, R>), dim3(nt), dim3(64), 0, 0, a);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k<N, R>), dim3(nt), dim3(64), 0, 0, a);
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
    printf("N=%3d  R=0 %6.2f  R=1 %6.2f  R=2 %6.2f  R=4 %6.2f  R=8 %6.2f us\n", N, run<N, 0>(a, nt),
           run<N, 1>(a, nt), run<N, 2>(a, nt), run<N, 4>(a, nt), run<N, 8>(a, nt));
}
int main() {
    Args a;
    for (int i = 0; i < 64; ++i) a.next[i] = (i + 1) & 63;
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
