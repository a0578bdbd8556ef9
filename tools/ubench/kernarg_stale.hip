// Probe: are by-value kernel arguments of ~12 KB read consistently by every wave of every
// launch (scalar loads), when consecutive launches pass different contents?
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/kernarg_stale.hip -o tools/ubench/kernarg_stale
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big {
    unsigned tag;
    unsigned v[3100];  // ~12.4 KB
};
__global__ void k(Big b, unsigned* bad, int spin) {
    // wave-uniform index -> scalar loads from the kernarg segment at several offsets
    const int w = blockIdx.x;
    const unsigned t0 = b.tag;
    const unsigned a = b.v[(w * 37) % 3100];
    const unsigned c = b.v[3099 - (w % 500)];
    double x = w;
    for (int i = 0; i < spin; ++i) x = x * 1.0000001 + 1e-9;
    const unsigned e = b.v[(w * 13 + 7) % 3100];
    const bool ok = a == t0 && c == t0 && e == t0;
    if (!ok && threadIdx.x == 0) atomicAdd(bad, 1u);
    if (x == 12345.0) bad[1] = 1;
}
int main() {
    unsigned* d;
    hipMalloc(&d, 8);
    hipMemset(d, 0, 8);
    static Big b;
    int total = 0;
    for (int mode = 0; mode < 3; ++mode) {
        hipMemset(d, 0, 8);
        for (int it = 0; it < 400; ++it) {
            b.tag = it * 7919 + mode;
            for (int i = 0; i < 3100; ++i) b.v[i] = b.tag;
            hipLaunchKernelGGL(k, dim3(16000), dim3(64), 0, 0, b, d, mode == 2 ? 2000 : 10);
            if (mode == 1) hipDeviceSynchronize();
        }
        hipDeviceSynchronize();
        unsigned h[2];
        hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
        printf("mode %d (%s): mismatching waves %u of %d\n", mode,
               mode == 0 ? "back-to-back" : mode == 1 ? "sync each" : "long kernels", h[0],
               400 * 16000);
        total += h[0];
    }
    return total ? 1 : 0;
}
