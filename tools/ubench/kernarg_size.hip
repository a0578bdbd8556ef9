// Probe: largest by-value kernel argument the HIP runtime passes intact (MI355X).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int N>
struct Big {
    int n;
    int v[N];
};
template <int N>
__global__ void k(Big<N> b, long long* out) {
    long long s = 0;
    for (int i = threadIdx.x; i < N; i += 64) s += b.v[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (threadIdx.x == 0) *out = s;
}
template <int N>
int run(long long* d) {
    static Big<N> b;
    b.n = N;
    long long ref = 0;
    for (int i = 0; i < N; i++) { b.v[i] = i * 7 + 3; ref += b.v[i]; }
    hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, 0, b, d);
    hipError_t e = hipDeviceSynchronize();
    long long h = -1;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("arg bytes %6zu: %s, sum %s\n", sizeof(Big<N>), hipGetErrorString(e), h == ref ? "ok" : "WRONG");
    return h == ref;
}
int main() {
    long long* d;
    hipMalloc(&d, 8);
    run<1000>(d);
    run<1020>(d);
    run<1100>(d);
    run<2000>(d);
    run<4000>(d);
    return 0;
}
