// Microbenchmark: issue rate of v_fma_f32, v_pk_fma_f32, v_fma_f64 on gfx950
// (8 independent accumulator chains per lane, 2048 blocks x 256 threads).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ void k_f32(float* out, float a, float b) {
    float x[8];
    for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 1e-3f + k;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_fmaf(x[k], a, b);
    float s = 0; for (int k = 0; k < 8; k++) s += x[k];
    if (s == 12345.f) out[0] = s;
}
__global__ void k_pk(float* out, float a, float b) {
    float2v x[8];
    for (int k = 0; k < 8; k++) x[k] = float2v{threadIdx.x * 1e-3f + k, k * 0.5f};
    const float2v va = {a, a}, vb = {b, b};
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_elementwise_fma(x[k], va, vb);
    float s = 0; for (int k = 0; k < 8; k++) s += x[k].x + x[k].y;
    if (s == 12345.f) out[0] = s;
}
__global__ void k_f64(double* out, double a, double b) {
    double x[8];
    for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_fma(x[k], a, b);
    double s = 0; for (int k = 0; k < 8; k++) s += x[k];
    if (s == 12345.) out[0] = s;
}
int main() {
    float* f; double* d;
    hipMalloc(&f, 64); hipMalloc(&d, 64);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 2048 * 4, threads = 256;
    const double lanes = (double)blocks * threads;
    for (int rep = 0; rep < 2; rep++) {
        float ms;
        hipEventRecord(e0); hipLaunchKernelGGL(k_f32, blocks, threads, 0, 0, f, 0.999f, 1e-3f); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("v_fma_f32    : %.1f TFLOP/s (%.3f ms)\n", lanes * ITERS * 8 * 2 / (ms * 1e-3) / 1e12, ms);
        hipEventRecord(e0); hipLaunchKernelGGL(k_pk, blocks, threads, 0, 0, f, 0.999f, 1e-3f); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("v_pk_fma_f32 : %.1f TFLOP/s (%.3f ms)\n", lanes * ITERS * 8 * 4 / (ms * 1e-3) / 1e12, ms);
        hipEventRecord(e0); hipLaunchKernelGGL(k_f64, blocks, threads, 0, 0, d, 0.999, 1e-3); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("v_fma_f64    : %.1f TFLOP/s (%.3f ms)\n", lanes * ITERS * 8 * 2 / (ms * 1e-3) / 1e12, ms);
    }
    return 0;
}
