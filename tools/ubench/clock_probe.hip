// Shader clock of the GPU at a point in a stream: one wave spins ~2 us of the 100 MHz
// constant clock (s_memrealtime) and counts shader-clock cycles (s_memtime) over it, so
// out = {shader cycles, realtime ticks}; MHz = 100 * cycles / ticks.  tools/window_probe.py
// brackets every timed window with it (is a slow window a slower clock?).
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/ubench/clock_probe.hip -o tools/ubench/libclock_probe.so
#include <hip/hip_runtime.h>

__global__ void k_clock(unsigned long long* out, unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = r0;
    while (r1 - r0 < ticks) r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    out[0] = c1 - c0;
    out[1] = r1 - r0;
}

extern "C" int clock_probe(void* stream, unsigned long long* d_out, unsigned long long ticks) {
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), d_out, ticks);
    return (int)hipGetLastError();
}
