// Diagnostic stand-in for a collective's kernel running beside the raw
// launches: `blocks` workgroups holding `lds` bytes of LDS each for ~`ns`
// nanoseconds (bounded: s_memrealtime, 100 MHz), launched on the caller's stream.
#include <hip/hip_runtime.h>

__global__ void k_block(unsigned long long ticks) {
    extern __shared__ float buf[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) buf[0] = 0.f;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int blocker_launch(int blocks, int threads, int lds, long long ns, void* stream) {
    hipLaunchKernelGGL(k_block, dim3(blocks), dim3(threads), lds, (hipStream_t)stream,
                       (unsigned long long)(ns / 10));
    return (int)hipGetLastError();
}
