// Kernel-argument latency probe: per wave, s_memrealtime at entry, after a
// scalar load of a kernel argument far into a 1 KiB argument block, after a
// vector load of another argument-block line, and after a dependent global load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/kernarg tools/probes/kernarg.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Big { const float* p[128]; };

__global__ void k_args(Big b, unsigned long long* rec, int pick) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_sched_barrier(0);
    const float* s = b.p[100];  // scalar load of a late kernarg line
    unsigned long long t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : "s"(s));
    const float* v = b.p[(threadIdx.x + pick) & 127];  // vector load from the argument block
    float x = *v;
    unsigned long long t2;
    asm volatile("s_waitcnt vmcnt(0)\n s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t2) : "v"(x));
    float y = s[threadIdx.x & 63];  // a global load (L2 / HBM)
    unsigned long long t3;
    asm volatile("s_waitcnt vmcnt(0)\n s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t3) : "v"(y));
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* r = rec + ((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 4;
        r[0] = t0;
        r[1] = t1 - t0;
        r[2] = t2 - t1;
        r[3] = t3 - t2 + (x == 12345.f ? 1 : 0) + (y == 12345.f ? 1 : 0);
    }
}

int main() {
    const int B = 256, T = 1024, W = T / 64;
    float* buf;
    hipMalloc(&buf, 1 << 20);
    hipMemset(buf, 0, 1 << 20);
    Big b;
    for (int i = 0; i < 128; ++i) b.p[i] = buf + i * 64;
    unsigned long long* rec;
    hipMalloc(&rec, sizeof(unsigned long long) * B * W * 4);
    std::vector<unsigned long long> h(B * W * 4);
    const char* names[3] = {"scalar kernarg load", "vector kernarg load", "global load"};
    for (int it = 0; it < 6; ++it) {
        for (int k = 0; k < 10; ++k) hipLaunchKernelGGL(k_args, dim3(B), dim3(T), 0, 0, b, rec, k);
        hipDeviceSynchronize();
        if (it < 2) continue;
        hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost);
        printf("launch %d:", it);
        for (int c = 1; c < 4; ++c) {
            std::vector<double> v;
            for (int w = 0; w < B * W; ++w) v.push_back((double)h[w * 4 + c]);
            std::sort(v.begin(), v.end());
            printf("  %s p50 %.0f p90 %.0f max %.0f |", names[c - 1], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
        }
        printf(" (10 ns ticks)\n");
    }
    return 0;
}
