// Does the kernel-argument block size change the launch ramp?  Same probe as
// ramp.hip (block entry times via s_memrealtime), 256 x 1024 threads with
// ~141 KB LDS and a ~10 us body, with a 16-B, 256-B and 1 KiB argument block
// (the staged query kernel passes a 1 KiB column-pointer table).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/ramp_kernarg tools/probes/ramp_kernarg.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Rec { unsigned long long t; unsigned xcc, hw; };
template <int NP> struct Tab { const float* p[NP]; };

template <int NP>
__global__ void __launch_bounds__(1024) k_ramp(Rec* rec, int spin_ticks, Tab<NP> tab) {
    extern __shared__ float lds[];
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) rec[(size_t)blockIdx.x * (blockDim.x / 64) + w] = Rec{t, xcc, 0};
    // touch the table like the query kernel does (one wave-uniform pointer load)
    const float* p = tab.p[(blockIdx.x & 7) % NP];
    float v = p ? p[threadIdx.x & 63] : 0.f;
    while (__builtin_amdgcn_s_memrealtime() - t < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) lds[0] = v;
    __syncthreads();
    if (threadIdx.x == 1 && lds[0] < -1.f) rec[0].hw = 1;
}

template <int NP>
static void run(const char* name, float* buf, int spin) {
    const int blocks = 256, threads = 1024, wpb = 16, lds = 141 * 1024;
    hipFuncSetAttribute((const void*)k_ramp<NP>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    Rec* d;
    hipMalloc(&d, sizeof(Rec) * blocks * wpb);
    std::vector<Rec> h(blocks * wpb);
    Tab<NP> tab;
    for (int i = 0; i < NP; ++i) tab.p[i] = buf + 64 * i;
    double spread = 0, lag = 0;
    const int R = 12;
    for (int it = 0; it < R + 3; ++it) {
        for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(k_ramp<NP>, dim3(blocks), dim3(threads), lds, 0, d, spin, tab);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, sizeof(Rec) * h.size(), hipMemcpyDeviceToHost);
        if (it < 3) continue;
        unsigned long long t0 = ~0ull, t1 = 0, xmin[8];
        for (int x = 0; x < 8; ++x) xmin[x] = ~0ull;
        for (int b = 0; b < blocks; ++b) {
            unsigned long long bmin = ~0ull;
            for (int w = 0; w < wpb; ++w) bmin = std::min(bmin, h[b * wpb + w].t);
            xmin[h[b * wpb].xcc & 7] = std::min(xmin[h[b * wpb].xcc & 7], bmin);
            t0 = std::min(t0, bmin);
            t1 = std::max(t1, bmin);
        }
        spread += t1 - t0;
        unsigned long long lo = ~0ull, hi = 0;
        for (int x = 0; x < 8; ++x) { lo = std::min(lo, xmin[x]); hi = std::max(hi, xmin[x]); }
        lag += hi - lo;
        if (it == R + 2) {
            printf("  per-XCD first entry (ticks):");
            for (int x = 0; x < 8; ++x) printf(" %llu", xmin[x] - t0);
            printf("\n");
        }
    }
    printf("%-36s grid entry spread %6.1f ticks, XCD first-entry lag %6.1f\n", name, spread / R, lag / R);
    hipFree(d);
}

int main() {
    float* buf;
    hipMalloc(&buf, 1 << 20);
    hipMemset(buf, 0, 1 << 20);
    for (int spin : {1000}) {
        run<2>("args 16 B + 16 B table", buf, spin);
        run<32>("args 16 B + 256 B table", buf, spin);
        run<128>("args 16 B + 1 KiB table", buf, spin);
        run<2>("args 16 B + 16 B table (again)", buf, spin);
    }
    return 0;
}
