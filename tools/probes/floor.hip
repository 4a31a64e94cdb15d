// Floor of a launch shaped like the fused query kernel (256 x 1024 threads,
// ~130 KB of dynamic LDS): back-to-back launches timed with events.
//   empty           : nothing
//   store 8 MB      : every lane stores two float4 (65 536 rows x 128 B)
//   load 5 MB       : every lane loads 5 floats of 19 x 256 KB columns (coalesced)
//   load + store    : both
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/floor tools/probes/floor.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(1024) k_empty(int* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0) *p = 1; }

__global__ void __launch_bounds__(1024) k_floor(const float* __restrict__ ev, float* __restrict__ out, int mode) {
    extern __shared__ float lds[];
    const int tid = threadIdx.x;
    const long long q = (long long)blockIdx.x * 256 + (tid >> 2);
    float a = 1.f;
    if (mode & 1) {
        // 20 columns of 65 536 floats; lane reads 5 of them (its 4-lane group covers 20)
        const int l = tid & 3;
#pragma unroll
        for (int j = 0; j < 5; ++j) a += ev[(long long)(l + 4 * j) * 65536 + q];
    }
    if (mode & 4) {
        lds[tid] = a;
        __syncthreads();
        a += lds[(tid + 64) & 1023];
    }
    if (mode & 2) {
        float4* o = reinterpret_cast<float4*>(out + q * 32) + (tid & 3) * 2;
        o[0] = make_float4(a, a, a, a);
        o[1] = make_float4(a, a, a, a);
    }
}

int main() {
    float *ev, *out;
    hipMalloc(&ev, 20LL * 65536 * 4);
    hipMalloc(&out, 65536LL * 32 * 4);
    hipMemset(ev, 0, 20LL * 65536 * 4);
    hipFuncSetAttribute((const void*)k_floor, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"empty", "load 5 MB", "store 8 MB", "load + store", "empty + barrier", "load + barrier",
                           "store + barrier", "load + barrier + store"};
    for (int lds : {0, 130 * 1024}) {
        for (int mode = 0; mode < 8; ++mode) {
            for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_floor, dim3(256), dim3(1024), lds, 0, ev, out, mode);
            hipEventRecord(e0, 0);
            const int K = 500;
            for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_floor, dim3(256), dim3(1024), lds, 0, ev, out, mode);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("LDS %6d B  %-24s %.2f us per launch\n", lds, names[mode], ms * 1000 / K);
        }
    }
    for (int lds : {0, 130 * 1024})
        for (int bt : {1024, 512, 256}) {
            for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(bt), lds, 0, nullptr);
            hipEventRecord(e0, 0);
            const int K = 500;
            for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(bt), lds, 0, nullptr);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("empty kernel 256 x %4d threads, LDS %6d B: %.2f us per launch\n", bt, lds, ms * 1000 / K);
        }
    return 0;
}
