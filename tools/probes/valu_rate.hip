// VALU issue-rate probe (round 4): cycles per wave64
// instruction per SIMD for the parametric kernels' instruction kinds --
// v_fma_f32, v_pk_fma_f32, v_pk_mul_f32, v_exp_f32, v_rcp_f32 and the NN
// kernel's mix -- at 1..8 waves per SIMD.  Each wave runs 8 independent
// chains (latency hidden within the wave); s_memtime (shader clock) brackets
// the loop.  cost = cycles / (waves per SIMD x instructions per wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/valu_rate tools/probes/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

template <int OP>
__global__ void __launch_bounds__(1024) k(unsigned long long* cyc, float* sink, float c) {
    float a[8];
    f2 b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = threadIdx.x * 1e-3f + j;
        b[j] = f2{a[j], a[j] + 0.5f};
    }
    const f2 c2 = f2{c, c * 0.5f};
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(c2));
            if (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(b[j]) : "v"(c2));
            if (OP == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(a[j]));
            if (OP == 4) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[j]));
            if (OP == 5) {  // NN-kernel-like mix: 6 fma : 3 pk_fma : 1 exp per 10 (static mix of k_param_query NN)
                if (j < 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
                else if (j < 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(c2));
                else if (j < 7) asm volatile("v_exp_f32 %0, %0" : "+v"(a[j]));
                else asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + b[j].x + b[j].y;
    if (s == 12345.f) sink[threadIdx.x] = s;
}

template <int OP>
void run(const char* name, int cus) {
    unsigned long long* dcyc;
    float* sink;
    const int maxb = cus * 8;
    hipMalloc(&dcyc, sizeof(unsigned long long) * maxb * 4);
    hipMalloc(&sink, 1024 * 4);
    printf("%-10s", name);
    for (int w : {1, 2, 4, 8}) {
        // one block of 256 w threads per CU (w <= 4), two of 1024 for w = 8:
        // every wave of a CU is dispatched at once
        const int per = w <= 4 ? w : 4;
        const int blocks = cus * (w / per);
        const int threads = 256 * per;
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, dcyc, sink, 0.999f);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, dcyc, sink, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const int nw = blocks * threads / 64;
        std::vector<unsigned long long> h(nw);
        hipMemcpy(h.data(), dcyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
        double avg = 0, mx = 0;
        for (auto v : h) { avg += (double)v; mx = std::max(mx, (double)v); }
        avg /= h.size();
        const double ins = (double)kIters * 8;
        // per SIMD: w co-resident waves each issuing `ins` instructions over ~avg cycles;
        // clock = the longest wave's cycles / the kernel's time (co-residency check)
        printf("  w=%d %.2f cyc/instr (wave avg %.0f max %.0f cyc, kernel %.1f us, %.2f GHz)", w, avg / (w * ins), avg,
               mx, ms * 1e3, mx / (ms * 1e6));
    }
    printf("\n");
    hipFree(dcyc);
    hipFree(sink);
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    printf("CUs %d, clock %d kHz\n", cus, prop.clockRate);
    run<0>("v_fma_f32", cus);
    run<1>("v_pk_fma", cus);
    run<2>("v_pk_mul", cus);
    run<3>("v_exp_f32", cus);
    run<4>("v_rcp_f32", cus);
    run<5>("mix", cus);
    return 0;
}
