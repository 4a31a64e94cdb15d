// VALU issue-rate probe (round 4; extended round 5,
// VERDICT r04 item 3): cycles per wave64 instruction per SIMD for the
// parametric kernels' instruction kinds at 1..8 waves per SIMD, with 8 or 16
// independent chains per wave, with and without `s_setprio 3`, and in the
// 8-byte VOP3 (`v_fma_f32`) and 4-byte VOP2 (`v_fmac_f32`) encodings.
// Every wave records s_memtime (shader cycles) and s_memrealtime (100 MHz,
// chip-wide) around its loop.  The shader clock = cycles / real time of the
// median wave; the SIMD's cycles = (last wave end - first wave start) in real
// time x that clock (so waves that were not all co-resident are not
// mistaken for overlap); cost = SIMD cycles / (waves per SIMD x instructions
// per wave).  "overlap" = the longest wave's span / that window (1.0: every
// wave of the SIMD ran the whole window, i.e. co-resident).
// MI355X_MICROARCH.md's constants table gives 2 cycles per wave64 v_fma_f32
// ("SIMD-32") with several waves resident, 4 for one wave alone.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/valu_rate tools/probes/valu_rate.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

// OP: 0 v_fma_f32 (VOP3), 1 v_pk_fma_f32, 2 v_pk_mul_f32, 3 v_exp_f32,
// 4 v_rcp_f32, 5 NN-like mix, 6 v_fmac_f32 (VOP2), 7 v_add_f32 (VOP2),
// 8 v_mul_f32 (VOP2), 9 v_fma_f32 with three distinct source registers
template <int OP, int CH, bool PRIO>
__global__ void __launch_bounds__(1024) k(unsigned long long* cyc, float* sink, float c) {
    const float d = c * 0.75f + threadIdx.x * 1e-6f;
    float a[CH];
    f2 b[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        a[j] = threadIdx.x * 1e-3f + j;
        b[j] = f2{a[j], a[j] + 0.5f};
    }
    const f2 c2 = f2{c, c * 0.5f};
    if (PRIO) __builtin_amdgcn_s_setprio(3);
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters * 8 / CH; ++i) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(c2));
            if (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(b[j]) : "v"(c2));
            if (OP == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(a[j]));
            if (OP == 4) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[j]));
            if (OP == 5) {  // NN-kernel-like mix: 6 fma : 3 pk_fma : 1 exp per 10 (static mix of k_param_query NN)
                if (j % 8 < 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
                else if (j % 8 < 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(c2));
                else if (j % 8 < 7) asm volatile("v_exp_f32 %0, %0" : "+v"(a[j]));
                else asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            }
            if (OP == 6) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if (OP == 7) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if (OP == 8) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if (OP == 9) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c), "v"(d));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* o = cyc + 3 * ((blockIdx.x * blockDim.x + threadIdx.x) / 64);
        o[0] = t1 - t0;
        o[1] = r0;
        o[2] = r1;
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) s += a[j] + b[j].x + b[j].y;
    if (s == 12345.f) sink[threadIdx.x] = s;
}

template <int OP, int CH, bool PRIO>
void run(const char* name, int cus) {
    unsigned long long* dcyc;
    float* sink;
    const int maxb = cus * 8;
    hipMalloc(&dcyc, sizeof(unsigned long long) * maxb * 16 * 3);
    hipMalloc(&sink, 1024 * 4);
    printf("%-12s ch=%2d prio=%d", name, CH, PRIO ? 3 : 0);
    for (int w : {1, 2, 4, 8}) {
        // one block of 256 w threads per CU (w <= 4), two of 1024 for w = 8:
        // every wave of a CU is dispatched at once
        const int per = w <= 4 ? w : 4;
        const int blocks = cus * (w / per);
        const int threads = 256 * per;
        hipLaunchKernelGGL((k<OP, CH, PRIO>), dim3(blocks), dim3(threads), 0, 0, dcyc, sink, 0.999f);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP, CH, PRIO>), dim3(blocks), dim3(threads), 0, 0, dcyc, sink, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const int nw = blocks * threads / 64;
        std::vector<unsigned long long> h(3 * nw);
        hipMemcpy(h.data(), dcyc, sizeof(unsigned long long) * 3 * nw, hipMemcpyDeviceToHost);
        std::vector<double> clk(nw);
        unsigned long long rlo = ~0ull, rhi = 0, rspan = 0;
        for (int i = 0; i < nw; ++i) {
            const unsigned long long rs = h[3 * i + 2] - h[3 * i + 1];
            clk[i] = (double)h[3 * i] / (rs * 10.0);  // GHz
            rlo = std::min(rlo, h[3 * i + 1]);
            rhi = std::max(rhi, h[3 * i + 2]);
            rspan = std::max(rspan, rs);
        }
        std::nth_element(clk.begin(), clk.begin() + nw / 2, clk.end());
        const double ghz = clk[nw / 2];
        const double ins = (double)kIters * 8;  // per wave
        const double simd_cyc = (rhi - rlo) * 10.0 * ghz;
        printf(" | w=%d %.2f cyc @%.2fGHz ovl %.2f", w, simd_cyc / (w * ins), ghz, (double)rspan / (rhi - rlo));
        (void)ms;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
    printf("\n");
    hipFree(dcyc);
    hipFree(sink);
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    printf("CUs %d, clock %d kHz; cycles per wave64 instruction per SIMD\n", cus, prop.clockRate);
    run<0, 8, false>("v_fma_f32", cus);
    run<0, 16, false>("v_fma_f32", cus);
    run<0, 16, true>("v_fma_f32", cus);
    run<9, 16, false>("v_fma_3src", cus);
    run<6, 16, false>("v_fmac_f32", cus);
    run<7, 16, false>("v_add_f32", cus);
    run<8, 16, false>("v_mul_f32", cus);
    run<1, 8, false>("v_pk_fma", cus);
    run<1, 16, false>("v_pk_fma", cus);
    run<1, 16, true>("v_pk_fma", cus);
    run<2, 16, false>("v_pk_mul", cus);
    run<3, 8, false>("v_exp_f32", cus);
    run<3, 16, false>("v_exp_f32", cus);
    run<4, 16, false>("v_rcp_f32", cus);
    run<5, 8, false>("mix", cus);
    run<5, 16, false>("mix", cus);
    return 0;
}
