// Launch-ramp probe: when does each workgroup of a back-to-back launch start?
// Every wave's lane 0 stores {s_memrealtime at entry, XCC_ID, HW_ID}; the host
// reports, per launch shape, the spread of block entry times over the grid and
// per XCD, and the spread of wave entries inside a block.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/ramp tools/probes/ramp.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Rec { unsigned long long t; unsigned xcc, hw; };

__global__ void k_ramp(Rec* rec, int spin_ticks) {
    extern __shared__ float lds[];
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        Rec r{t, xcc, hw};
        rec[(size_t)blockIdx.x * (blockDim.x / 64) + w] = r;
    }
    if (spin_ticks > 0) {
        while (__builtin_amdgcn_s_memrealtime() - t < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
        if (threadIdx.x == 0) lds[0] = (float)t;  // keep LDS allocated/used
        __syncthreads();
        if (threadIdx.x == 1 && lds[0] < 0.f) rec[0].hw = 0;
    }
}

static void run(const char* name, int blocks, int threads, int lds, int spin) {
    const int wpb = threads / 64;
    Rec* d;
    hipMalloc(&d, sizeof(Rec) * blocks * wpb);
    std::vector<Rec> h(blocks * wpb);
    double spread_sum = 0, intra_sum = 0, xcdlag_sum = 0;
    const int R = 12;
    for (int it = 0; it < R + 3; ++it) {
        for (int k = 0; k < 8; ++k) hipLaunchKernelGGL(k_ramp, dim3(blocks), dim3(threads), lds, 0, d, spin);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, sizeof(Rec) * h.size(), hipMemcpyDeviceToHost);
        if (it < 3) continue;
        unsigned long long t0 = ~0ull, t1 = 0;
        double intra = 0;
        unsigned long long xmin[8], xmax[8];
        for (int x = 0; x < 8; ++x) xmin[x] = ~0ull, xmax[x] = 0;
        for (int b = 0; b < blocks; ++b) {
            unsigned long long bmin = ~0ull, bmax = 0;
            for (int w = 0; w < wpb; ++w) {
                bmin = std::min(bmin, h[b * wpb + w].t);
                bmax = std::max(bmax, h[b * wpb + w].t);
            }
            const unsigned x = h[b * wpb].xcc & 7;
            xmin[x] = std::min(xmin[x], bmin);
            xmax[x] = std::max(xmax[x], bmin);
            t0 = std::min(t0, bmin);
            t1 = std::max(t1, bmin);
            intra = std::max(intra, (double)(bmax - bmin));
        }
        spread_sum += t1 - t0;
        intra_sum += intra;
        unsigned long long lo = ~0ull, hi = 0;
        for (int x = 0; x < 8; ++x) if (xmax[x]) { lo = std::min(lo, xmin[x]); hi = std::max(hi, xmin[x]); }
        xcdlag_sum += hi - lo;
        if (it == R + 2) {
            printf("  last launch per XCD [first, last block entry] (10 ns ticks after grid start):");
            for (int x = 0; x < 8; ++x) if (xmax[x]) printf(" x%d[%llu,%llu]", x, xmin[x] - t0, xmax[x] - t0);
            printf("\n");
        }
    }
    printf("%-44s grid entry spread %6.1f ticks, XCD first-entry lag %6.1f, max intra-block wave spread %6.1f\n",
           name, spread_sum / R, xcdlag_sum / R, intra_sum / R);
    hipFree(d);
}

int main() {
    hipFuncSetAttribute((const void*)k_ramp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int spin : {0, 1000}) {
        printf("predecessor/self duration: %s\n", spin ? "~10 us spin" : "empty");
        run("256 x 1024 thr, no LDS", 256, 1024, 0, spin);
        run("256 x 1024 thr, 114 KB LDS", 256, 1024, 114 * 1024, spin);
        run("256 x 512 thr, 114 KB LDS", 256, 512, 114 * 1024, spin);
        run("256 x 256 thr, no LDS", 256, 256, 0, spin);
        run("512 x 512 thr, 60 KB LDS", 512, 512, 60 * 1024, spin);
        run("1024 x 256 thr, no LDS", 1024, 256, 0, spin);
        run("128 x 1024 thr, 114 KB LDS", 128, 1024, 114 * 1024, spin);
    }
    return 0;
}
