// Host cost of the sharded step's HIP calls on this box: kernel launches with
// small vs 3.3 KB kernel arguments (the fast kernel's per-(factor, parent)
// evidence pointer table), hipEventRecord, hipStreamWaitEvent.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { const float* p[416]; };

__global__ void k_small(float* o, int n) { if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) o[0] = 1.f; }
__global__ void k_big(Big b, float* o, int n) { if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) o[0] = b.p[5][0]; }

template <class F> double per_call(F f, int K = 20000) {
    for (int i = 0; i < 200; ++i) f();
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < K; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    hipDeviceSynchronize();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / K;
}

int main() {
    hipStream_t a, c;
    hipStreamCreate(&a);
    hipStreamCreate(&c);
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    float* o;
    hipMalloc(&o, 64);
    Big b{};
    for (auto& p : b.p) p = o;
    printf("launch 256x1024, 12 B args      : %.2f us\n", per_call([&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1); }));
    printf("launch 256x1024, 3.3 KB args    : %.2f us\n", per_call([&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 0, a, b, o, 1); }));
    printf("launch 256x1024, 3.3 KB + 96 KB LDS: %.2f us\n", per_call([&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 96 * 1024, a, b, o, 1); }));
    printf("hipEventRecord                  : %.2f us\n", per_call([&] { hipEventRecord(e, a); }));
    printf("hipStreamWaitEvent              : %.2f us\n", per_call([&] { hipStreamWaitEvent(c, e, 0); }));
    printf("record + wait + small launch on c: %.2f us\n", per_call([&] {
        hipEventRecord(e, a);
        hipStreamWaitEvent(c, e, 0);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c, o, 1);
    }));
    printf("launch a + launch c, no dependency: %.2f us\n", per_call([&] {
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c, o, 1);
    }));
    printf("launch a + record a + wait c + launch c: %.2f us\n", per_call([&] {
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1);
        hipEventRecord(e, a);
        hipStreamWaitEvent(c, e, 0);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c, o, 1);
    }));
    printf("launch a + launch a (same stream): %.2f us\n", per_call([&] {
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, a, o, 1);
    }));
    unsigned* flag;
    hipMalloc(&flag, 64);
    hipMemset(flag, 0, 64);
    unsigned v = 0;
    printf("launch a + writeValue a + waitValue c + launch c: %.2f us\n", per_call([&] {
        ++v;
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1);
        hipStreamWriteValue32(a, flag, v, 0);
        hipStreamWaitValue32(c, flag, v, hipStreamWaitValueGte, 0xFFFFFFFFu);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c, o, 1);
    }));
    hipEvent_t e2;
    hipEventCreateWithFlags(&e2, hipEventDisableTiming | hipEventReleaseToDevice);
    printf("launch a + record(ReleaseToDevice) a + wait c + launch c: %.2f us\n", per_call([&] {
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, a, o, 1);
        hipEventRecord(e2, a);
        hipStreamWaitEvent(c, e2, 0);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c, o, 1);
    }));
    printf("hipGetLastError                 : %.3f us\n", per_call([&] { (void)hipGetLastError(); }));
    return 0;
}
