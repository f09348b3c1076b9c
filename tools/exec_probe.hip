// exec_probe.hip — does a wave64 VALU op cost less with fewer active lanes, and how much
// does ILP buy at one wave per SIMD?  (design probe for the latency-bound step kernels)
//
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/exec_probe tools/exec_probe.hip
// Each variant runs the same per-lane dependent FMA work; we time K iterations per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ void __launch_bounds__(256) chain(float* out, int iters, int active) {
    const int l = threadIdx.x & 63;
    if (l >= active) return;
    float x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = out[blockIdx.x * 64 + l] + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = __builtin_fmaf(x[c], 0.999f, 0.001f);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * 64 + l] = s;
}

template <int CH>
float run(float* d, int blocks, int threads, int iters, int active) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    chain<CH><<<blocks, threads>>>(d, iters, active);
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) chain<CH><<<blocks, threads>>>(d, iters, active);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 100.0f;  // us per launch
}

int main() {
    float* d;
    hipMalloc(&d, 1 << 24);
    hipMemset(d, 0, 1 << 24);
    const int iters = 20000;
    printf("iters %d; us per launch; FMA ops per lane = iters*CH\n", iters);
    for (int act : {64, 32, 16, 4, 1}) {
        printf("1 wave/WG, 64 WGs, %2d active lanes: CH1 %8.2f  CH2 %8.2f  CH4 %8.2f  CH8 %8.2f\n", act,
               run<1>(d, 64, 64, iters, act), run<2>(d, 64, 64, iters, act), run<4>(d, 64, 64, iters, act),
               run<8>(d, 64, 64, iters, act));
    }
    // 4 waves per WG (one per SIMD) vs 1
    printf("4 waves/WG, 64 WGs, 64 active: CH1 %8.2f  CH4 %8.2f\n", run<1>(d, 64, 256, iters, 64),
           run<4>(d, 64, 256, iters, 64));
    printf("1 wave/WG, 256 WGs, 64 active: CH1 %8.2f  CH4 %8.2f\n", run<1>(d, 256, 64, iters, 64),
           run<4>(d, 256, 64, iters, 64));
    printf("1 wave/WG, 1024 WGs, 64 active: CH1 %8.2f  CH4 %8.2f\n", run<1>(d, 1024, 64, iters, 64),
           run<4>(d, 1024, 64, iters, 64));
    hipFree(d);
    return 0;
}
