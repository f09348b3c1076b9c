// Issue / dependency latency of the instruction classes the race sub-step chain is made of, at one
// wave per SIMD (the config-4 launch shape): cycles per instruction of a dependent chain and of four
// independent chains, by s_memtime.  Measurement-only (tools/, not part of the library).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// one v_mad_u64_u32 (x * 0xD2511F53 + 0, 64-bit result)
__device__ __forceinline__ uint64_t __builtin_amdgcn_mad_u64_u32_probe(uint32_t x) {
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "v"(0xD2511F53u) : "vcc");
    return r;
}

constexpr int kIters = 256;

#define CHAIN(NAME, T, INIT, STEP)                                                                   \
    __global__ void NAME##_dep(T* out, uint64_t* cyc, T seed) {                                      \
        T x = seed + T(threadIdx.x) * T(1e-7) + T(T(0.5) == T(0) ? threadIdx.x : 0);  /* integer T: lane-varying */                                                       \
        const T a = seed * T(0.999), b = seed * T(1e-3);                                             \
        (void)a; (void)b;                                                                            \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                            \
        _Pragma("unroll 16") for (int i = 0; i < kIters; ++i) { STEP(x); }                           \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                                      \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                             \
    }                                                                                                \
    __global__ void NAME##_ind(T* out, uint64_t* cyc, T seed) {                                      \
        T x = seed + T(threadIdx.x) * T(1e-7) + T(T(0.5) == T(0) ? threadIdx.x : 0), y = x + T(1e-3), z = x + T(2e-3), w = x + T(3e-3);    \
        const T a = seed * T(0.999), b = seed * T(1e-3);                                             \
        (void)a; (void)b;                                                                            \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                            \
        _Pragma("unroll 4") for (int i = 0; i < kIters / 4; ++i) { STEP(x); STEP(y); STEP(z); STEP(w); } \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x + y + z + w;                                          \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                             \
    }

#define FMA_STEP(x) x = __builtin_fma(x, a, b)
#define FMAF_STEP(x) x = __builtin_fmaf(x, a, b)
#define MUL_STEP(x) x = x * a
#define ADD_STEP(x) x = x + b
#define RCP64_STEP(x) x = __builtin_amdgcn_rcp(x)
#define RCP32_STEP(x) x = __builtin_amdgcn_rcpf(x)
#define RSQ64_STEP(x) x = __builtin_amdgcn_rsq(x)
#define DPP_STEP(x) x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x1b, 0xf, 0xf, false)) + b
#define DIV32_STEP(x) x = b / x
#define DIV64_STEP(x) x = b / x
#define CVT_STEP(x) x = double(float(x)) * a
// an SGPR constant materialised next to each FMA (the fp64 kernels' 64-bit literals)
#define SMOV_STEP(x) do { int lo_, hi_; asm volatile("s_mov_b32 %0, 0x3ff00001" : "=s"(lo_)); \
    asm volatile("s_mov_b32 %0, 0x3ff00000" : "=s"(hi_)); x = __builtin_fma(x, __hiloint2double(hi_, lo_), b); } while (0)

// Philox's 32 x 32 -> 64 products: v_mul_hi_u32 + v_mul_lo_u32, or one v_mad_u64_u32
#define MULHL_STEP(x) do { const uint32_t h_ = __umulhi(x, 0xD2511F53u), l_ = x * 0xD2511F53u; x = h_ ^ l_ ^ b; } while (0)
#define MAD64_STEP(x) do { const uint64_t p_ = __builtin_amdgcn_mad_u64_u32_probe(x); x = uint32_t(p_ >> 32) ^ uint32_t(p_) ^ b; } while (0)

CHAIN(fma64, double, 0, FMA_STEP)
CHAIN(fma32, float, 0, FMAF_STEP)
CHAIN(mul64, double, 0, MUL_STEP)
CHAIN(add64, double, 0, ADD_STEP)
CHAIN(rcp64, double, 0, RCP64_STEP)
CHAIN(rcp32, float, 0, RCP32_STEP)
CHAIN(rsq64, double, 0, RSQ64_STEP)
CHAIN(dpp32, float, 0, DPP_STEP)
CHAIN(div32, float, 0, DIV32_STEP)
CHAIN(div64, double, 0, DIV64_STEP)
CHAIN(cvt64, double, 0, CVT_STEP)
CHAIN(smov64, double, 0, SMOV_STEP)
CHAIN(mulhl32, uint32_t, 0, MULHL_STEP)
CHAIN(mad64u32, uint32_t, 0, MAD64_STEP)

template <typename T>
static void run(const char* name, void (*dep)(T*, uint64_t*, T), void (*ind)(T*, uint64_t*, T), T seed,
                int waves_per_block = 1) {
    const int blocks = 1024;
    T* out;
    uint64_t* cyc;
    hipMalloc(&out, blocks * 64 * waves_per_block * sizeof(T));
    hipMalloc(&cyc, blocks * sizeof(uint64_t));
    uint64_t h[blocks];
    double r[2];
    for (int m = 0; m < 2; ++m) {
        for (int rep = 0; rep < 3; ++rep)
            hipLaunchKernelGGL(m ? ind : dep, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc, seed);
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; ++i) s += double(h[i]);
        r[m] = s / blocks / kIters;
    }
    printf("{\"op\": \"%s\", \"waves_per_block\": %d, \"dep_cycles_per_op\": %.2f, \"indep4_cycles_per_op\": %.2f}\n",
           name, waves_per_block, r[0], r[1]);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<double>("v_fma_f64", fma64_dep, fma64_ind, 1.0001);
    run<float>("v_fma_f32", fma32_dep, fma32_ind, 1.0001f);
    run<double>("v_mul_f64", mul64_dep, mul64_ind, 1.0001);
    run<double>("v_add_f64", add64_dep, add64_ind, 1.0001);
    run<double>("v_rcp_f64", rcp64_dep, rcp64_ind, 1.0001);
    run<float>("v_rcp_f32", rcp32_dep, rcp32_ind, 1.0001f);
    run<double>("v_rsq_f64", rsq64_dep, rsq64_ind, 1.0001);
    run<float>("dpp_mov+add_f32", dpp32_dep, dpp32_ind, 1.0001f);
    run<float>("ieee_div_f32", div32_dep, div32_ind, 1.0001f);
    run<double>("ieee_div_f64", div64_dep, div64_ind, 1.0001);
    run<double>("cvt_f32_f64+mul", cvt64_dep, cvt64_ind, 1.0001);
    run<double>("2x s_mov_b32+v_fma_f64", smov64_dep, smov64_ind, 1.0001);
    run<uint32_t>("v_mul_hi_u32+v_mul_lo_u32+2xor", mulhl32_dep, mulhl32_ind, 12345u);
    run<uint32_t>("v_mad_u64_u32+2xor", mad64u32_dep, mad64u32_ind, 12345u);
    // several waves per SIMD: cycles per op of each wave (throughput per SIMD = waves / this)
    run<double>("v_fma_f64", fma64_dep, fma64_ind, 1.0001, 4);
    run<double>("v_fma_f64", fma64_dep, fma64_ind, 1.0001, 8);
    run<float>("v_fma_f32", fma32_dep, fma32_ind, 1.0001f, 4);
    run<float>("v_fma_f32", fma32_dep, fma32_ind, 1.0001f, 8);
    run<double>("2x s_mov_b32+v_fma_f64", smov64_dep, smov64_ind, 1.0001, 8);
    return 0;
}
