// math_probe.hip — adrp_math_probe: evaluates the fp64 fast transcendentals of adrp_device.h
// (namespace f64, the exp-map forms, the race noise Box-Muller) over a device array, so
// tests/test_math_gpu.py can check them against extended-precision references and the oracle (the
// step kernels inline the same functions).
#include <hip/hip_runtime.h>

#include "adrp_device.h"
#include "../../include/adrp.h"

namespace {
__global__ void __launch_bounds__(256) math_probe_kernel(int fn, const double* __restrict__ in, double* __restrict__ out,
                                                         int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = in[i];
    double r = 0.0, c = 0.0;
    switch (fn) {
        case ADRP_MATH_RCP: r = adrp::f64::rcp(x); break;
        case ADRP_MATH_RSQ: r = adrp::f64::rsq(x); break;
        case ADRP_MATH_SQRT: r = adrp::f64::sqrt(x); break;
        case ADRP_MATH_SIN_SMALL: adrp::f64::sincos_small(x, &r, &c); break;
        case ADRP_MATH_COS_SMALL: adrp::f64::sincos_small(x, &c, &r); break;
        case ADRP_MATH_ATAN2: r = adrp::f64::atan2(x, in[n + i]); break;
        case ADRP_MATH_ASIN: r = adrp::f64::asin(x); break;
        case ADRP_MATH_EXP: r = adrp::f64::exp(x); break;
        case ADRP_MATH_SQRT_NN: r = adrp::f64::sqrt_nn(x); break;
        case ADRP_MATH_RCP_NC: r = adrp::f64::rcp_nc(x); break;
        case ADRP_MATH_RSQ_NC: r = adrp::f64::rsq_nc(x); break;
        case ADRP_MATH_SIN_TINY: adrp::f64::sincos_tiny(x, &r, &c); break;
        case ADRP_MATH_COS_TINY: adrp::f64::sincos_tiny(x, &c, &r); break;
        case ADRP_MATH_EXPMAP_SINC: adrp::expmap_sinc_cos(x, &r, &c); break;
        case ADRP_MATH_EXPMAP_COS: adrp::expmap_sinc_cos(x, &c, &r); break;
        case ADRP_MATH_QUAT_INV_NORM: r = adrp::quat_inv_norm(x); break;
        case ADRP_MATH_DIVC: r = adrp::f64::div_c(x, in[n + i]); break;
        case ADRP_MATH_SIN_FAST: adrp::f64::sincos_fast(x, &r, &c); break;
        case ADRP_MATH_COS_FAST: adrp::f64::sincos_fast(x, &c, &r); break;
        case ADRP_MATH_EXP_TAB: r = adrp::f64::exp_tab(x, adrp::f64::kExp2Tab32); break;
        case ADRP_MATH_ATAN2_NC: r = adrp::f64::atan2_nc(x, in[n + i]); break;
        case ADRP_MATH_FDIV_RCP: r = adrp::f64::fdiv_rcp(float(x), adrp::f64::rcp(double(float(in[n + i])))); break;
        case ADRP_MATH_NORMAL_Z0:
        case ADRP_MATH_NORMAL_Z1: {
            const unsigned long long b = (unsigned long long)__double_as_longlong(x);
            float z0, z1;
            adrp::normal_pair_f(uint32_t(b), uint32_t(b >> 32), &z0, &z1);
            r = fn == ADRP_MATH_NORMAL_Z0 ? z0 : z1;
            break;
        }
        default: r = __builtin_nan(""); break;
    }
    out[i] = r;
}
}  // namespace

extern "C" int adrp_math_probe(int fn, const double* in_dev, double* out_dev, int n, void* stream) {
    if (fn < ADRP_MATH_RCP || fn > ADRP_MATH_FDIV_RCP || n < 0 || (n > 0 && (!in_dev || !out_dev))) return ADRP_ERR_INVALID;
    if (n == 0) return ADRP_OK;
    hipLaunchKernelGGL(math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, in_dev, out_dev, n);
    return hipGetLastError() == hipSuccess ? ADRP_OK : ADRP_ERR_DEVICE;
}
