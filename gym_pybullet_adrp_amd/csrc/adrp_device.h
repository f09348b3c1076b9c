// adrp_device.h — device-side math for the fused quadrotor step (gfx950).
//
// Everything here is __device__ inline, templated on the arithmetic type Real
// (float for the production kernel, double for the fp64 variant).  One lane owns one
// drone-env; all state lives in VGPRs across the fused sub-step loop.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace adrp {

// obs copy-out store (a row block written once per step, read by the next launch or the host);
// ADRP_NT_STORES: non-temporal (A/B: no change at hover E = 4096 or race config 4, so off)
__device__ __forceinline__ void store_out(float4* p, float4 v) {
#ifdef ADRP_NT_STORES
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
#else
    *p = v;
#endif
}

// phase timing (build with -DADRP_RACE_TIMING; tools/race_phases.py, tools/hover_phases.py):
// lane 0 of every wave adds its s_memtime deltas per phase of the step kernel
#ifdef ADRP_RACE_TIMING
__device__ unsigned long long g_race_phase[32];   // [0..8] sums, [10..17] per-phase max, 9/18/19 GJK
#define RACE_MARK(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define RACE_SET(var) var = __builtin_amdgcn_s_memtime()
#define RACE_ACC(i, dt) do { atomicAdd(&g_race_phase[i], (unsigned long long)(dt)); \
        atomicMax(&g_race_phase[10 + (i)], (unsigned long long)(dt)); } while (0)
// race kernels: one slot of 8 phases per workgroup, plain stores (the same-address atomics of
// RACE_ACC from 1024 waves serialise in L2 and stretch the phases they are meant to measure)
constexpr int kWaveSlots = 16384;
__device__ unsigned long long g_race_wave[kWaveSlots * 8];
#define RACE_WAVE(i, dt) do { if (blockIdx.x < kWaveSlots) g_race_wave[blockIdx.x * 8 + (i)] = (unsigned long long)(dt); } while (0)
#ifdef ADRP_RACE_GJK_STATS
// GJK queries that ran at least ADRP_GJK_DUMP_MIN_IT iterations (default: the cap): the first
// kGjkDumps of them (two shapes, the cut, the last |v|^2, the iterations, the decision and the seed),
// for a CPU replay (tools/gjk_replay.py, tools/gjk_slow.py)
#ifndef ADRP_GJK_DUMP_MIN_IT
#define ADRP_GJK_DUMP_MIN_IT 48
#endif
constexpr int kGjkDumps = 512, kGjkDumpF = 44;
__device__ double g_gjk_dump[kGjkDumps * kGjkDumpF];
__device__ unsigned int g_gjk_dump_n;
#endif
#else
#define RACE_MARK(var)
#define RACE_SET(var)
#define RACE_ACC(i, dt)
#define RACE_WAVE(i, dt)
#endif


// XCD-aware workgroup order.  The command processor deals consecutive workgroups round-robin over the
// 8 XCDs, each with its own L2; this bijection gives XCD x the contiguous range of logical blocks
// [x q + min(x, r), ...) (q, r = n / 8, n % 8), so neighbouring blocks that share cache lines (the race
// quad kernel: 16 drones x 4 B = half a 128-B line per field per block) share one L2 instead of each
// fetching the line into its own.
__device__ __forceinline__ int xcd_block(int b, int n) {
    constexpr int X = 8;
    const int x = b % X, i = b / X, q = n / X, r = n % X;
    return x * q + (x < r ? x : r) + i;
}

template <typename Real>
struct V3 {
    Real x, y, z;
};
template <typename Real>
struct Q4 {  // x, y, z, w (pybullet order); body-to-world
    Real x, y, z, w;
};
template <typename Real>
struct M3 {  // row-major rotation body->world
    Real a00, a01, a02, a10, a11, a12, a20, a21, a22;
};

template <typename Real>
__device__ __forceinline__ V3<Real> v3(Real x, Real y, Real z) {
    return V3<Real>{x, y, z};
}
template <typename Real>
__device__ __forceinline__ V3<Real> operator+(V3<Real> a, V3<Real> b) {
    return {a.x + b.x, a.y + b.y, a.z + b.z};
}
template <typename Real>
__device__ __forceinline__ V3<Real> operator-(V3<Real> a, V3<Real> b) {
    return {a.x - b.x, a.y - b.y, a.z - b.z};
}
template <typename Real>
__device__ __forceinline__ V3<Real> operator*(Real s, V3<Real> a) {
    return {s * a.x, s * a.y, s * a.z};
}
template <typename Real>
__device__ __forceinline__ Real dot(V3<Real> a, V3<Real> b) {
    return a.x * b.x + a.y * b.y + a.z * b.z;
}
template <typename Real>
__device__ __forceinline__ V3<Real> cross(V3<Real> a, V3<Real> b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// ---- fp64 fast transcendentals -------------------------------------------------------------
// The fp64 kernels compute at the reference's precision (float64), but CDNA has no correctly
// rounded fp64 division / sqrt / sin instruction: IEEE 1/x is a ~10-instruction scale / fixup
// sequence, libm sqrt / sincos / atan2 / exp add range checks and branches, and the fp64 step is
// one wave's dependent chain at E = 4096.  These are the hardware approximations (v_rcp_f64,
// v_rsq_f64) refined by Newton-Raphson to <= 2 ulp, and polynomials on the reduced ranges the
// kernels use (coefficients and their error: tools/fit_f64_poly.py; device check against
// longdouble references: tests/test_math_gpu.py through adrp_math_probe).
namespace f64 {
__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
// 1/x: v_rcp_f64 + 2 Newton steps (quadratic convergence); 0 / inf / NaN keep the hardware result
__device__ __forceinline__ double rcp(double x) {
    const double y0 = __builtin_amdgcn_rcp(x);
    double e = fma_(-x, y0, 1.0);
    double y = fma_(y0, e, y0);
    e = fma_(-x, y, 1.0);
    y = fma_(y, e, y);
    return __builtin_isfinite(y) ? y : y0;
}
// 1/sqrt(x): v_rsq_f64 + 2 Newton steps
__device__ __forceinline__ double rsq(double x) {
    const double y0 = __builtin_amdgcn_rsq(x);
    double y = y0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double e = fma_(-x * y, y, 1.0);
        y = fma_(0.5 * y, e, y);
    }
    return __builtin_isfinite(y) ? y : y0;
}
// rcp / rsq without the non-finite fix-up (3 ops each), for arguments known finite and non-zero on
// the lanes that use the result (the quaternion norm ~1; 1/|w| under an |w| >= 0.001 select)
__device__ __forceinline__ double rcp_nc(double x) {
    const double y0 = __builtin_amdgcn_rcp(x);
    double e = fma_(-x, y0, 1.0);
    double y = fma_(y0, e, y0);
    e = fma_(-x, y, 1.0);
    return fma_(y, e, y);
}
__device__ __forceinline__ double rsq_nc(double x) {
    double y = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double e = fma_(-x * y, y, 1.0);
        y = fma_(0.5 * y, e, y);
    }
    return y;
}
// sqrt(x), x >= 0: Goldschmidt on v_rsq_f64 (g -> sqrt x, h -> 1/(2 sqrt x)) + a final residual step
__device__ __forceinline__ double sqrt(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double r = fma_(-g, h, 0.5);
        g = fma_(g, r, g);
        h = fma_(h, r, h);
    }
    const double d = fma_(-g, g, x);
    g = fma_(d, h, g);
    // +0 / -0 / +inf return x (rsq(inf) = 0 would give inf * 0 = NaN), x < 0 and NaN give NaN
    return x > 0.0 && x < __builtin_inf() ? g : (x == 0.0 || x == __builtin_inf() ? x : __builtin_nan(""));
}
// sqrt of a sum of squares (x >= 0 or NaN): the same iteration on rsq(max(x, 1e-300)), so x = 0
// gives 0 (0 * 1e150) without the zero / negative selects of sqrt (6 fewer ops on the chain); NaN
// stays NaN through x * y.  Differs from sqrt only below x = 1e-300.
__device__ __forceinline__ double sqrt_nn(double x) {
    const double y = __builtin_amdgcn_rsq(__builtin_fmax(x, 1e-300));
    double g = x * y, h = 0.5 * y;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double r = fma_(-g, h, 0.5);
        g = fma_(g, r, g);
        h = fma_(h, r, h);
    }
    const double d = fma_(-g, g, x);
    return fma_(d, h, g);
}
// x / c for a constant c > 0, equal to the IEEE (correctly rounded) quotient for normal x and quotient:
// y = RN(1 / c) folds at compile time, q = RN(x y) is within 1 ulp of x / c, r = x - q c is exact
// (one FMA), and RN(q + r y) = RN(x / c) (Markstein's correction theorem; checked on 1.4e9 random x
// for each divisor the kernels use, and on the device by tests/test_math_gpu.py).  3 ops instead of the
// ~12-op v_div_scale / v_div_fmas / v_div_fixup sequence; a zero quotient takes x's sign.
__device__ __forceinline__ double div_c(double x, double c) {
    const double y = 1.0 / c;
    const double q = x * y;
    const double r = fma_(-q, c, x);
    return __builtin_copysign(fma_(r, y, q), x);
}
// sin / cos for |x| <= pi/8: Taylor to x^13 / x^14 (relative error <= 1.7e-16 before rounding)
__device__ __forceinline__ void sincos_small(double x, double* s, double* c) {
    const double x2 = x * x;
    double ps = 1.6059043836821613e-10;
    ps = fma_(ps, x2, -2.505210838544172e-08);
    ps = fma_(ps, x2, 2.7557319223985893e-06);
    ps = fma_(ps, x2, -0.0001984126984126984);
    ps = fma_(ps, x2, 0.008333333333333333);
    ps = fma_(ps, x2, -0.16666666666666666);
    double pc = -1.1470745597729725e-11;
    pc = fma_(pc, x2, 2.08767569878681e-09);
    pc = fma_(pc, x2, -2.755731922398589e-07);
    pc = fma_(pc, x2, 2.48015873015873e-05);
    pc = fma_(pc, x2, -0.001388888888888889);
    pc = fma_(pc, x2, 0.041666666666666664);
    pc = fma_(pc, x2, -0.5);
    *s = fma_(x * x2, ps, x);
    *c = fma_(x2, pc, 1.0);
}
// sin / cos for |x| < 2^20 (gate / part yaws, reset attitudes): octant n = rint(4 x / pi), r = x - n pi/4
// (two-part pi/4 through FMAs, |r| <= pi/8), sincos_small(r), then the octant's rotation without a
// branch: odd n starts from (sin, cos)(pi/4 + r) = sqrt(1/2) (c + s, c - s), bit 1 maps (s, c) ->
// (c, -s), bit 2 negates both.  Within 2 ulp of the correctly rounded values (tests/test_math_gpu.py);
// ~40 instructions where the libm sincos pays a range-reduction branch and ~3x the work.
__device__ __forceinline__ void sincos_fast(double x, double* s, double* c) {
    const double n = __builtin_rint(x * 1.2732395447351628);
    double r = fma_(-n, 0.78539816339744828, x);
    r = fma_(-n, 3.0616169978683830e-17, r);
    double sx, cx;
    sincos_small(r, &sx, &cx);
    const double h = 0.70710678118654752440;
    const double a = h * (cx + sx), b = h * (cx - sx);
    const uint32_t o = uint32_t(int(n)) & 7u;
    const bool odd = (o & 1u) != 0;
    const double s0 = odd ? a : sx, c0 = odd ? b : cx;
    const bool turn = (o & 2u) != 0;
    const double s1 = turn ? c0 : s0, c1 = turn ? -s0 : c0;
    const bool neg = (o & 4u) != 0;
    *s = neg ? -s1 : s1;
    *c = neg ? -c1 : c1;
}
// sin / cos for |x| <= 0.03 (the exp-map half angle |w| dt / 2 below 14 rad/s at 240 Hz): Taylor to
// x^7 / x^8; the first omitted terms are x^8/9! = 1.8e-18 and x^10/10! = 1.6e-22 relative
__device__ __forceinline__ void sincos_tiny(double x, double* s, double* c) {
    const double x2 = x * x;
    double ps = -0.0001984126984126984;
    ps = fma_(ps, x2, 0.008333333333333333);
    ps = fma_(ps, x2, -0.16666666666666666);
    double pc = 2.48015873015873e-05;
    pc = fma_(pc, x2, -0.001388888888888889);
    pc = fma_(pc, x2, 0.041666666666666664);
    pc = fma_(pc, x2, -0.5);
    *s = fma_(x * x2, ps, x);
    *c = fma_(x2, pc, 1.0);
}
// atan2(y, x): octant reduction to a = min/max in [0, 1], then t = a or (a - 1)/(a + 1) (one
// division either way: (min - max)/(min + max)) so |t| <= tan(pi/8), atan t = t + t^3 P(t^2)
// with a degree-9 near-minimax P (1.7e-16 relative).  atan2(0, 0) = 0 (as the fp32 fatan2_).
// NC: finite arguments only (the race controller's Euler angles): no non-finite fix-ups
template <bool NC>
__device__ __forceinline__ double atan2_t(double y, double x) {
    const double ax = __builtin_fabs(x), ay = __builtin_fabs(y);
    const double mx = __builtin_fmax(ax, ay), mn = __builtin_fmin(ax, ay);
    const bool big = mn > 0.41421356237309504880 * mx;
    const double num = big ? mn - mx : mn, den = big ? mn + mx : mx;
    const double t = mx > 0.0 ? num * (NC ? rcp_nc(den) : rcp(den)) : 0.0;
    const double s = t * t;
    double p = 0.021428368220326288;
    p = fma_(p, s, -0.04375458729368037);
    p = fma_(p, s, 0.05699267039194693);
    p = fma_(p, s, -0.06642647883966969);
    p = fma_(p, s, 0.07690277001250925);
    p = fma_(p, s, -0.09090800003785938);
    p = fma_(p, s, 0.11111107550967636);
    p = fma_(p, s, -0.14285714221246087);
    p = fma_(p, s, 0.19999999999459742);
    p = fma_(p, s, -0.3333333333333199);
    double r = fma_(t * s, p, t);
    if (big) r += 0.78539816339744830962;
    if (ay > ax) r = 1.57079632679489661923 - r;
    if (x < 0.0) r = 3.14159265358979323846 - r;
    // NaN in -> NaN out as libm (fmax / fmin above drop a NaN operand)
    if constexpr (NC) return __builtin_copysign(r, y);
    return __builtin_isunordered(x, y) ? x + y : __builtin_copysign(r, y);
}
// Correctly rounded float x / y from a float64 reciprocal of y: f64::rcp is within 2 ulp, so
// x * rcp(y) is the quotient to 1.25 * 2^-51 relative, while an exact quotient of two floats keeps at
// least 2^-49 relative from every float rounding boundary (significands X, Y < 2^24: |X 2^n -
// (2k + 1) Y| is a nonzero integer), so rounding that double to float IS the IEEE float x / y.  A
// divisor shared by several quotients pays one reciprocal (the race firmware's normalisations).
__device__ __forceinline__ float fdiv_rcp(float x, double ry) { return float(double(x) * ry); }
__device__ __forceinline__ double atan2(double y, double x) { return atan2_t<false>(y, x); }
__device__ __forceinline__ double atan2_nc(double y, double x) { return atan2_t<true>(y, x); }
// 2^(j/32), j = 0..31 (correctly rounded), the table of f64::exp_tab (the race kernel copies it to LDS)
static __device__ __constant__ double kExp2Tab32[32] = {
    1.0, 1.0218971486541166, 1.0442737824274138, 1.0671404006768237, 1.0905077326652577, 1.1143867425958924,
    1.1387886347566916, 1.1637248587775775, 1.189207115002721, 1.215247359980469, 1.241857812073484,
    1.2690509571917332, 1.2968395546510096, 1.3252366431597413, 1.3542555469368927, 1.383909881963832,
    1.4142135623730951, 1.4451808069770467, 1.4768261459394993, 1.5091644275934228, 1.5422108254079407,
    1.5759808451078865, 1.6104903319492543, 1.645755478153965, 1.681792830507429, 1.718619298122478,
    1.7562521603732995, 1.7947090750031072, 1.8340080864093424, 1.8741676341103, 1.9152065613971474,
    1.9571441241754002};
// exp(x), x <= 0 (the race downwash): k = 32 m + j = rint(32 x / ln 2), 2^(j/32) from a table the
// caller holds in LDS (kExp2Tab32), r = x - k ln2/32 (two-part, |r| <= ln2/64), exp r by Taylor to r^6
// (truncation 3.4e-18 relative), 2^m by v_ldexp_f64: 7 FMAs and 7 two-word constants where exp() pays
// 14 FMAs and 14 constants on the chain (tests/test_math_gpu.py, ADRP_MATH_EXP_TAB)
__device__ __forceinline__ double exp_tab(double x, const double* tab) {
    x = __builtin_fmax(x, -1000.0);
    const double k = __builtin_rint(x * 46.16624130844683);
    double r = fma_(-k, 0.021660849390173098, x);   // ln2/32, 33 significant bits: k * hi is exact
    r = fma_(-k, 2.325192846878874e-12, r);
    const int ki = int(k);
    const double t = tab[ki & 31];
    double p = 1.0 / 720;
    p = fma_(p, r, 1.0 / 120);
    p = fma_(p, r, 1.0 / 24);
    p = fma_(p, r, 1.0 / 6);
    p = fma_(p, r, 0.5);
    p = fma_(p, r, 1.0);
    p = fma_(p, r, 1.0);
    return __builtin_amdgcn_ldexp(t * p, ki >> 5);
}
// asin(s), |s| < 1: atan2(s, sqrt((1 - s)(1 + s)))
__device__ __forceinline__ double asin(double s) { return atan2(s, sqrt((1.0 - s) * (1.0 + s))); }
// exp(x): k = rint(x log2 e), r = x - k ln2 (two-part ln2), Taylor to r^13 on |r| <= ln2/2, 2^k by
// v_ldexp_f64 (underflows to 0 below -745; the kernels call it with x <= 0)
__device__ __forceinline__ double exp(double x) {
    x = __builtin_fmax(x, -1000.0);
    const double k = __builtin_rint(x * 1.4426950408889634);
    const double r = fma_(-k, 1.9082149292705877e-10, fma_(-k, 0.6931471803691238, x));
    double p = 1.6059043836821613e-10;
    p = fma_(p, r, 2.08767569878681e-09);
    p = fma_(p, r, 2.505210838544172e-08);
    p = fma_(p, r, 2.755731922398589e-07);
    p = fma_(p, r, 2.7557319223985893e-06);
    p = fma_(p, r, 2.48015873015873e-05);
    p = fma_(p, r, 0.0001984126984126984);
    p = fma_(p, r, 0.001388888888888889);
    p = fma_(p, r, 0.008333333333333333);
    p = fma_(p, r, 0.041666666666666664);
    p = fma_(p, r, 0.16666666666666666);
    p = fma_(p, r, 0.5);
    p = fma_(p, r, 1.0);
    p = fma_(p, r, 1.0);
    return __builtin_amdgcn_ldexp(p, int(k));
}
}  // namespace f64

__device__ __forceinline__ float rsqrt_(float x) { return __frsqrt_rn(x); }
__device__ __forceinline__ double rsqrt_(double x) { return 1.0 / ::sqrt(x); }
__device__ __forceinline__ float sqrt_(float x) { return __fsqrt_rn(x); }
__device__ __forceinline__ double sqrt_(double x) { return ::sqrt(x); }
__device__ __forceinline__ void sincos_(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void sincos_(double x, double* s, double* c) { ::sincos(x, s, c); }
// sincos_ for the kernels' angles (|x| < 2^20): fp64 the octant-reduced polynomial, fp32 libm
__device__ __forceinline__ void sincos_f_(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void sincos_f_(double x, double* s, double* c) { f64::sincos_fast(x, s, c); }
__device__ __forceinline__ float atan2_(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double atan2_(double y, double x) { return ::atan2(y, x); }
__device__ __forceinline__ float asin_(float x) { return asinf(x); }
__device__ __forceinline__ double asin_(double x) { return ::asin(x); }
__device__ __forceinline__ float exp_(float x) { return expf(x); }
__device__ __forceinline__ double exp_(double x) { return ::exp(x); }
__device__ __forceinline__ float fabs_(float x) { return fabsf(x); }
__device__ __forceinline__ double fabs_(double x) { return fabs(x); }

// latency-oriented primitives of the step loops: 1-ulp hardware ops in fp32, the refined
// hardware approximations above in fp64 (sqrt_ / rsqrt_ / atan2_ / asin_ / exp_ / sincos_ keep
// the correctly rounded / libm forms for code outside the loops)
// x / c for a constant c: fp64 the correctly rounded f64::div_c, fp32 the IEEE division
__device__ __forceinline__ double divc_(double x, double c) { return f64::div_c(x, c); }
__device__ __forceinline__ float divc_(float x, float c) { return x / c; }
__device__ __forceinline__ float rcp_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp_(double x) { return f64::rcp(x); }
__device__ __forceinline__ float hsqrt_(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double hsqrt_(double x) { return f64::sqrt(x); }
// rcp_ / hrsqrt_ of arguments known finite and non-zero where the result is used
__device__ __forceinline__ float rcp_nc_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp_nc_(double x) { return f64::rcp_nc(x); }
__device__ __forceinline__ float hrsqrt_nc_(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double hrsqrt_nc_(double x) { return f64::rsq_nc(x); }
// hsqrt_ of a sum of squares (argument >= 0 or NaN)
__device__ __forceinline__ float hsqrt_nn_(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double hsqrt_nn_(double x) { return f64::sqrt_nn(x); }
__device__ __forceinline__ float hrsqrt_(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double hrsqrt_(double x) { return f64::rsq(x); }

// sin/cos for |x| <= pi/8 (the exp-map half angle is clamped there): Taylor to x^7 / x^8,
// truncation error < 2e-9 relative, i.e. exact in fp32; fp64 to x^13 / x^14 (f64::sincos_small).
__device__ __forceinline__ void small_sincos(float x, float* s, float* c) {
    const float x2 = x * x;
    *s = x * (1.0f + x2 * (-1.0f / 6.0f + x2 * (1.0f / 120.0f + x2 * (-1.0f / 5040.0f))));
    *c = 1.0f + x2 * (-0.5f + x2 * (1.0f / 24.0f + x2 * (-1.0f / 720.0f + x2 * (1.0f / 40320.0f))));
}
__device__ __forceinline__ void small_sincos(double x, double* s, double* c) { f64::sincos_small(x, s, c); }
// the exp map's sin(x) / x and cos(x) (x = |w| dt / 2): the series above with the leading x of the
// sine factored out, so the axis factor sin(x) / |w| = (dt / 2) sinc(x) needs no reciprocal and no
// small-angle select (Bullet's |w| < 0.001 form 0.5 dt - dt^3 |w|^2 / 48 is this series' first two
// terms, equal to rounding there)
__device__ __forceinline__ void expmap_sinc_cos(float x, float* sinc, float* c) {
    const float x2 = x * x;
    *sinc = 1.0f + x2 * (-1.0f / 6.0f + x2 * (1.0f / 120.0f + x2 * (-1.0f / 5040.0f)));
    *c = 1.0f + x2 * (-0.5f + x2 * (1.0f / 24.0f + x2 * (-1.0f / 720.0f + x2 * (1.0f / 40320.0f))));
}
__device__ __forceinline__ void expmap_sinc_cos(double x, double* sinc, double* c) {
    // per lane: the short series where |x| <= 0.03, the full one elsewhere, so an env's result never
    // depends on which other envs share its wave; the wave-uniform test only skips the full series
    // when no lane needs it
    const double x2 = x * x;
    const bool tiny = __builtin_fabs(x) <= 0.03;
    double ps = -0.0001984126984126984;                                // f64::sincos_tiny's terms
    ps = f64::fma_(ps, x2, 0.008333333333333333);
    ps = f64::fma_(ps, x2, -0.16666666666666666);
    double pc = 2.48015873015873e-05;
    pc = f64::fma_(pc, x2, -0.001388888888888889);
    pc = f64::fma_(pc, x2, 0.041666666666666664);
    pc = f64::fma_(pc, x2, -0.5);
    if (__builtin_expect(!__all(tiny), 0)) {                            // f64::sincos_small's terms
        double fs = 1.6059043836821613e-10;
        fs = f64::fma_(fs, x2, -2.505210838544172e-08);
        fs = f64::fma_(fs, x2, 2.7557319223985893e-06);
        fs = f64::fma_(fs, x2, -0.0001984126984126984);
        fs = f64::fma_(fs, x2, 0.008333333333333333);
        fs = f64::fma_(fs, x2, -0.16666666666666666);
        double fc = -1.1470745597729725e-11;
        fc = f64::fma_(fc, x2, 2.08767569878681e-09);
        fc = f64::fma_(fc, x2, -2.755731922398589e-07);
        fc = f64::fma_(fc, x2, 2.48015873015873e-05);
        fc = f64::fma_(fc, x2, -0.001388888888888889);
        fc = f64::fma_(fc, x2, 0.041666666666666664);
        fc = f64::fma_(fc, x2, -0.5);
        ps = tiny ? ps : fs;
        pc = tiny ? pc : fc;
    }
    *sinc = f64::fma_(x2, ps, 1.0);
    *c = f64::fma_(x2, pc, 1.0);
}
// expmap_sinc_cos with the full series and no wave-uniform branch (the race quad kernel, where the
// branchy short forms measured slower)
__device__ __forceinline__ void expmap_sinc_cos_full(float x, float* sinc, float* c) { expmap_sinc_cos(x, sinc, c); }
__device__ __forceinline__ void expmap_sinc_cos_full(double x, double* sinc, double* c) {
    const double x2 = x * x;
    double ps = 1.6059043836821613e-10;
    ps = f64::fma_(ps, x2, -2.505210838544172e-08);
    ps = f64::fma_(ps, x2, 2.7557319223985893e-06);
    ps = f64::fma_(ps, x2, -0.0001984126984126984);
    ps = f64::fma_(ps, x2, 0.008333333333333333);
    ps = f64::fma_(ps, x2, -0.16666666666666666);
    double pc = -1.1470745597729725e-11;
    pc = f64::fma_(pc, x2, 2.08767569878681e-09);
    pc = f64::fma_(pc, x2, -2.755731922398589e-07);
    pc = f64::fma_(pc, x2, 2.48015873015873e-05);
    pc = f64::fma_(pc, x2, -0.001388888888888889);
    pc = f64::fma_(pc, x2, 0.041666666666666664);
    pc = f64::fma_(pc, x2, -0.5);
    *sinc = f64::fma_(x2, ps, 1.0);
    *c = f64::fma_(x2, pc, 1.0);
}
// 1/|q| of the exp-map quaternion: |q1|^2 = |q0|^2 (cos^2 + sin^2) = 1 up to rounding unless the
// |w| dt threshold clamped the angle, so where |n2 - 1| <= 1e-9 one Newton step from 1,
// 1 + (1 - n2) / 2 (error 3/8 (n2 - 1)^2 <= 4e-19), else the refined rsq (fp32: v_rsq).  The choice is
// per lane (batch-invariant); the wave-uniform test only skips the rsq when no lane needs it.
__device__ __forceinline__ float quat_inv_norm(float n2) { return __builtin_amdgcn_rsqf(n2); }
__device__ __forceinline__ double quat_inv_norm(double n2) {
    const bool near1 = __builtin_fabs(n2 - 1.0) <= 1e-9;
    const double newton = f64::fma_(0.5, 1.0 - n2, 1.0);
    if (__builtin_expect(__all(near1), 1)) return newton;
    const double r = f64::rsq_nc(n2);
    return near1 ? newton : r;
}

// fast fp32 transcendentals for the latency-bound sub-step loop (fp64: the f64 forms above).
// atan on [0,1] is an odd minimax polynomial (|err| <= 1.1e-7 rad, fitted by IRLS on
// Chebyshev nodes, checked in fp32 Horner), after octant reduction with a hardware reciprocal.
__device__ __forceinline__ float fatan2_(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    const float t = a * a;
    float p = 0.0028487828094512224f;
    p = p * t - 0.016064105555415154f;
    p = p * t + 0.04268398508429527f;
    p = p * t - 0.07503638416528702f;
    p = p * t + 0.10640615969896317f;
    p = p * t - 0.1420356035232544f;
    p = p * t + 0.19992607831954956f;
    p = p * t - 0.3333307206630707f;
    p = p * t + 1.0f;
    float r = a * p;
    if (ay > ax) r = 1.57079632679489661923f - r;
    if (x < 0.0f) r = 3.14159265358979323846f - r;
    return copysignf(r, y);
}
__device__ __forceinline__ double fatan2_(double y, double x) { return f64::atan2(y, x); }
// finite arguments (no NaN / inf fix-ups in fp64)
__device__ __forceinline__ float fatan2_nc_(float y, float x) { return fatan2_(y, x); }
__device__ __forceinline__ double fatan2_nc_(double y, double x) { return f64::atan2_nc(y, x); }
__device__ __forceinline__ float fasin_(float s) { return fatan2_(s, __builtin_amdgcn_sqrtf((1.0f - s) * (1.0f + s))); }
__device__ __forceinline__ double fasin_(double s) { return f64::asin(s); }
__device__ __forceinline__ float fexp_(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ double fexp_(double x) { return f64::exp(x); }

// ---- literal constants of the fp64 sub-step chains, held in VGPRs ----------------------------
// gfx950 has no 64-bit literal operand: an fp64 constant costs two s_mov / v_mov at every use the
// compiler rematerialises it for (about a sixth of the hover fp64 sub-step's instructions).  The
// chains take their constants from a ChainK that the kernel pins into VGPRs once, before the
// sub-step loop (an empty asm that "modifies" the value: it cannot be re-derived as a literal).
template <typename Real>
struct ChainK {
    Real k004, c100, nn_min, near1, tiny;   // 0.04, 100, 1e-300, 1e-9, 0.03
    Real ts[3], tc[4];                      // the exp map's short series (f64::sincos_tiny's terms)
};
template <typename Real>
__device__ __forceinline__ ChainK<Real> chain_consts() {
    return ChainK<Real>{Real(0.04), Real(100), Real(1e-300), Real(1e-9), Real(0.03),
                        {Real(-0.0001984126984126984), Real(0.008333333333333333), Real(-0.16666666666666666)},
                        {Real(2.48015873015873e-05), Real(-0.001388888888888889), Real(0.041666666666666664), Real(-0.5)}};
}
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(float&) {}
template <typename Real>
__device__ __forceinline__ void pin_all(ChainK<Real>& k) {
    pin(k.k004); pin(k.c100); pin(k.nn_min); pin(k.near1); pin(k.tiny);
#pragma unroll
    for (int i = 0; i < 3; ++i) pin(k.ts[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) pin(k.tc[i]);
}
// the pinned-constant forms of sqrt_nn / expmap_sinc_cos / quat_inv_norm (same arithmetic)
__device__ __forceinline__ float hsqrt_nn_(float x, const ChainK<float>&) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double hsqrt_nn_(double x, const ChainK<double>& k) {
    const double y = __builtin_amdgcn_rsq(__builtin_fmax(x, k.nn_min));
    double g = x * y, h = 0.5 * y;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double r = f64::fma_(-g, h, 0.5);
        g = f64::fma_(g, r, g);
        h = f64::fma_(h, r, h);
    }
    const double d = f64::fma_(-g, g, x);
    return f64::fma_(d, h, g);
}
__device__ __forceinline__ void expmap_sinc_cos(float x, float* sinc, float* c, const ChainK<float>&) {
    expmap_sinc_cos(x, sinc, c);
}
__device__ __forceinline__ void expmap_sinc_cos(double x, double* sinc, double* c, const ChainK<double>& k) {
    const double x2 = x * x;
    const bool tiny = __builtin_fabs(x) <= k.tiny;
    double ps = f64::fma_(k.ts[0], x2, k.ts[1]);
    ps = f64::fma_(ps, x2, k.ts[2]);
    double pc = f64::fma_(k.tc[0], x2, k.tc[1]);
    pc = f64::fma_(pc, x2, k.tc[2]);
    pc = f64::fma_(pc, x2, k.tc[3]);
    if (__builtin_expect(!__all(tiny), 0)) {   // the full series (cold: literal coefficients)
        double fs, fc;
        expmap_sinc_cos_full(x, &fs, &fc);
        *sinc = tiny ? f64::fma_(x2, ps, 1.0) : fs;
        *c = tiny ? f64::fma_(x2, pc, 1.0) : fc;
        return;
    }
    *sinc = f64::fma_(x2, ps, 1.0);
    *c = f64::fma_(x2, pc, 1.0);
}
__device__ __forceinline__ float quat_inv_norm(float n2, const ChainK<float>&) { return quat_inv_norm(n2); }
__device__ __forceinline__ double quat_inv_norm(double n2, const ChainK<double>& k) {
    const bool near1 = __builtin_fabs(n2 - 1.0) <= k.near1;
    const double newton = f64::fma_(0.5, 1.0 - n2, 1.0);
    if (__builtin_expect(__all(near1), 1)) return newton;
    const double r = f64::rsq_nc(n2);
    return near1 ? newton : r;
}

// btClamp(x, -100, 100) of the six coordinate velocities (btMultiBody m_maxCoordinateVelocity) after
// the semi-implicit Euler update.  fp32: one v_med3 each.  fp64 has no med3, and the select form
// (x < -100 ? -100 : x > 100 ? 100 : x) is 2 compares + 4 32-bit selects per component on every
// sub-step of the dependent chain; the clamp is the identity unless a component exceeds 100 in
// magnitude, so a wave-uniform test guards the exact select form (NaN passes through as in btClamp).
__device__ __forceinline__ void clamp100_wv(V3<float>& w, V3<float>& v) {
    w = {__builtin_amdgcn_fmed3f(w.x, -100.0f, 100.0f), __builtin_amdgcn_fmed3f(w.y, -100.0f, 100.0f),
         __builtin_amdgcn_fmed3f(w.z, -100.0f, 100.0f)};
    v = {__builtin_amdgcn_fmed3f(v.x, -100.0f, 100.0f), __builtin_amdgcn_fmed3f(v.y, -100.0f, 100.0f),
         __builtin_amdgcn_fmed3f(v.z, -100.0f, 100.0f)};
}
__device__ __forceinline__ double clamp100_sel(double x) { return x < -100.0 ? -100.0 : (x > 100.0 ? 100.0 : x); }
__device__ __forceinline__ void clamp100_wv(V3<double>& w, V3<double>& v) {
    const bool big = (__builtin_fabs(w.x) > 100.0) | (__builtin_fabs(w.y) > 100.0) | (__builtin_fabs(w.z) > 100.0) |
                     (__builtin_fabs(v.x) > 100.0) | (__builtin_fabs(v.y) > 100.0) | (__builtin_fabs(v.z) > 100.0);
    if (__builtin_expect(__any(big), 0)) {
        w = {clamp100_sel(w.x), clamp100_sel(w.y), clamp100_sel(w.z)};
        v = {clamp100_sel(v.x), clamp100_sel(v.y), clamp100_sel(v.z)};
    }
}

__device__ __forceinline__ void clamp100_wv(V3<float>& w, V3<float>& v, const ChainK<float>&) { clamp100_wv(w, v); }
__device__ __forceinline__ void clamp100_wv(V3<double>& w, V3<double>& v, const ChainK<double>& k) {
    const double c = k.c100;
    const bool big = (__builtin_fabs(w.x) > c) | (__builtin_fabs(w.y) > c) | (__builtin_fabs(w.z) > c) |
                     (__builtin_fabs(v.x) > c) | (__builtin_fabs(v.y) > c) | (__builtin_fabs(v.z) > c);
    if (__builtin_expect(__any(big), 0)) {
        w = {clamp100_sel(w.x), clamp100_sel(w.y), clamp100_sel(w.z)};
        v = {clamp100_sel(v.x), clamp100_sel(v.y), clamp100_sel(v.z)};
    }
}

// rotation matrix of a unit quaternion (body->world)
template <typename Real>
__device__ __forceinline__ M3<Real> rot(Q4<Real> q) {
    const Real x2 = q.x + q.x, y2 = q.y + q.y, z2 = q.z + q.z;
    const Real xx = q.x * x2, yy = q.y * y2, zz = q.z * z2;
    const Real xy = q.x * y2, xz = q.x * z2, yz = q.y * z2;
    const Real wx = q.w * x2, wy = q.w * y2, wz = q.w * z2;
    return {Real(1) - (yy + zz), xy - wz, xz + wy,
            xy + wz, Real(1) - (xx + zz), yz - wx,
            xz - wy, yz + wx, Real(1) - (xx + yy)};
}
template <typename Real>
__device__ __forceinline__ V3<Real> mul(const M3<Real>& R, V3<Real> v) {
    return {R.a00 * v.x + R.a01 * v.y + R.a02 * v.z,
            R.a10 * v.x + R.a11 * v.y + R.a12 * v.z,
            R.a20 * v.x + R.a21 * v.y + R.a22 * v.z};
}
template <typename Real>
__device__ __forceinline__ V3<Real> mulT(const M3<Real>& R, V3<Real> v) {
    return {R.a00 * v.x + R.a10 * v.y + R.a20 * v.z,
            R.a01 * v.x + R.a11 * v.y + R.a21 * v.z,
            R.a02 * v.x + R.a12 * v.y + R.a22 * v.z};
}
template <typename Real>
__device__ __forceinline__ V3<Real> col2(const M3<Real>& R) {  // body z axis in world
    return {R.a02, R.a12, R.a22};
}

// pybullet getEulerFromQuaternion (extrinsic x-y-z), incl. its gimbal-lock branches
template <typename Real>
__device__ __forceinline__ V3<Real> euler_xyz(Q4<Real> q) {
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    const Real half_pi = Real(1.57079632679489661923);
    if (sarg <= Real(-0.99999)) return {Real(0), -half_pi, Real(2) * atan2_(q.x, -q.y)};
    if (sarg >= Real(0.99999)) return {Real(0), half_pi, Real(2) * atan2_(-q.x, q.y)};
    return {atan2_(Real(2) * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz), asin_(sarg),
            atan2_(Real(2) * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz)};
}

// euler_xyz with the fast fp32 atan2/asin (controller input inside the sub-step loop)
template <typename Real>
__device__ __forceinline__ V3<Real> euler_xyz_fast(Q4<Real> q) {
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    const Real half_pi = Real(1.57079632679489661923);
    if (sarg <= Real(-0.99999)) return {Real(0), -half_pi, Real(2) * fatan2_(q.x, -q.y)};
    if (sarg >= Real(0.99999)) return {Real(0), half_pi, Real(2) * fatan2_(-q.x, q.y)};
    return {fatan2_(Real(2) * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz), fasin_(sarg),
            fatan2_(Real(2) * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz)};
}

// euler_xyz_fast with the gimbal-lock branches behind a wave-uniform test: the common path
// evaluates 3 atan2 instead of the 5 an if-converted select computes (call with the lanes
// that need the result active; inactive lanes do not vote)
template <typename Real>
__device__ __forceinline__ V3<Real> euler_xyz_fast_u(Q4<Real> q) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) return euler_xyz_fast(q);
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    return {fatan2_(Real(2) * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz), fasin_(sarg),
            fatan2_(Real(2) * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz)};
}

// getQuaternionFromEuler (rpy extrinsic xyz)
template <typename Real>
__device__ __forceinline__ Q4<Real> quat_from_euler(Real r, Real p, Real y) {
    Real sr, cr, sp, cp, sy, cy;
    sincos_(r * Real(0.5), &sr, &cr);
    sincos_(p * Real(0.5), &sp, &cp);
    sincos_(y * Real(0.5), &sy, &cy);
    return {sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
            cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy};
}

// getQuaternionFromEuler with the half-angle sin/cos from the small-angle polynomial when all
// three half angles are within pi/8 (exact in fp32, as small_sincos; fp64: f64::sincos_small, within
// an ulp of libm), else from libm (fp32) / the octant-reduced f64::sincos_fast (fp64)
template <typename Real>
__device__ __forceinline__ Q4<Real> quat_from_euler_fast(Real r, Real p, Real y) {
    const Real hr = r * Real(0.5), hp = p * Real(0.5), hy = y * Real(0.5);
    const Real lim = Real(0.39269908169872414);
    Real sr, cr, sp, cp, sy, cy;
    if (fabs_(hr) <= lim && fabs_(hp) <= lim && fabs_(hy) <= lim) {
        small_sincos(hr, &sr, &cr);
        small_sincos(hp, &sp, &cp);
        small_sincos(hy, &sy, &cy);
    } else {
        if constexpr (sizeof(Real) == 4) return quat_from_euler(r, p, y);
        sincos_f_(hr, &sr, &cr);
        sincos_f_(hp, &sp, &cp);
        sincos_f_(hy, &sy, &cy);
    }
    return {sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
            cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy};
}

// Box-Muller of one Philox word pair from IEEE float operations only (+ - * /, correctly rounded
// sqrtf, fmaf, frexpf, rintf), the same sequence as the oracle's normal_pair_f (oracle/race.c), so the
// fp64 kernels' action noise is bit-identical to the oracle's: u1 = (x0 >> 8 + 1) 2^-24,
// u2 = (x1 >> 8) 2^-24, r = sqrt(-2 log u1) with log u1 = e ln2 + 2 atanh((m - 1) / (m + 1)),
// (sin, cos)(2 pi u2) from the octant rint(8 u2) and a Taylor pair on |x| <= pi / 8 (~2 float ulp).
// No contraction: every fma is explicit.  (The fp32 kernels keep the hardware v_log / v_sin / v_cos
// form, which differs by float rounding.)
__device__ __forceinline__ void normal_pair_f(uint32_t x0, uint32_t x1, float* z0, float* z1) {
#pragma clang fp contract(off)
    const float u1 = (float(x0 >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = float(x1 >> 8) * (1.0f / 16777216.0f);
    int e;
    float m = __builtin_frexpf(u1, &e);
    if (m < 0.70710677f) { m = m * 2.0f; e -= 1; }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float z = s * s;
    float p = 1.0f / 11;
    p = __builtin_fmaf(p, z, 1.0f / 9); p = __builtin_fmaf(p, z, 1.0f / 7);
    p = __builtin_fmaf(p, z, 1.0f / 5); p = __builtin_fmaf(p, z, 1.0f / 3);
    const float lm = __builtin_fmaf(2.0f * s * z, p, 2.0f * s);
    const float fe = float(e);
    const float lg = __builtin_fmaf(fe, 0.693145751953125f, __builtin_fmaf(fe, 1.428606765330187e-06f, lm));
    const float r = __builtin_sqrtf(-2.0f * lg);
    const float n = __builtin_rintf(u2 * 8.0f);
    const float x = (u2 - n * 0.125f) * 6.28318548f;
    const float x2 = x * x;
    float ps = -1.98412698e-4f;
    ps = __builtin_fmaf(ps, x2, 8.33333377e-3f); ps = __builtin_fmaf(ps, x2, -0.166666672f);
    float pc = 2.48015876e-5f;
    pc = __builtin_fmaf(pc, x2, -1.38888892e-3f); pc = __builtin_fmaf(pc, x2, 4.16666679e-2f);
    pc = __builtin_fmaf(pc, x2, -0.5f);
    const float sx = __builtin_fmaf(x * x2, ps, x), cx = __builtin_fmaf(x2, pc, 1.0f);
    const float h = 0.70710677f;
    const float a = h * (cx + sx), b = h * (cx - sx);
    // sin / cos of o pi / 4 + x, o = n mod 8, branch-free (the oracle's octant table, the same values):
    // odd o starts from (sin, cos)(pi / 4 + x) = (a, b), even o from (sx, cx); then the quadrant
    // q = o >> 1 turns it by q pi / 2: bit 0 maps (s, c) -> (c, -s), bit 1 negates both
    const uint32_t o = uint32_t(int(n)) & 7u;
    const bool odd = (o & 1u) != 0;
    const float s0 = odd ? a : sx, c0 = odd ? b : cx;
    const bool turn = (o & 2u) != 0;
    const uint32_t neg = (o & 4u) << 29;                    // sign bit when bit 2 is set
    const float s1 = turn ? c0 : s0;
    const float c1 = turn ? __uint_as_float(__float_as_uint(s0) ^ 0x80000000u) : c0;
    const float sn = __uint_as_float(__float_as_uint(s1) ^ neg);
    const float cs = __uint_as_float(__float_as_uint(c1) ^ neg);
    *z0 = r * cs;
    *z1 = r * sn;
}

// ---- Philox4x32-10 (Salmon et al. SC'11) -------------------------------------------------
struct U4 {
    uint32_t a, b, c, d;
};
__device__ __forceinline__ U4 philox4x32_10(U4 ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.a), lo0 = 0xD2511F53u * ctr.a;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.c), lo1 = 0xCD9E8D57u * ctr.c;
        ctr = U4{hi1 ^ ctr.b ^ k0, lo1, hi0 ^ ctr.d ^ k1, lo0};
    }
    return ctr;
}
// uniform in [0,1) with 24 random bits: exact in float and double alike
__device__ __forceinline__ double u01(uint32_t x) { return double(x >> 8) * (1.0 / 16777216.0); }
// the same value in Real (a 24-bit integer times 2^-24 is exact in fp32 too)
template <typename Real>
__device__ __forceinline__ Real u01r(uint32_t x) { return Real(x >> 8) * Real(1.0 / 16777216.0); }

// counter layout (shared by specification with the oracle):
//   {global env id (low 32 bits), episode, tag, index}, key = {seed lo, seed hi}
__device__ __forceinline__ U4 draw(uint64_t seed, uint64_t gid, uint32_t episode, uint32_t tag,
                                   uint32_t idx) {
    return philox4x32_10(U4{uint32_t(gid), episode, tag, idx}, uint32_t(seed), uint32_t(seed >> 32));
}

constexpr uint32_t TAG_HOVER_RESET = 0x48520000u;

}  // namespace adrp
