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
#else
#define RACE_MARK(var)
#define RACE_SET(var)
#define RACE_ACC(i, dt)
#define RACE_WAVE(i, dt)
#endif


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

__device__ __forceinline__ float rsqrt_(float x) { return __frsqrt_rn(x); }
__device__ __forceinline__ double rsqrt_(double x) { return 1.0 / sqrt(x); }
__device__ __forceinline__ float sqrt_(float x) { return __fsqrt_rn(x); }
__device__ __forceinline__ double sqrt_(double x) { return sqrt(x); }
__device__ __forceinline__ void sincos_(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void sincos_(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ float atan2_(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double atan2_(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float asin_(float x) { return asinf(x); }
__device__ __forceinline__ double asin_(double x) { return asin(x); }
__device__ __forceinline__ float exp_(float x) { return expf(x); }
__device__ __forceinline__ double exp_(double x) { return exp(x); }
__device__ __forceinline__ float fabs_(float x) { return fabsf(x); }
__device__ __forceinline__ double fabs_(double x) { return fabs(x); }

// latency-oriented fp32 primitives (1-ulp hardware ops); fp64 keeps IEEE-exact ones
__device__ __forceinline__ float rcp_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp_(double x) { return 1.0 / x; }
__device__ __forceinline__ float hsqrt_(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double hsqrt_(double x) { return sqrt(x); }
__device__ __forceinline__ float hrsqrt_(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double hrsqrt_(double x) { return 1.0 / sqrt(x); }

// sin/cos for |x| <= pi/8 (the exp-map half angle is clamped there): Taylor to x^7 / x^8,
// truncation error < 2e-9 relative, i.e. exact in fp32; fp64 uses the libm call.
__device__ __forceinline__ void small_sincos(float x, float* s, float* c) {
    const float x2 = x * x;
    *s = x * (1.0f + x2 * (-1.0f / 6.0f + x2 * (1.0f / 120.0f + x2 * (-1.0f / 5040.0f))));
    *c = 1.0f + x2 * (-0.5f + x2 * (1.0f / 24.0f + x2 * (-1.0f / 720.0f + x2 * (1.0f / 40320.0f))));
}
__device__ __forceinline__ void small_sincos(double x, double* s, double* c) { sincos(x, s, c); }

// fast fp32 transcendentals for the latency-bound sub-step loop (the fp64 overloads keep
// libm). atan on [0,1] is an odd minimax polynomial (|err| <= 1.1e-7 rad, fitted by IRLS on
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
__device__ __forceinline__ double fatan2_(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float fasin_(float s) { return fatan2_(s, __builtin_amdgcn_sqrtf((1.0f - s) * (1.0f + s))); }
__device__ __forceinline__ double fasin_(double s) { return asin(s); }
__device__ __forceinline__ float fexp_(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ double fexp_(double x) { return exp(x); }

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
// three half angles are within pi/8 (exact in fp32, as small_sincos), else from libm; fp64
// is always libm
template <typename Real>
__device__ __forceinline__ Q4<Real> quat_from_euler_fast(Real r, Real p, Real y) {
    if constexpr (sizeof(Real) == 4) {
        const Real hr = r * Real(0.5), hp = p * Real(0.5), hy = y * Real(0.5);
        const Real lim = Real(0.39269908169872414);
        if (fabs_(hr) <= lim && fabs_(hp) <= lim && fabs_(hy) <= lim) {
            Real sr, cr, sp, cp, sy, cy;
            small_sincos(hr, &sr, &cr);
            small_sincos(hp, &sp, &cp);
            small_sincos(hy, &sy, &cy);
            return {sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                    cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy};
        }
    }
    return quat_from_euler(r, p, y);
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
