// race_quad.h — MultiRaceAviary env.step, four lanes per drone (gfx950), fp32 and fp64.
//
// The one-lane kernel (race_kernel.h) puts a drone on a lane, so config 4 (16,384 drones) is 256
// waves: one per CU, on one of its four SIMDs, each issuing one VALU instruction per 4 cycles
// through a ~1000-instruction dependent chain per 500 Hz sub-step.  Here a drone owns a quad of
// lanes (lane = 4 * drone + ql), so the same batch is 1024 waves, one per SIMD, and the chain of
// each wave is shorter wherever the quad splits the work of one drone:
//   * downwash: lane ql evaluates the partner drone ql (ds_bpermute of its position), the
//     contributions are summed in partner order as in the one-lane loop;
//   * Euler angles of the controller input: lane ql evaluates angle min(ql, 2) (one atan2 instead
//     of three), and keeps that axis's rate history and 2-pole gyro filter state;
//   * the PWM -> thrust -> noise -> RPM chain: lane ql runs motor ql, the firmware's thrust
//     reorder [3,2,1,0] is one DPP quad mirror, the RPMs come back by DPP quad broadcasts;
//   * the rotation matrices of the current and the cached link pose are carried across sub-steps
//     (one quaternion -> matrix per sub-step instead of three);
//   * the sub-step disturbance draws are made by the quad's lanes up front (sub-steps s = ql mod 4)
//     into LDS, and the env's actual track is copied to LDS for the post-loop queries.
// Everything else (the Bullet step, the firmware controllerMellinger, rays, obs, contacts,
// reward, reset) runs redundantly on the quad's four lanes; lane ql = 0 owns the stores.  The
// per-element arithmetic is the one-lane kernel's, operation for operation (the same functions
// with the same contraction scopes), so the two layouts agree (tests/test_race_gpu.py
// test_quad_matches_lane).  Real = double is the reference-precision kernel: float64 physics and
// MellingerControl wrapper (numpy's divisions), float firmware, as in the one-lane fp64 kernel;
// cross-lane moves of doubles are two 32-bit DPP / swizzle moves.
#pragma once

#include <type_traits>

#include "race_kernel.h"

namespace adrp {

constexpr int kQuadDrones = kRaceBlock / 4;   // drones per 64-lane block

// the downwash exponential: fp32 v_exp_f32; fp64 the table form (x <= 0)
__device__ __forceinline__ float dw_exp(float x, const double*) { return fexp_(x); }
__device__ __forceinline__ double dw_exp(double x, const double* tab) { return f64::exp_tab(x, tab); }

// DPP quad moves (one VALU op): value of quad lane k (k must fold to a constant), and the mirror
// lane 3 - ql
__device__ __forceinline__ int qbc_i(int v, int k) {
    switch (k) {
        case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false);
        case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false);
        case 2: return __builtin_amdgcn_mov_dpp(v, 0xaa, 0xf, 0xf, false);
        default: return __builtin_amdgcn_mov_dpp(v, 0xff, 0xf, 0xf, false);
    }
}
__device__ __forceinline__ float qbc(float v, int k) { return __int_as_float(qbc_i(__float_as_int(v), k)); }
__device__ __forceinline__ double qbc(double v, int k) {
    return __hiloint2double(qbc_i(__double2hiint(v), k), qbc_i(__double2loint(v), k));
}
// quad butterfly partners: quad_perm [1, 0, 3, 2] and [2, 3, 0, 1]
__device__ __forceinline__ float qswap1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));
}
__device__ __forceinline__ float qswap2(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false));
}
__device__ __forceinline__ double qswap1(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0xb1, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0xb1, 0xf, 0xf, false));
}
__device__ __forceinline__ double qswap2(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x4e, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x4e, 0xf, 0xf, false));
}
__device__ __forceinline__ float qmirror(float v) {   // quad_perm [3, 2, 1, 0]
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x1b, 0xf, 0xf, false));
}
__device__ __forceinline__ double qmirror(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x1b, 0xf, 0xf, false),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x1b, 0xf, 0xf, false));
}

// value of drone k of this lane's env (its quad lane ql): the env's G quads are 4G <= 32 aligned
// lanes, so ds_swizzle's bit mode (within 32 lanes: src = (lane & and) | or) addresses it without
// an index register.  k must fold to a constant.
template <int G>
__device__ __forceinline__ int grpq_i(int v, int k) {
    if constexpr (G == 1) {
        return v;
    } else {
        constexpr int am = 31 & ~((G - 1) << 2);   // or_mask = 4k sits at bits [9:5] of the pattern
        switch (k) {
            case 0: return __builtin_amdgcn_ds_swizzle(v, am);
            case 1: return __builtin_amdgcn_ds_swizzle(v, am | (1 << 7));
            case 2: return __builtin_amdgcn_ds_swizzle(v, am | (2 << 7));
            case 3: return __builtin_amdgcn_ds_swizzle(v, am | (3 << 7));
            case 4: return __builtin_amdgcn_ds_swizzle(v, am | (4 << 7));
            case 5: return __builtin_amdgcn_ds_swizzle(v, am | (5 << 7));
            case 6: return __builtin_amdgcn_ds_swizzle(v, am | (6 << 7));
            default: return __builtin_amdgcn_ds_swizzle(v, am | (7 << 7));
        }
    }
}
template <int G>
__device__ __forceinline__ float grpq(float v, int k) { return __int_as_float(grpq_i<G>(__float_as_int(v), k)); }
template <int G>
__device__ __forceinline__ double grpq(double v, int k) {
    return __hiloint2double(grpq_i<G>(__double2hiint(v), k), grpq_i<G>(__double2loint(v), k));
}

// this lane's controller Euler angle (axis a = min(ql, 2)) of euler_xyz_fast_u(q): the same
// atan2 / asin expressions, one per lane; the rare gimbal-lock branch evaluates all three
template <typename Real>
__device__ __forceinline__ Real euler_axis_q4(Q4<Real> q, int a) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) {
        const V3<Real> r = euler_xyz_fast(q);
        return a == 0 ? r.x : (a == 1 ? r.y : r.z);
    }
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    const Real y0 = Real(2) * (q.y * q.z + q.w * q.x), x0 = squ - sqx - sqy + sqz;
    const Real y2 = Real(2) * (q.x * q.y + q.w * q.z), x2 = squ + sqx - sqy - sqz;
    // fasin_(sarg); the argument is > 0 here (|sarg| < 0.99999), the operands finite
    const Real x1 = hsqrt_nn_((Real(1) - sarg) * (Real(1) + sarg));
    const Real yy = a == 0 ? y0 : (a == 1 ? sarg : y2), xx = a == 0 ? x0 : (a == 1 ? x1 : x2);
    return fatan2_nc_(yy, xx);
}

// MellingerControl.computeControl (154-262) for the quad: lane ql owns axis min(ql, 2) of the
// rates / gyro filter (rpy_a, prv, l1, l2) and motor ql of the PWM chain (noise_m).  Same
// arithmetic as mellinger_compute<Real> (FP contraction off; fp32: reciprocal multiplies, fp64:
// numpy's correctly rounded divisions (by constants: divc_) and the firmware's C float divisions),
// split across the quad.
// measurement-only (make devx XD=-DADRP_EXP_DUP_...): a phase evaluated twice, the second pass
// made to wait for the first through an empty asm, so the kernel's time grows by the phase's cost on
// the chain while every result (and so the trajectory) is unchanged
template <typename T, typename U>
__device__ __forceinline__ void exp_dep(T& x, const U& after) { asm volatile("" : "+v"(x) : "v"(after)); }
template <typename T>
__device__ __forceinline__ void exp_sink(const T& x) { asm volatile("" ::"v"(x)); }

template <typename T>
__device__ __forceinline__ T sel3(const T (&v)[3], int a) { return a == 0 ? v[0] : (a == 1 ? v[1] : v[2]); }

#ifdef ADRP_CTRL_PHASES   // measurement-only: the controller's sub-phases (tools/race_phases.py, make devc)
#define CP_PARAM , uint64_t (&cp)[8]
#define CP_ARG , cp
#define CP_MARK(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define CP_ADD(i, dt) cp[i] += (dt)
#else
#define CP_PARAM
#define CP_ARG
#define CP_MARK(var)
#define CP_ADD(i, dt)
#endif
template <typename Real>
__device__ __forceinline__ void mellinger_q4(RDrone<Real>& d, const Lpf& lpf, const float sp[3], float xc_x,
                                             float xc_y, Real rpy_a, Real& prv, float& l1, float& l2, Real noise_m,
                                             int ql, const M3<Real>& Rq CP_PARAM) {
#pragma clang fp contract(off)
    constexpr bool F32 = sizeof(Real) == 4;
    CP_MARK(m0);
    const Real rate = F32 ? (rpy_a - prv) * Real(500) : divc_(rpy_a - prv, Real(0.002));
    prv = rpy_a;
    const Real acc_z = F32 ? (d.vel.z - d.prev_vel[2]) * Real(500.0 / 9.8) + Real(1)
                           : divc_(divc_(d.vel.z - d.prev_vel[2], Real(0.002)), Real(9.8)) + Real(1);
    d.prev_vel[0] = d.vel.x; d.prev_vel[1] = d.vel.y; d.prev_vel[2] = d.vel.z;
    const float g_a = lpf_apply(lpf, l1, l2, float(rate * Real(57.29577951308232)));
    const float gyro[3] = {qbc(g_a, 0), qbc(g_a, 1), qbc(g_a, 2)};
    Real pwm;
    CP_MARK(m1);
    CP_ADD(1, m1 - m0);
    if (float(acc_z) < -0.5f) d.tumble += 1; else d.tumble = 0;
    if (d.tumble >= 30) {
        d.tick += 1;
        pwm = Real(0);
    } else {
        const int da = d.tick - d.last_att, dp = d.tick - d.last_pos, bit = d.tick - d.tick_base;
        const bool att_due = (da >= 2) | ((da == 1) & (((d.att_bits >> bit) & 1u) != 0));
        const bool pos_due = (dp >= 6) | ((dp == 5) & (((d.pos_bits >> bit) & 1u) != 0));
        d.last_pos = (att_due & pos_due) ? d.tick : d.last_pos;
        d.last_att = att_due ? d.tick : d.last_att;
        if (att_due) {
            float Rm[9];
            const Real sarg = Real(-2) * (d.q.x * d.q.z - d.q.w * d.q.y);
            Rm[0] = float(Rq.a00); Rm[1] = float(Rq.a01); Rm[2] = float(Rq.a02);
            Rm[3] = float(Rq.a10); Rm[4] = float(Rq.a11); Rm[5] = float(Rq.a12);
            Rm[6] = float(Rq.a20); Rm[7] = float(Rq.a21); Rm[8] = float(Rq.a22);
            if (__builtin_expect(__any(!(fabs_(sarg) < Real(0.99999))), 0)) {
                if (!(fabs_(sarg) < Real(0.99999))) {
                    const V3<Real> rpy = euler_xyz_fast(d.q);
                    float sr, cr, sp_, cp, sy, cy;
                    sincosf(float(rpy.x), &sr, &cr);
                    sincosf(float(rpy.y), &sp_, &cp);
                    sincosf(float(rpy.z), &sy, &cy);
                    Rm[0] = cy * cp; Rm[1] = cy * sp_ * sr - sy * cr; Rm[2] = cy * sp_ * cr + sy * sr;
                    Rm[3] = sy * cp; Rm[4] = sy * sp_ * sr + cy * cr; Rm[5] = sy * sp_ * cr - cy * sr;
                    Rm[6] = -sp_; Rm[7] = cp * sr; Rm[8] = cp * cr;
                }
            }
            const float pos[3] = {float(d.pos.x), float(d.pos.y), float(d.pos.z)};
            const float vel[3] = {float(d.vel.x), float(d.vel.y), float(d.vel.z)};
            // (a quad split of the firmware, one division per lane for the thrust / z_des / y_des
            // components and DPP broadcasts, measured slower in both precisions: +1.1 us fp64,
            // +0.1 us fp32 on config 4, A/B round 4)
#ifdef ADRP_EXP_DUP_FW
            {
                RDrone<Real> d2 = d;
                mellinger_fw<Real, F32, false>(d2, sp, xc_x, xc_y, gyro, pos, vel, Rm);
                float p0 = pos[0];
                exp_dep(p0, d2.ctl[0]);
                const float pos2[3] = {p0, pos[1], pos[2]};
                mellinger_fw<Real, F32, false>(d, sp, xc_x, xc_y, gyro, pos2, vel, Rm);
            }
#else
            mellinger_fw<Real, F32, false>(d, sp, xc_x, xc_y, gyro, pos, vel, Rm);
#endif
        }
        CP_MARK(m2);
        CP_ADD(2, m2 - m1);
        d.tick += 1;
        // _compute_pwms (423-442), motor ql of [t-r+p+y, t-r-p-y, t+r-p+y, t+r+p-y]
        // (reusing the thrust between firmware calls, where control_t is unchanged, measured slower:
        // config 4 fp64 69.5 -> 73.8 us, config 3 47.1 -> 49.8 us, A/B round 5)
        const Real r = Real(d.ctl[0]) / Real(2), p = Real(d.ctl[1]) / Real(2), y = Real(d.ctl[2]), th = Real(d.ctl[3]);
        const Real m = ((th + (ql < 2 ? -r : r)) + ((ql == 0 || ql == 3) ? p : -p)) + ((ql & 1) ? -y : y);
        const Real x = F32 ? clampr_(m, Real(0), Real(65535)) * Real(60.0 / 65535)
                           : divc_(clampr_(m, Real(0), Real(65535)), Real(65535)) * Real(60);
        const Real volts = Real(-0.0006239) * x * x + Real(0.088) * x;
        pwm = minr_(F32 ? volts * Real(1.0 / 3) : divc_(volts, Real(3)), Real(1)) * Real(65535);
    }
    // clip -> thrust -> reorder [3,2,1,0] -> + noise -> _thr2pwm -> rpm (246-262)
    const Real rp = Real(0.2685) * clampr_(pwm, Real(20000), Real(65535)) + Real(4070.3);
    const Real thr = qmirror(Real(3.16e-10) * rp * rp);
    const Real t = maxr_(thr + noise_m, Real(0));
    const Real mp = clampr_(F32 ? (hsqrt_(t * Real(1.0 / 3.16e-10)) - Real(4070.3)) * Real(1.0 / 0.2685)
                                : divc_(sqrt_(divc_(t, Real(3.16e-10))) - Real(4070.3), Real(0.2685)),
                            Real(20000), Real(65535));
    const Real rnew = Real(0.2685) * mp + Real(4070.3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        d.prev[k] = d.rpm[k];
        d.rpm[k] = qbc(rnew, k);
    }
    CP_MARK(m3);
    CP_ADD(3, m3 - m0);   // whole wrapper (pwm / rpm chain = slot 3 - 1 - 2)
}

// the block's LDS copy of its drones' env tracks, [field][drone] (owner lane l -> drone l / 4)
template <typename Real>
struct TrackSrcQ {
    const Real* lds;
    int qd;
    __device__ __forceinline__ Real operator()(int field) const { return lds[(field - RF_GATE) * kQuadDrones + qd]; }
    __device__ __forceinline__ TrackSrcQ lane(int l, int, int, int) const { return TrackSrcQ{lds, l >> 2}; }
};

__device__ __forceinline__ uint32_t quad_or(uint32_t v) {   // OR over the quad (DPP quad_perm [1,0,3,2], [2,3,0,1])
    v |= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xb1, 0xf, 0xf, false));
    v |= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x4e, 0xf, 0xf, false));
    return v;
}

// track_bounds with the track dealt over the quad: lane ql tests gate ql and obstacle ql (same
// per-part arithmetic), the bit masks are OR-ed over the quad
// The support-bound refinement of part_bounds_refined, pooled over the block: each (lane, part) pair
// whose centre bounds straddle a cut is queued in LDS and the block's 64 lanes work the queue, so a
// wave runs ceil(jobs / 64) refinements (usually one) instead of one per part index that any lane
// needs (up to 7, ~330 instructions each in fp64).  The pool holds every lane's part-frame inputs
// (gate-frame drone centre / axis, obstacle offsets, gate type) and the refined bounds per (lane,
// part); the results are the inline form's, operation for operation.
template <typename Real>
struct RefinePool {
    Real in[12][kRaceBlock];   // lg.xyz, ag.xyz (gate frame), dp.xyz, ax.xyz (obstacle frame) per lane
    Real lo[kRaceBlock * 7], up[kRaceBlock * 7];
    uint16_t job[kRaceBlock * 7];
    int low[kRaceBlock];
};

template <typename Real>
__device__ __forceinline__ void refine_part(const RaceConst<Real>& C, int k, int low, V3<Real> lg, V3<Real> ag,
                                            V3<Real> dp, V3<Real> ax, Real& lo2, Real& up2) {
    V3<Real> off, h;
    Real r;
    int cyl;
    if (k < kGateParts) {
        M3<Real> R;
        gate_part(k, low, off, R, h, r, cyl);
        part_bounds_refined(mulT(R, lg - off), mulT(R, ag), h, r, cyl, C.coll_r, C.coll_hh, lo2, up2);
    } else {
        obst_part(k - kGateParts, off, h, r, cyl);
        part_bounds_refined(dp - off, ax, h, r, cyl, C.coll_r, C.coll_hh, lo2, up2);
    }
}

// pool: nullptr refines inline (the auto-reset's divergent lanes); otherwise every lane of the block
// must call it (two barriers)
template <typename Real, class TS>
__device__ __forceinline__ void track_bounds_q4(const RaceConst<Real>& C, const TS& T, const Shape<Real>& ds,
                                                Real cut, Real ccut, int ql, bool want_contact, uint32_t& gin,
                                                uint32_t& oin, uint32_t& amb, uint32_t& camb_all, bool& ccert,
                                                RefinePool<Real>* pool = nullptr) {
    const Real tol = Real(1e-5);
    const Real dr = hsqrt_(ds.r * ds.r + ds.h.z * ds.h.z);
    const V3<Real> p = ds.c, ax = col2(ds.R);
    amb = 0; camb_all = 0;
    gin = 0; oin = 0;
    ccert = false;
    const int g = ql, o = ql;
    const bool has_g = g < C.num_gates, has_o = o < C.num_obstacles;
    // centre bounds of this lane's gate (parts 0-4) and obstacle (parts 5-6)
    Real plo[7], pup[7];
    uint32_t need = 0;
    V3<Real> lg = v3(Real(0), Real(0), Real(0)), ag = lg, dp = lg;
    int low = 0;
    if (has_g) {
        const V3<Real> dg = p - v3(T(RF_GATE + 4 * g), T(RF_GATE + 4 * g + 1), T(RF_GATE + 4 * g + 2));
        Real sn, cs;
        sincos_f_(T(RF_GATE + 4 * g + 3), &sn, &cs);
        lg = v3(cs * dg.x + sn * dg.y, -sn * dg.x + cs * dg.y, dg.z);
        ag = v3(cs * ax.x + sn * ax.y, -sn * ax.x + cs * ax.y, ax.z);
        low = C.gate_type[g] > 0;
    }
    if (has_o) dp = p - v3(T(RF_OBST + 3 * o), T(RF_OBST + 3 * o + 1), T(RF_OBST + 3 * o + 2));
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        V3<Real> off, h, lp;
        Real r;
        int cyl;
        if (k < kGateParts) {
            M3<Real> R;
            gate_part(k, low, off, R, h, r, cyl);
            lp = mulT(R, lg - off);
        } else {
            obst_part(k - kGateParts, off, h, r, cyl);
            lp = dp - off;
        }
        const Real pd = point_part_dist(lp, h, r, cyl);
        plo[k] = pd - dr;
        pup[k] = pd;
        const bool live = k < kGateParts ? has_g : has_o;
        if (live && C.refine && ((!(pd < cut - tol) && plo[k] < cut + tol) || (want_contact && plo[k] < ccut + tol)))
            need |= 1u << k;
    }
    if (pool == nullptr) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            if ((need >> k) & 1u) {
                Real lo2, up2;
                refine_part(C, k, low, lg, ag, dp, ax, lo2, up2);
                plo[k] = fmaxr_(plo[k], lo2);
                pup[k] = up2 < pup[k] ? up2 : pup[k];
            }
        }
    } else {
        const int tl = threadIdx.x;
        const Real iv[12] = {lg.x, lg.y, lg.z, ag.x, ag.y, ag.z, dp.x, dp.y, dp.z, ax.x, ax.y, ax.z};
#pragma unroll
        for (int i = 0; i < 12; ++i) pool->in[i][tl] = iv[i];
        pool->low[tl] = low;
        const int n = __popc(need);
        int incl = n;   // inclusive scan of the queue lengths
#pragma unroll
        for (int s = 1; s < kRaceBlock; s <<= 1) {
            const int t = __shfl_up(incl, s, kRaceBlock);
            if (tl >= s) incl += t;
        }
        const int total = __shfl(incl, kRaceBlock - 1, kRaceBlock);
        int pos = incl - n;
        for (uint32_t m = need; m; m &= m - 1) pool->job[pos++] = uint16_t((tl << 3) | __builtin_ctz(m));
        __syncthreads();
        for (int base = 0; base < total; base += kRaceBlock) {
            const int j = base + tl;
            if (j < total) {
                const int job = pool->job[j], L = job >> 3, k = job & 7;
                const V3<Real> jl = v3(pool->in[0][L], pool->in[1][L], pool->in[2][L]);
                const V3<Real> ja = v3(pool->in[3][L], pool->in[4][L], pool->in[5][L]);
                const V3<Real> jd = v3(pool->in[6][L], pool->in[7][L], pool->in[8][L]);
                const V3<Real> jx = v3(pool->in[9][L], pool->in[10][L], pool->in[11][L]);
                Real lo2, up2;
                refine_part(C, k, pool->low[L], jl, ja, jd, jx, lo2, up2);
                pool->lo[L * 7 + k] = lo2;
                pool->up[L * 7 + k] = up2;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            if ((need >> k) & 1u) {
                const Real lo2 = pool->lo[tl * 7 + k], up2 = pool->up[tl * 7 + k];
                plo[k] = fmaxr_(plo[k], lo2);
                pup[k] = up2 < pup[k] ? up2 : pup[k];
            }
        }
    }
    // classification (race_kernel.h track_bounds): in the cut / ambiguous / contact certain or open
    if (has_g) {
        bool in = false;
        uint32_t gamb = 0, camb = 0;
#pragma unroll
        for (int k = 0; k < kGateParts; ++k) {
            in |= pup[k] < cut - tol;
            if (plo[k] < cut + tol) gamb |= 1u << k;
            if (want_contact && plo[k] < ccut + tol) {   // centre inside the part: contact (race_kernel.h)
                if (pup[k] == Real(0)) ccert = true;
                else camb |= 1u << k;
            }
        }
        if (in) gin |= 1u << g;
        amb |= ((in ? 0u : gamb) | camb) << (g * kGateParts);
        camb_all |= camb << (g * kGateParts);
    }
    if (has_o) {
        bool in = false;
        uint32_t gamb = 0, camb = 0;
#pragma unroll
        for (int k = 0; k < kObstParts; ++k) {
            in |= pup[kGateParts + k] < cut - tol;
            if (plo[kGateParts + k] < cut + tol) gamb |= 1u << k;
            if (want_contact && plo[kGateParts + k] < ccut + tol) {
                if (pup[kGateParts + k] == Real(0)) ccert = true;
                else camb |= 1u << k;
            }
        }
        if (in) oin |= 1u << o;
        amb |= ((in ? 0u : gamb) | camb) << (kObstBit0 + o * kObstParts);
        camb_all |= camb << (kObstBit0 + o * kObstParts);
    }
    gin = quad_or(gin); oin = quad_or(oin); amb = quad_or(amb); camb_all = quad_or(camb_all);
    ccert = quad_or(ccert ? 1u : 0u) != 0;
}


// ---- auto-reset of a done drone by its quad ----
// race_reset_lane's arithmetic (MultiRaceAviary.reset 127-167, _addObstacles 347-403, _drone_init
// 407-467) with the work dealt over the quad: lane ql draws gate ql, obstacle ql and drone draw ql;
// the track reaches every lane by DPP broadcasts and stays in registers (the one-lane reset reads it
// back from HBM after storing it); lane ql tests gate ql / obstacle ql at the nominal pose.  A wave
// that resets an env waits for it after its sub-steps, and the kernel for its slowest wave.

// this lane's own gate ql / obstacle ql, addressed like the track fields (the bounds pass and the
// part shapes of lane ql only ask for gate ql and obstacle ql)
template <typename Real>
struct TrackOne {
    Real g[4], o[3];
    int ql;
    __device__ __forceinline__ Real operator()(int field) const {
        if (field < RF_OBST) {
            const int c = field - RF_GATE - 4 * ql;
            return c == 0 ? g[0] : c == 1 ? g[1] : c == 2 ? g[2] : g[3];
        }
        const int c = field - RF_OBST - 3 * ql;
        return c == 0 ? o[0] : c == 1 ? o[1] : o[2];
    }
};
// the whole track in registers (field indices fold to constants in the unrolled obs-row loops)
template <typename Real>
struct TrackRegs {
    Real v[kTrackFields];
    __device__ __forceinline__ Real operator()(int field) const { return v[field - RF_GATE]; }
};

// Where a reset's results go: the drone slot's state in HBM (the quad resetting a done env after its
// step).  A sink, so a staging variant can take the same values (a reset helper wave computing every
// drone's next episode into LDS during the sub-steps was measured and dropped: DESIGN.md §3.2.1).
template <typename Real>
struct ResetToHBM {
    const RaceArgs<Real>* a;
    __device__ __forceinline__ void track(bool active, size_t EN, size_t slot, int ql, const TrackOne<Real>& own) const {
        if (!active) return;   // the quad stores the drone slot's replicated track, a gate and an obstacle per lane
#pragma unroll
        for (int k = 0; k < 4; ++k) st(a->f, RF_GATE + 4 * ql + k, EN, slot, own.g[k]);
#pragma unroll
        for (int k = 0; k < 3; ++k) st(a->f, RF_OBST + 3 * ql + k, EN, slot, own.o[k]);
    }
    __device__ __forceinline__ void wrapper(size_t EN, size_t slot, const Real tgt[3], const Real prv[3]) const {
        for (int k = 0; k < 3; ++k) {
            st(a->f, RF_WR_TARGET + k, EN, slot, tgt[k]);
            st(a->f, RF_WR_PREV + k, EN, slot, prv[k]);
        }
    }
    // the reset drone's state (store_drone(params = true) of the RDrone race_reset_lane builds), field
    // by field from its values: an RDrone aggregate here went to scratch memory (~500 B per lane stored
    // and reloaded on the resetting wave)
    __device__ __forceinline__ void drone(size_t EN, size_t slot, V3<Real> pos, Q4<Real> q, V3<Real> vel, V3<Real> w,
                                          V3<Real> angv, V3<Real> kpos, V3<Real> prpy, Real mass, const Real inertia[3],
                                          int episode) const {
        Real* f = a->f;
#define S_(k, v) st(f, (k), EN, slot, Real(v))
        S_(RF_POS, pos.x); S_(RF_POS + 1, pos.y); S_(RF_POS + 2, pos.z);
        S_(RF_QUAT, q.x); S_(RF_QUAT + 1, q.y); S_(RF_QUAT + 2, q.z); S_(RF_QUAT + 3, q.w);
        S_(RF_VEL, vel.x); S_(RF_VEL + 1, vel.y); S_(RF_VEL + 2, vel.z);
        S_(RF_OMEGA, w.x); S_(RF_OMEGA + 1, w.y); S_(RF_OMEGA + 2, w.z);
        S_(RF_ANGV, angv.x); S_(RF_ANGV + 1, angv.y); S_(RF_ANGV + 2, angv.z);
        S_(RF_LINK_QUAT, q.x); S_(RF_LINK_QUAT + 1, q.y); S_(RF_LINK_QUAT + 2, q.z); S_(RF_LINK_QUAT + 3, q.w);
        S_(RF_LINK_POS, pos.x); S_(RF_LINK_POS + 1, pos.y); S_(RF_LINK_POS + 2, pos.z);
        S_(RF_KIN_POS, kpos.x); S_(RF_KIN_POS + 1, kpos.y); S_(RF_KIN_POS + 2, kpos.z);
#pragma unroll
        for (int k = 0; k < 4; ++k) { S_(RF_RPM + k, 0); S_(RF_PREV_RPM + k, 0); S_(RF_CTL + k, 0); }
        const Real pr[3] = {prpy.x, prpy.y, prpy.z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            S_(RF_PREV_RPY + k, pr[k]); S_(RF_PREV_VEL + k, 0);
            S_(RF_LPF_D1 + k, 0); S_(RF_LPF_D2 + k, 0);
            S_(RF_I_ERR + k, 0); S_(RF_I_ERR_M + k, 0);
        }
        const Real nan = Real(__builtin_nanf(""));   // D-term memory: no D term on the first call
        S_(RF_PREV_OMEGA_ROLL, nan); S_(RF_PREV_OMEGA_PITCH, nan);
        S_(RF_PREV_SP_ROLL, 0); S_(RF_PREV_SP_PITCH, 0);
        S_(RF_MASS, mass);
        S_(RF_INERTIA, inertia[0]); S_(RF_INERTIA + 1, inertia[1]); S_(RF_INERTIA + 2, inertia[2]);
#undef S_
        int32_t* ist = a->ist;
        ist[RI_TICK * EN + slot] = 0; ist[RI_LAST_ATT * EN + slot] = 0;
        ist[RI_LAST_POS * EN + slot] = 0; ist[RI_TUMBLE * EN + slot] = 0;
        ist[RI_GATE * EN + slot] = 0; ist[RI_FLAGS * EN + slot] = 0;
        ist[RI_STEP * EN + slot] = 0;
        ist[RI_EPISODE * EN + slot] = episode + 1;
        ist[RI_WR_GATE * EN + slot] = 0;
    }
};

#if defined(ADRP_RACE_TIMING) && defined(ADRP_RESET_PHASES)
// measurement-only (tools/race_phases.py with a -DADRP_RESET_PHASES timing build): s_memtime marks
// inside the reset, reported in the kernel's 8 per-block phase slots instead of the step phases
__shared__ uint64_t g_reset_mark[9];   // per workgroup (LDS): blocks do not race
#define RESET_MARK(k) g_reset_mark[k] = __builtin_amdgcn_s_memtime()
#else
#define RESET_MARK(k)
#endif

template <typename Real, int G, class Sink>
__device__ __forceinline__ void race_reset_q4(const RaceArgs<Real>& a, const RaceConst<Real>& C, int e, int dn, int ql,
                                              bool active, size_t EN, size_t slot, int episode, float* obs_row,
                                              const Sink& out) {
    RESET_MARK(0);
    const bool owner = active && ql == 0;
    const uint64_t gid = uint64_t(a.env_offset + e);
    const uint32_t ep = uint32_t(episode);
    TrackOne<Real> own;
    own.ql = ql;
    {   // gate ql, obstacle ql of the next track
        const int g = ql;
        Real gx = C.gate_nom[g][0], gy = C.gate_nom[g][1], gyaw = C.gate_nom[g][3];
        if (C.random_gates && g < C.num_gates) {
            const U4 u = draw(a.seed, gid, ep, TAG_RACE_TRACK, uint32_t(g));
            const Real lo = C.gate_off[0], hi = C.gate_off[1];
            gx += lo + (hi - lo) * Real(u01(u.a));
            gy += lo + (hi - lo) * Real(u01(u.b));
            gyaw += lo + (hi - lo) * Real(u01(u.c));
        }
        own.g[0] = gx; own.g[1] = gy; own.g[2] = C.gate_nom[g][2]; own.g[3] = gyaw;
        const int o = ql;
        Real ox = C.obst_nom[o][0], oy = C.obst_nom[o][1];
        if (C.random_gates && o < C.num_obstacles) {
            const U4 u = draw(a.seed, gid, ep, TAG_RACE_TRACK, uint32_t(4 + o));
            const Real lo = C.obst_off[0], hi = C.obst_off[1];
            ox += lo + (hi - lo) * Real(u01(u.a));
            oy += lo + (hi - lo) * Real(u01(u.b));
        }
        own.o[0] = ox; own.o[1] = oy; own.o[2] = C.obst_nom[o][2];
        RESET_MARK(1);
        out.track(active, EN, slot, ql, own);
    }
    RESET_MARK(2);
    TrackRegs<Real> T;
#pragma unroll
    for (int g = 0; g < ADRP_MAX_GATES; ++g)
#pragma unroll
        for (int k = 0; k < 4; ++k) T.v[4 * g + k] = qbc(own.g[k], g);
#pragma unroll
    for (int o = 0; o < ADRP_MAX_OBSTACLES; ++o)
#pragma unroll
        for (int k = 0; k < 3; ++k) T.v[RF_OBST - RF_GATE + 3 * o + k] = qbc(own.o[k], o);
    // initial obs at the nominal (loadURDF) pose, at rest; lane ql tests gate ql / obstacle ql
    const V3<Real> npos = v3(C.init_pos[dn][0], C.init_pos[dn][1], C.init_pos[dn][2]);
    const Q4<Real> nq = nominal_q(C, dn);
    const Shape<Real> ds = drone_shape(C, npos, nq);
    RESET_MARK(3);
    uint32_t gin, oin, amb, camb_all;
    bool ccert;
#ifdef ADRP_EXP_RESET_NOQ
    gin = oin = amb = camb_all = 0; ccert = false;
#else
    track_bounds_q4(C, own, ds, Real(0.45), Real(0), ql, false, gin, oin, amb, camb_all, ccert);
#endif
    uint32_t mine = amb & ((0x1fu << (kGateParts * ql)) | (0x3u << (kObstBit0 + kObstParts * ql)));
    uint32_t g2 = 0, o2 = 0;
    while (mine) {   // this lane's undecided parts (track_query)
        const int b = __builtin_ctz(mine);
        mine &= mine - 1;
        if (gjk_within(ds, track_part_shape(C, own, b), Real(0.45))) {
            if (b < kObstBit0) g2 |= 1u << (b / kGateParts);
            else o2 |= 1u << ((b - kObstBit0) / kObstParts);
        }
    }
    gin |= quad_or(g2);
    oin |= quad_or(o2);
    RESET_MARK(4);
    Real row0[15];
    const V3<Real> zero = v3(Real(0), Real(0), Real(0));
#ifdef ADRP_EXP_RESET_NOROW
    for (int k = 0; k < 15; ++k) row0[k] = T.v[k];
#else
    race_obs_row_rpy(C, T, npos, nominal_rpy(C, dn), zero, zero, 0, obs_row, owner, row0, gin, oin);
#endif
    RESET_MARK(5);
    // the nominal Euler angles (RaceConst::nom_rpy, race_const_init_kernel)
    const V3<Real> nrpy = nominal_rpy(C, dn);
    if (C.compete && owner) {   // other drones' nominal pos + rpy
        int idx = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (k < C.N && k != dn) {
                float* p = obs_row + 49 + 6 * idx;
                p[0] = C.init_pos[k][0]; p[1] = C.init_pos[k][1]; p[2] = C.init_pos[k][2];
                p[3] = C.nom_rpy[k][0]; p[4] = C.nom_rpy[k][1]; p[5] = C.nom_rpy[k][2];
                ++idx;
            }
        }
    }
    RESET_MARK(6);
    // _drone_init draws: lane 0 position offsets, lane 1 rotation offsets, lane 2 mass / inertia
    // (the uniforms travel; the ranges are applied as race_reset_lane does)
    const uint32_t dtag = TAG_RACE_DRONE | uint32_t(dn);
    Real u[4] = {Real(0), Real(0), Real(0), Real(0)};
    if (ql < 2 ? C.random_state != 0 : (ql == 2 && C.random_inertia != 0)) {
        const U4 w = draw(a.seed, gid, ep, dtag, uint32_t(ql));
        u[0] = Real(u01(w.a)); u[1] = Real(u01(w.b)); u[2] = Real(u01(w.c)); u[3] = Real(u01(w.d));
    }
    Real uq[3][4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) uq[j][k] = qbc(u[k], j);
    RESET_MARK(7);
    if (!owner) return;
    {   // RewardWrapper.reset: current_target = obs[0, 12:15], previous_pos = obs[0, :3]
        Real tgt[3], prv[3];
        for (int k = 0; k < 3; ++k) {
            tgt[k] = dn == 0 && C.num_gates > 0 ? row0[3 + k] : Real(0);
            prv[k] = dn == 0 ? row0[k] : Real(0);
        }
        out.wrapper(EN, slot, tgt, prv);
    }
    Real mass = C.race_mass;
    Real inertia[3] = {C.race_inertia[0], C.race_inertia[1], C.race_inertia[2]};
    if (C.random_inertia) {
        Real v[4] = {mass, inertia[0], inertia[1], inertia[2]};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const Real lo = C.inertia_off[k][0], hi = C.inertia_off[k][1];
            v[k] = clampr_(v[k] + lo + (hi - lo) * uq[2][k], Real(0), Real(100));
        }
        mass = v[0]; inertia[0] = v[1]; inertia[1] = v[2]; inertia[2] = v[3];
    }
    Real po[3] = {0, 0, 0}, ro[3] = {0, 0, 0};
    if (C.random_state) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            po[k] = C.pos_off[k][0] + (C.pos_off[k][1] - C.pos_off[k][0]) * uq[0][k];
            ro[k] = C.rot_off[k][0] + (C.rot_off[k][1] - C.rot_off[k][0]) * uq[1][k];
        }
    }
    const V3<Real> pos = v3(npos.x + po[0], npos.y + po[1], npos.z + po[2]);
    const Q4<Real> q = quat_from_euler_fast(C.init_rpy[dn][0] + ro[0], C.init_rpy[dn][1] + ro[1], C.init_rpy[dn][2] + ro[2]);
    const V3<Real> w0 = v3(C.init_pqr[dn][0], C.init_pqr[dn][1], C.init_pqr[dn][2]);
    const V3<Real> w = C.physics == ADRP_PHYS_DYN ? v3(Real(0), Real(0), Real(0)) : w0;   // rpy_rates zeroed by _housekeeping
    const V3<Real> kpos = C.physics == ADRP_PHYS_PYB ? npos : pos;   // self.pos: nominal until the first read
    out.drone(EN, slot, pos, q, v3(C.init_vel[dn][0], C.init_vel[dn][1], C.init_vel[dn][2]), w, w0, kpos, nrpy, mass,
              inertia, episode);
    RESET_MARK(8);
}

// Next-reset images.  Everything an auto-reset writes (the drone slot's 98 state fields and 9 ints,
// its reset obs row) is a function of (seed, env, episode) and the constant block only: the track and
// drone-init draws are keyed by the episode, the range tests and the obs row are taken at the nominal
// pose.  race_refill_q4 computes it ahead, with race_reset_q4 itself (the same code, so the same bits),
// into image buffers tagged with the episode it is for; the step kernel's auto-reset of an env whose
// image is for its current episode then copies it (loads and stores, no arithmetic) instead of running
// the reset's ~5 us chain on the wave that the whole launch waits for.  An env whose image is not ready
// (reset twice between refills, or images off) resets inline as before.
// n floats from LDS to global memory by the wave's 64 lanes (all reads, then the stores)
template <int MAXN>
__device__ __forceinline__ void wave_copy_rows(const float* src, float* dst, int n, int tl) {
    constexpr int K = (MAXN + kRaceBlock - 1) / kRaceBlock;
    float v[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const int k = tl + kRaceBlock * i;
        v[i] = k < n ? src[k] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const int k = tl + kRaceBlock * i;
        if (k < n) dst[k] = v[i];
    }
}

// one env's image (its N drone slots from slot0: 98 fields and 9 ints each, and its N obs rows) into
// the state and the block's LDS rows, by the wave's 64 lanes: every load in flight, then the stores
template <typename Real, int G, int ROWF>
__device__ __forceinline__ void reset_from_image(const RaceArgs<Real>& a, size_t EN, size_t slot0, int N, float* rows,
                                                 int D, int tl) {
    constexpr int KF = (RF_N * G + kRaceBlock - 1) / kRaceBlock, KI = (RI_N * G + kRaceBlock - 1) / kRaceBlock;
    constexpr int KR = (ROWF * G + kRaceBlock - 1) / kRaceBlock;
    const int nf = RF_N * N, ni = RI_N * N, nr = N * D;
    Real v[KF];
    int32_t iv[KI];
    float rv[KR];
    size_t fo[KF], io[KI];
#pragma unroll
    for (int i = 0; i < KF; ++i) {   // field k of drone slot0 + j: idx = k * N + j
        const int idx = tl + kRaceBlock * i;
        const int k = idx / N, j = idx - k * N;
        fo[i] = size_t(k) * EN + slot0 + j;
        v[i] = idx < nf ? a.img_f[fo[i]] : Real(0);
    }
#pragma unroll
    for (int i = 0; i < KI; ++i) {
        const int idx = tl + kRaceBlock * i;
        const int k = idx / N, j = idx - k * N;
        io[i] = size_t(k) * EN + slot0 + j;
        iv[i] = idx < ni ? a.img_i[io[i]] : 0;
    }
    const float* src = a.img_row + slot0 * size_t(D);
#pragma unroll
    for (int i = 0; i < KR; ++i) {
        const int k = tl + kRaceBlock * i;
        rv[i] = k < nr ? src[k] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < KF; ++i)
        if (tl + kRaceBlock * i < nf) a.f[fo[i]] = v[i];
#pragma unroll
    for (int i = 0; i < KI; ++i)
        if (tl + kRaceBlock * i < ni) a.ist[io[i]] = iv[i];
#pragma unroll
    for (int i = 0; i < KR; ++i) {
        const int k = tl + kRaceBlock * i;
        if (k < nr) rows[k] = rv[i];
    }
}

// The refill: the step's lane layout (a quad per drone, 4G lanes per env); an env whose image is not
// for its current episode gets one.  Waves with nothing to refill end after two loads.
// The constant block (RaceConst, ~2 KB) into LDS in two halves: load() issues every 16-byte chunk's
// load before any store and store() writes them later, so the copy costs one memory latency, which
// the step kernel overlaps with its state loads.  (The plain strided loop compiled to a load, a
// vmcnt(0) wait and a store per 256 bytes: nine serialised misses at kernel start, where the
// kernel-start acquire has just invalidated L2.)
template <class T>
struct LdsCopy {
    static constexpr int NB = int(sizeof(T)), N4 = NB / 16, R = (NB % 16) / 4;
    static constexpr int IT = (N4 + kRaceBlock - 1) / kRaceBlock;
    uint4 v[IT];
    uint32_t r;
    __device__ __forceinline__ void load(const T* g, int tl) {
        const uint4* s4 = reinterpret_cast<const uint4*>(g);   // (the device allocation's start: aligned)
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const int i = tl + j * kRaceBlock;
            if (i < N4) v[j] = s4[i];
        }
        r = 0;
        if (R > 0 && tl < R) r = reinterpret_cast<const uint32_t*>(g)[N4 * 4 + tl];
    }
    __device__ __forceinline__ void store(T* lds, int tl) const {
        uint4* d4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const int i = tl + j * kRaceBlock;
            if (i < N4) d4[i] = v[j];
        }
        if (R > 0 && tl < R) reinterpret_cast<uint32_t*>(lds)[N4 * 4 + tl] = r;
    }
};

template <typename Real, int G>
__global__ void __launch_bounds__(kRaceBlock) race_refill_q4(RaceArgs<Real> a) {
    const int tl = threadIdx.x;
    const int ql = tl & 3, qd = tl >> 2;
    const int dl = blockIdx.x * kQuadDrones + qd;
    const RaceConst<Real>& CG = *a.c;
    const int N = CG.N;
    const int e_raw = dl / G, d_raw = dl % G;
    const bool active = e_raw < a.E && d_raw < N;
    const int e = e_raw < a.E ? e_raw : a.E - 1;
    const int dn = d_raw < N ? d_raw : 0;
    const size_t EN = size_t(a.E) * N;
    const size_t slot = size_t(e) * N + dn;
    const int episode = a.ist[RI_EPISODE * EN + slot];
    const bool need = a.img_ep[e] != episode;   // env-uniform: the env's drones share the episode
    if (!__any(need)) return;                   // wave-uniform exit
    __shared__ __attribute__((aligned(16))) RaceConst<Real> c_lds;
    __shared__ float rows[kQuadDrones * (49 + 6 * (G - 1))];
    // (the wave that reaches here is the whole block: kRaceBlock = one wave)
    {
        LdsCopy<RaceConst<Real>> cc;
        cc.load(a.c, tl);
        cc.store(&c_lds, tl);
    }
    __syncthreads();
    const RaceConst<Real>& C = c_lds;
    RaceArgs<Real> b = a;   // the reset's sink writes the image instead of the state
    b.f = a.img_f;
    b.ist = a.img_i;
    float* row = rows + qd * C.D;
    if (need) race_reset_q4<Real, G>(b, C, e, dn, ql, active, EN, slot, episode, row, ResetToHBM<Real>{&b});
    __syncthreads();   // the owner lane's row
    if (need && active) {   // the quad's lanes copy the row out
        float* dst = a.img_row + slot * size_t(C.D);
        for (int k = ql; k < C.D; k += 4) dst[k] = row[k];
        if (ql == 0 && dn == 0) a.img_ep[e] = episode;
    }
}

// the sub-step draws of drone qd's sub-steps s = ql, ql + 4, ... into the LDS table [s][7][drone]:
// fp32 the 3 force components and the 4 motor noises; fp64 the 3 force uniforms (exact in float;
// the force is formed in Real at use) and the 4 noise samples (normal_pair_f, float, scaled at use)
template <typename Real>
__device__ __forceinline__ void quad_draws(const RaceConst<Real>& H, float* pre_draws, uint64_t seed, uint64_t gid,
                                           uint32_t ep, int dn, int sc0, int ql, int qd, int S) {
    for (int s = ql; s < S; s += 4) {
        float* dst = pre_draws + s * 7 * kQuadDrones + qd;
        if constexpr (sizeof(Real) == 4) {
            Real fd[3], nz[4];
            race_substep_draws(H, seed, gid, ep, dn, uint32_t(sc0 + s), fd, nz);
#pragma unroll
            for (int k = 0; k < 3; ++k) dst[k * kQuadDrones] = fd[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[(3 + k) * kQuadDrones] = nz[k];
        } else {
            const U4 u = draw(seed, gid, ep, TAG_RACE_DIST | uint32_t(dn), uint32_t(sc0 + s));
            dst[0] = u01r<float>(u.a); dst[kQuadDrones] = u01r<float>(u.b); dst[2 * kQuadDrones] = u01r<float>(u.c);
            const U4 v = draw(seed, gid, ep, TAG_RACE_NOISE | uint32_t(dn), uint32_t(sc0 + s));
            float z[4];   // race_noise_draws' fp64 samples (before the std scale): the oracle's, bit for bit
            normal_pair_f(v.a, v.b, &z[0], &z[1]);
            normal_pair_f(v.c, v.d, &z[2], &z[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[(3 + k) * kQuadDrones] = z[k];
        }
    }
}

// Block = 64 lanes = 16 drones (kQuadDrones); one wave.  DRAWS: the disturbance draws of the
// step's S <= kRacePreS sub-steps go through LDS (disturbances on); else none are needed, or (S
// larger) each lane draws in the loop.
template <typename Real, int PH, int G, bool DRAWS, bool DEF>
__global__ void __launch_bounds__(kRaceBlock) race_step_q4(RaceArgs<Real> a) {
    constexpr bool F32 = sizeof(Real) == 4;
    RACE_MARK(t0);
    constexpr int kRowF = 49 + 6 * (G - 1);   // widest obs row of this G
    // the sub-step draw table is dead after the loop: the GJK job pool reuses its LDS
    constexpr size_t kDrawBytes = DRAWS ? size_t(kRacePreS) * 7 * kQuadDrones * sizeof(float) : 16;
    constexpr size_t kPost = sizeof(TrackJobs) > sizeof(RefinePool<Real>) ? sizeof(TrackJobs) : sizeof(RefinePool<Real>);
    constexpr size_t kScratchBytes = kDrawBytes > kPost ? kDrawBytes : kPost;
    __shared__ __attribute__((aligned(16))) unsigned char scratch_lds[kScratchBytes];
    float* const pre_draws = reinterpret_cast<float*>(scratch_lds);
    TrackJobs& tjobs = *reinterpret_cast<TrackJobs*>(scratch_lds);
    RefinePool<Real>* const rpool = reinterpret_cast<RefinePool<Real>*>(scratch_lds);   // (bounds, then tjobs)
    __shared__ Real trk_lds[kTrackFields * kQuadDrones];                   // [field][drone]
    __shared__ float4 rows4[kQuadDrones * kRowF / 4];
    // the constant block in LDS: the post-loop phases and the auto-reset index it by drone / gate /
    // obstacle (lane-varying), which from global memory is a dependent miss per table
    __shared__ __attribute__((aligned(16))) RaceConst<Real> c_lds;
    __shared__ double exp_lds[32];
    constexpr bool kDwF64 = !F32 && (PH == ADRP_PHYS_PYB_DW || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    // the constant block and the exp table: loads issued here, LDS stores after the state loads
    // (before the barrier ahead of the sub-step loop); C is read only after the loop
    LdsCopy<RaceConst<Real>> ccopy;
    ccopy.load(a.c, int(threadIdx.x));
    double exp_v = 0.0;
    if constexpr (kDwF64) {
        if (threadIdx.x < 32) exp_v = f64::kExp2Tab32[threadIdx.x];
    }
    const RaceConst<Real>& CG = *a.c;   // uniform fields: scalar loads (SGPRs)
    const RaceConst<Real>& C = c_lds;   // after the loop
    const int tl = threadIdx.x;
    const int ql = tl & 3, qd = tl >> 2;                 // quad lane, drone within the block
    const int cax = ql < 3 ? ql : 2;                     // this lane's Euler axis
    RaceConst<Real> H;
    H.S = CG.S; H.link_lag = CG.link_lag; H.disturbances = CG.disturbances;
#pragma unroll
    for (int i = 0; i < 3; ++i) { H.dist_lo[i] = CG.dist_lo[i]; H.dist_hi[i] = CG.dist_hi[i]; }
    H.noise_std = CG.noise_std;
    if constexpr (DEF) {   // the reference's race drone: the physical constants as literals
        race_cf2x_phys(H);
    } else {
        H.dt = CG.dt; H.gravity = CG.gravity; H.kf = CG.kf; H.km = CG.km;
#pragma unroll
        for (int i = 0; i < 4; ++i) { H.px[i] = CG.px[i]; H.py[i] = CG.py[i]; H.pz[i] = CG.pz[i]; }
        H.gnd_kf = CG.gnd_kf; H.prop_r4 = CG.prop_r4; H.gnd_clip = CG.gnd_clip;
#pragma unroll
        for (int i = 0; i < 3; ++i) { H.drag[i] = CG.drag[i]; H.dyn_i[i] = CG.dyn_i[i]; H.dyn_inv_i[i] = CG.dyn_inv_i[i]; }
        H.dw1 = CG.dw1; H.dw2 = CG.dw2; H.dw3 = CG.dw3; H.prop_r = CG.prop_r;
        H.dyn_mass = CG.dyn_mass; H.dyn_inv_mass = CG.dyn_inv_mass; H.dyn_arm = CG.dyn_arm;
        H.coll_hh = CG.coll_hh; H.coll_r = CG.coll_r; H.coll_zoff = CG.coll_zoff; H.ang_max = CG.ang_max;
    }
    const int lb = xcd_block(blockIdx.x, gridDim.x);     // logical block (XCD-aware order)
    const int dl = lb * kQuadDrones + qd;                // drone lane of the one-lane layout
    const int e_raw = dl / G, d_raw = dl % G;
    const int N = CG.N;
    const bool active = e_raw < a.E && d_raw < N;
    const bool owner = active && ql == 0;
    const int e = e_raw < a.E ? e_raw : a.E - 1;
    const int dn = d_raw < N ? d_raw : 0;
    const size_t EN = size_t(a.E) * N;
    const size_t slot = size_t(e) * N + dn;
    const uint64_t gid = uint64_t(a.env_offset + e);
    // the draw keys and the tick first: the draws wait for these loads only, and the tick-schedule
    // window (a second, dependent load) is issued before the bulk of the state
    const int sc0 = a.ist[RI_STEP * EN + slot];
    const int episode = a.ist[RI_EPISODE * EN + slot];
    const uint32_t ep = uint32_t(episode - 1);
    const int tick0 = a.ist[RI_TICK * EN + slot];
    uint32_t att0, pos0;
    tick_window(a.ticks, tick0, att0, pos0);
    // the env's actual track: 7 of its 28 fields per lane, into LDS for the post-loop queries (written
    // before the loop, so no register holds them through the sub-steps)
#pragma unroll
    for (int i = 0; i < (kTrackFields + 3) / 4; ++i) {
        const int k = ql + 4 * i;
        if (k < kTrackFields) trk_lds[k * kQuadDrones + qd] = ld(a.f, RF_GATE + k, EN, slot);
    }
    RDrone<Real> d;
    load_drone<Real, false, PH == ADRP_PHYS_DYN>(a, EN, slot, d);   // (angv: only DYN changes it)
    d.tick_base = tick0;
    d.att_bits = att0;
    d.pos_bits = pos0;
    const float4 av = reinterpret_cast<const float4*>(a.act)[slot];
    const float sp[3] = {av.x, av.y, av.z};
    float xc_x, xc_y;
    {
#pragma clang fp contract(off)
        const float yaw = CG.obs_wrapper ? 0.0f : av.w;   // DroneObservationWrapper: yaw 0
        if (__builtin_expect(__all(yaw == 0.0f), 1)) {
            // yaw +-0 (the wrapper, or a FULLSTATE target without yaw, in every lane of the wave):
            // sincos(+-0) = (+-0, 1), 2 (1 (+-0) + 0 0) = +0, atan2f(+0, 1) = +0, (cos, sin)(+0) = (1, +0):
            // the general form's bits without its four libm calls
            xc_x = 1.0f;
            xc_y = 0.0f;
        } else {
            Real qs, qc;
            sincos_(Real(yaw) * Real(0.5), &qs, &qc);
            const float qz = float(qs), qw = float(qc);
            const float yaw_deg = degf_(atan2f(2.0f * (qw * qz + 0.0f * 0.0f), 1 - 2 * (0.0f * 0.0f + qz * qz)));
            xc_x = cosf(radf_(yaw_deg));
            xc_y = sinf(radf_(yaw_deg));
        }
    }
    const Lpf lpf = {CG.lpf[0], CG.lpf[1], CG.lpf[2], CG.lpf[3], CG.lpf[4]};   // lpf2pInit(gyrolpf, 500, 30), host
#if defined(ADRP_RACE_TIMING) && defined(ADRP_RACE_GJK_STATS)
    if (threadIdx.x == 0) g_gjk_wave_iters = 0;
#endif
    ccopy.store(&c_lds, tl);
    if constexpr (kDwF64) {
        if (tl < 32) exp_lds[tl] = exp_v;
    }
    if constexpr (!DRAWS && kDwF64) __syncthreads();   // the exp table (DRAWS: the barrier below)
    if constexpr (DRAWS) {   // sub-steps s = ql, ql + 4, ... of this drone
        quad_draws<Real>(H, pre_draws, a.seed, gid, ep, dn, sc0, ql, qd, H.S);
        __syncthreads();
#ifdef ADRP_EXP_DUP_DRAWS
        {
            uint32_t ep2 = ep;
            exp_dep(ep2, pre_draws[tl]);
            quad_draws<Real>(H, pre_draws, a.seed, gid, ep2, dn, sc0, ql, qd, H.S);
            __syncthreads();
        }
#endif
    }
    // lane-distributed controller state: axis cax of the rate history and the gyro filter
    Real prv = sel3(d.prev_rpy, cax);
    float l1 = sel3(d.lpf1, cax), l2 = sel3(d.lpf2, cax);
    M3<Real> Rq = rot(d.q), Rl = rot(d.ql);
    RACE_MARK(t1);
#ifdef ADRP_RACE_TIMING
    uint64_t acc_phys = 0;
#endif
#ifdef ADRP_CTRL_PHASES
    uint64_t cp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    for (int s0 = 0; s0 < H.S; s0 += 32) {
    if (s0 > 0) {
        d.tick_base = d.tick;
        tick_window(a.ticks, d.tick, d.att_bits, d.pos_bits);
    }
    const int s1 = H.S < s0 + 32 ? H.S : s0 + 32;
    for (int s = s0; s < s1; ++s) {
#ifdef ADRP_RACE_TIMING
        RACE_MARK(ta);
#endif
        if (PH != ADRP_PHYS_PYB) d.kpos = d.pos;
        Real noise_m = Real(0);
        if constexpr (PH == ADRP_PHYS_DYN) {
            race_dyn_substep(H, d);
            Rq = rot(d.q);
        } else {
            V3<Real> Fx = v3(Real(0), Real(0), Real(0)), Tx = v3(Real(0), Real(0), Real(0));
            if constexpr (PH == ADRP_PHYS_PYB_DW || PH == ADRP_PHYS_PYB_GND_DRAG_DW) {
#ifdef ADRP_EXP_DUP_DW
              V3<Real> dwp = d.pos;
              for (int rep = 0; rep < 2; ++rep) {
                if (rep == 1) exp_dep(dwp.x, Fx.z);
                const V3<Real> pos = dwp;
#else
              {
                const V3<Real>& pos = d.pos;
#endif
                // _downwash (BaseAviary.py:792-818): lane ql evaluates partner drones ql, ql + 4 (its
                // term alpha exp(-(dxy / beta)^2 / 2); 4 dz and beta are > 0 where it is used, dxy
                // a root of a sum of squares); the quad sums the terms by a DPP butterfly, so every
                // lane holds the same (t0 + t1) + (t2 + t3)
                Real tsum = Real(0);
#pragma unroll
                for (int j = 0; j < (G + 3) / 4; ++j) {
                    const int k = ql + 4 * j;
                    // ds_bpermute: DPP row broadcasts of the four partners' positions (row_newbcast +
                    // selects) measured 2.5-3 us slower on config 4 (round-3 A/B)
                    const int src = (tl & ~(4 * G - 1)) + 4 * (k < G ? k : 0);
                    const Real ox = __shfl(pos.x, src), oy = __shfl(pos.y, src), oz = __shfl(pos.z, src);
                    const Real dz = oz - pos.z, dx = ox - pos.x, dy = oy - pos.y;
                    const Real dxy = hsqrt_nn_(dx * dx + dy * dy);
                    const Real kk = H.prop_r * rcp_nc_(Real(4) * dz);
                    const Real qq = dxy * rcp_nc_(H.dw2 * dz + H.dw3);
                    const Real term = H.dw1 * kk * kk * dw_exp(Real(-0.5) * qq * qq, exp_lds);
                    tsum += (k < N && dz > Real(0) && dxy < Real(10)) ? term : Real(0);
                }
                tsum += qswap1(tsum);
                tsum += qswap2(tsum);
                const Real fz = -tsum;
                const M3<Real>& Rs = H.link_lag && !(PH == ADRP_PHYS_PYB_GND_DRAG_DW) ? Rl : Rq;
                Fx = fz * col2(Rs);
              }
            }
            // disturbances: compile-time (the host runs this kernel with DRAWS = disturbances on and
            // the draws made up front; parity-mode injection and in-loop draws go to the one-lane
            // kernel), so no uniform branch splits the sub-step
            if constexpr (DRAWS) {
                V3<Real> fd;
                const float* src = pre_draws + s * 7 * kQuadDrones + qd;
                if constexpr (F32) {
                    fd = v3(src[0], src[kQuadDrones], src[2 * kQuadDrones]);
                    noise_m = src[(3 + ql) * kQuadDrones];
                } else {   // race_substep_draws' arithmetic on the stored uniforms / samples
                    fd = v3(H.dist_lo[0] + (H.dist_hi[0] - H.dist_lo[0]) * Real(src[0]),
                            H.dist_lo[1] + (H.dist_hi[1] - H.dist_lo[1]) * Real(src[kQuadDrones]),
                            H.dist_lo[2] + (H.dist_hi[2] - H.dist_lo[2]) * Real(src[2 * kQuadDrones]));
                    noise_m = Real(src[(3 + ql) * kQuadDrones]) * H.noise_std;
                }
                const V3<Real> lo = (PH == ADRP_PHYS_PYB_GND || PH == ADRP_PHYS_PYB_GND_DRAG_DW) ? d.pos : d.lpos;
                Fx = Fx + fd;
                Tx = cross(d.kpos - lo, fd);
            }
            CP_MARK(f1);
            CP_ADD(4, f1 - ta);
#ifdef ADRP_EXP_DUP_STEP
            {
                RDrone<Real> d2 = d;
                M3<Real> Rq2 = Rq, Rl2 = Rl;
                race_pyb_substep_r<Real, PH>(H, d2, Fx, Tx, Rq2, Rl2);
                exp_dep(Fx.x, d2.q.x);
            }
#endif
            race_pyb_substep_r<Real, PH>(H, d, Fx, Tx, Rq, Rl);
        }
#ifdef ADRP_RACE_TIMING
        RACE_MARK(tb);
        acc_phys += tb - ta;
#endif
        d.kpos = d.pos;
        if (d.flags & 1) {      // eliminated: motors off (233-235)
#pragma unroll
            for (int k = 0; k < 4; ++k) d.rpm[k] = d.prev[k] = Real(0);
        } else {
            CP_MARK(e0);
#ifdef ADRP_EXP_DUP_EUL
            Q4<Real> q2 = d.q;
            exp_dep(q2.x, euler_axis_q4(d.q, cax));
            const Real rpy_a = euler_axis_q4(q2, cax);
#else
            const Real rpy_a = euler_axis_q4(d.q, cax);
#endif
#ifdef ADRP_EXP_DUP_WRAP
            {
                RDrone<Real> d2 = d;
                Real prv2 = prv;
                float l12 = l1, l22 = l2;
                mellinger_q4(d2, lpf, sp, xc_x, xc_y, rpy_a, prv2, l12, l22, noise_m, ql, Rq CP_ARG);
                exp_dep(prv, d2.rpm[0]);
            }
#endif
            CP_MARK(e1);
            CP_ADD(0, e1 - e0);
            mellinger_q4(d, lpf, sp, xc_x, xc_y, rpy_a, prv, l1, l2, noise_m, ql, Rq CP_ARG);
        }
    }
    }
    RACE_MARK(t2);
    // gather the distributed controller state back (all lanes active)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d.prev_rpy[k] = qbc(prv, k);
        d.lpf1[k] = qbc(l1, k);
        d.lpf2[k] = qbc(l2, k);
    }
    // the state the post-loop phases do not change goes out now, so its registers are free for the
    // track queries and the reset (a done env's auto-reset overwrites it below)
    // (fp64 since round 3: config 4 95 -> 80.5 us; fp32 since round 5, with the auto-reset copying
    // images: config 3 30.4 -> 30.0 us, config 3 + actor 54.5 -> 53.7 us, config 4 unchanged, where
    // rounds 3 and 4 had measured it +0.3-0.5 us)
    constexpr bool kEarlyStore = true;
    if constexpr (kEarlyStore) {
        if (owner) store_drone_body<Real, PH == ADRP_PHYS_DYN>(a, EN, slot, d);
    }
    // the episode this env's next-reset image is for, loaded here so that its latency hides behind
    // the post-loop phases (the barrier keeps the load from sinking to its use in the auto-reset)
    const int img_for = a.img_ep != nullptr ? a.img_ep[e] : -2;
    __syncthreads();
    const TrackSrcQ<Real> T{trk_lds, qd};
    // ---- _gate_progress (471-506) ----
    V3<Real> gpos[ADRP_MAX_DRONES];
    Q4<Real> gq[ADRP_MAX_DRONES];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        gpos[k] = v3(grpq<G>(d.pos.x, k), grpq<G>(d.pos.y, k), grpq<G>(d.pos.z, k));
        gq[k] = {grpq<G>(d.q.x, k), grpq<G>(d.q.y, k), grpq<G>(d.q.z, k), grpq<G>(d.q.w, k)};
    }
    const int gate0 = d.gate;
    if (C.num_gates > 0 && gate0 < C.num_gates) {
        const Real gx = T(RF_GATE + 4 * gate0), gy = T(RF_GATE + 4 * gate0 + 1);
        const Real rotg = T(RF_GATE + 4 * gate0 + 3);
        const Real h = C.gate_type[gate0] == 0 ? Real(1.0) : Real(0.525), half = Real(0.1875);
        Real sn, cs;
        sincos_f_(rotg, &sn, &cs);
        const Real dx = Real(0.05) * cs, dy = Real(0.05) * sn;
        const Real br = fabs_(C.coll_zoff) + hsqrt_(C.coll_r * C.coll_r + C.coll_hh * C.coll_hh) + Real(1e-5);
        uint32_t near = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const Real ex = gpos[k].x - gx, ey = gpos[k].y - gy;
            const Real ta = fmaxr_(fabs_(cs * ex + sn * ey) - Real(0.15), Real(0)), tb = -sn * ex + cs * ey;
            const Real tz = fmaxr_(fabs_(gpos[k].z - h) - half, Real(0));
            if (k < N && ta * ta + tb * tb + tz * tz < br * br) near |= 1u << k;
        }
        bool passed = false;
        for (int r = -3; r <= 3 && !passed && ((near >> dn) & 1u); ++r) {
            const V3<Real> p0 = v3(gx + Real(r) * dx, gy + Real(r) * dy, h - half);
            const V3<Real> p1 = v3(gx + Real(r) * dx, gy + Real(r) * dy, h + half);
            Real best = Real(2);
            int who = -1;
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if ((near >> k) & 1u) {
                    const Shape<Real> sk = drone_shape(C, gpos[k], gq[k]);
                    const Real fr = ray_cylinder(sk, p0, p1);
                    if (fr < best) { best = fr; who = k; }
                }
            }
            if (who == dn && best < Real(0.9999)) passed = true;
        }
        if (passed) d.gate += 1;
    }
    if (gate0 >= C.num_gates) d.flags |= 2;
    RACE_MARK(t3);
    // ---- obs row, elimination (674-698) ----
    const V3<Real> wv = PH == ADRP_PHYS_DYN ? d.angv : d.w;
    float* const rows = reinterpret_cast<float*>(rows4);
    float* row = rows + ((qd / G) * N + dn) * C.D;
    Real row0[15];
    const Shape<Real> ds = drone_shape(C, d.pos, d.q);
    uint32_t gin, oin;
    uint32_t amb, camb_all;
    bool ccert;
#ifdef ADRP_OBS_PHASES
    RACE_MARK(o0);
#endif
    // the pooled refinement in fp64 (config 3 + actor 82.4 -> 78.5 us, config 4 71.5 -> 71.2 us); fp32
    // refines inline (pooled: config 4 43.7 -> 44.1 us, config 3 + actor 58.4 -> 57.4 us; A/B round 4)
    track_bounds_q4(C, T, ds, Real(0.45), Real(1e-6), ql, !(d.flags & 1), gin, oin, amb, camb_all, ccert,
                    F32 ? nullptr : rpool);
    if constexpr (!F32) __syncthreads();   // the refine pool's LDS becomes the GJK job pool
#ifdef ADRP_OBS_PHASES
    RACE_MARK(o1);
#endif
    bool crashed = track_gjk_pool<Real, TrackSrcQ<Real>, 2>(C, T, ds, owner, Real(0.45), Real(1e-6), gin, oin, amb, camb_all,
                                                     tjobs, tl, G, N, a.E) || ccert;
#ifdef ADRP_OBS_PHASES
    RACE_MARK(o2);
#endif
    V3<Real> rpy;
    race_obs_row(C, T, d.pos, d.q, d.vel, wv, d.gate, row, owner, row0, gin, oin, &rpy);
#ifdef ADRP_OBS_PHASES
    RACE_MARK(o3);
#endif
    if (C.compete) {   // other drones' pos + rpy (653-659): the rpy of their own obs rows
        V3<Real> grpy[ADRP_MAX_DRONES];
#pragma unroll
        for (int k = 0; k < G; ++k) grpy[k] = v3(grpq<G>(rpy.x, k), grpq<G>(rpy.y, k), grpq<G>(rpy.z, k));
        int idx = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (owner && k < N && k != dn) {
                const V3<Real> orpy = grpy[k];
                float* p = row + 49 + 6 * idx;
                p[0] = gpos[k].x; p[1] = gpos[k].y; p[2] = gpos[k].z;
                p[3] = orpy.x; p[4] = orpy.y; p[5] = orpy.z;
                ++idx;
            }
        }
    }
    RACE_MARK(t4);
    {
        const M3<Real>& R = ds.R;
        const Real low = ds.c.z - ds.h.z * fabs_(R.a22) - ds.r * sqrt_(R.a02 * R.a02 + R.a12 * R.a12);
        if (low <= Real(1e-6)) crashed = true;
        if (C.compete) {
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if (k < N && k != dn && !crashed && !(d.flags & 1)) {   // eliminated: contacts change nothing
                    const V3<Real> dc = gpos[k] - d.pos;
                    const Real dr = hsqrt_(ds.r * ds.r + ds.h.z * ds.h.z);
                    if (dot(dc, dc) < (Real(2) * dr + Real(1e-4)) * (Real(2) * dr + Real(1e-4))) {
                        const Shape<Real> sk = drone_shape(C, gpos[k], gq[k]);
                        crashed = gjk_within(ds, sk, Real(1e-6));
                    }
                }
            }
        }
    }
    RACE_MARK(t5);
    const bool oob = fabs_(d.pos.x) > C.bounds[0] || fabs_(d.pos.y) > C.bounds[1] || fabs_(d.pos.z) > C.bounds[2];
    const bool unstable = fabs_(wv.x) > Real(20) || fabs_(wv.y) > Real(20) || fabs_(wv.z) > Real(20);
    if (oob || unstable || crashed) d.flags |= 1;
    const int mydone = ((d.flags & 1) || (d.flags & 2)) ? 1 : 0, myfin = (d.flags & 2) ? 1 : 0;
    int all_done = 1, all_fin = 1;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int dk = grpq_i<G>(mydone, k), fk = grpq_i<G>(myfin, k);
        if (k < N) {
            all_done &= dk;
            all_fin &= fk;
        }
    }
    const int gate_d0 = grpq_i<G>(d.gate, 0);
    const bool te_env = all_done != 0;
    const bool te = te_env || (C.obs_wrapper && gate_d0 >= 2);   // DroneObservationWrapper (wrapper.py:61-63)
    const bool te_rw = C.obs_wrapper == 1 ? te : te_env;
    const bool tr = sc0 >= C.trunc_steps;
    // ---- RewardWrapper (wrapper.py:121-186), drone 0 ----
    float reward = 0.0f;
    int wr_gate = a.ist[RI_WR_GATE * EN + slot];
    if (C.reward_wrapper && dn == 0) {
        const int gate_id = d.gate;
        Real tgt[3] = {ld(a.f, RF_WR_TARGET, EN, slot), ld(a.f, RF_WR_TARGET + 1, EN, slot), ld(a.f, RF_WR_TARGET + 2, EN, slot)};
        const Real prvp[3] = {ld(a.f, RF_WR_PREV, EN, slot), ld(a.f, RF_WR_PREV + 1, EN, slot), ld(a.f, RF_WR_PREV + 2, EN, slot)};
        Real r_passed = 0;
        if (gate_id > wr_gate % 4) {
            wr_gate = gate_id;
            if (gate_id < 4 && gate_id < C.num_gates) {
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int k = 0; k < 3; ++k) tgt[k] = g == gate_id ? row0[3 + 3 * g + k] : tgt[k];
            }
            r_passed = Real(5);
        }
        const Real r_col = (te_rw && !all_fin) ? Real(-1) : Real(0), r_lab = (te_rw && all_fin) ? Real(10) : Real(0);
        const Real pxy = sqrt_((tgt[0] - prvp[0]) * (tgt[0] - prvp[0]) + (tgt[1] - prvp[1]) * (tgt[1] - prvp[1]));
        const Real cxy = sqrt_((tgt[0] - row0[0]) * (tgt[0] - row0[0]) + (tgt[1] - row0[1]) * (tgt[1] - row0[1]));
        const Real pz = fabs_(tgt[2] - prvp[2]), cz = fabs_(tgt[2] - row0[2]);
        reward = float((pxy - cxy) + (pz - cz) + r_passed + r_col + r_lab);
        if (owner)
            for (int k = 0; k < 3; ++k) { st(a.f, RF_WR_TARGET + k, EN, slot, tgt[k]); st(a.f, RF_WR_PREV + k, EN, slot, row0[k]); }
    }
    const bool reset = C.autoreset && (te || tr);   // env-uniform: every lane of the env's quads agrees
    if (owner) {
        if (dn == 0) {
            a.rew[e] = reward;
            a.term[e] = te;
            a.trunc[e] = tr;
        }
        if (!reset) {
            if constexpr (!kEarlyStore) store_drone_body<Real, PH == ADRP_PHYS_DYN>(a, EN, slot, d);
            store_drone_flags(a, EN, slot, d);
            a.ist[RI_STEP * EN + slot] = sc0 + C.S;
            if (dn == 0) a.ist[RI_WR_GATE * EN + slot] = wr_gate;
        }
    }
    // terminal obs, then the resets: a done env's work is dealt over the wave's 64 lanes (the
    // other envs' lanes are idle here), one resetting env at a time (rarely more than one per wave)
    const bool img = reset && img_for == episode;          // (env-uniform)
    const bool env_lead = reset && owner && dn == 0;        // one lane per resetting env
    for (uint64_t rm = __ballot(env_lead && a.tobs != nullptr); rm; rm &= rm - 1) {
        const int L = __builtin_ctzll(rm);
        const int er = __builtin_amdgcn_readlane(e, L), eb = __builtin_amdgcn_readlane(qd, L) / G;
        wave_copy_rows<G * kRowF>(rows + eb * N * C.D, a.tobs + size_t(er) * N * C.D, N * C.D, tl);
    }
    for (uint64_t rm = __ballot(env_lead && img); rm; rm &= rm - 1) {
        const int L = __builtin_ctzll(rm);
        const int er = __builtin_amdgcn_readlane(e, L), eb = __builtin_amdgcn_readlane(qd, L) / G;
        reset_from_image<Real, G, kRowF>(a, EN, size_t(er) * N, N, rows + eb * N * C.D, C.D, tl);
    }
    if (reset && !img) race_reset_q4<Real, G>(a, C, e, dn, ql, active, EN, slot, episode, row, ResetToHBM<Real>{&a});
    if (a.reset_count && env_lead) atomicAdd(a.reset_count + (img ? 0 : 1), 1);
#ifdef ADRP_RACE_TIMING
    RACE_MARK(t6);   // tail: reward, flags, stores and the auto-reset of done envs
    if (threadIdx.x == 0) {
#if defined(ADRP_CTRL_PHASES)   // euler, wrapper head, firmware, wrapper (all), forces, physics, loop
        RACE_WAVE(0, cp[0]); RACE_WAVE(1, cp[1]); RACE_WAVE(2, cp[2]); RACE_WAVE(3, cp[3]);
        RACE_WAVE(4, cp[4]); RACE_WAVE(5, acc_phys); RACE_WAVE(6, t2 - t1); RACE_WAVE(7, t6 - t0);
#elif defined(ADRP_RESET_PHASES)   // the reset's sub-phases of this block's last reset (0 if none)
        for (int k = 0; k < 8; ++k) RACE_WAVE(k, reset ? g_reset_mark[k + 1] - g_reset_mark[k] : 0);
#else
        RACE_WAVE(0, t1 - t0); RACE_WAVE(1, acc_phys); RACE_WAVE(2, (t2 - t1) - acc_phys); RACE_WAVE(3, t3 - t2);
#if defined(ADRP_OBS_PHASES)   // measurement-only: the obs phase split (bounds, GJK pool, row, compete rows)
        RACE_WAVE(0, o1 - o0); RACE_WAVE(1, o2 - o1); RACE_WAVE(2, o3 - o2); RACE_WAVE(3, t4 - o3);
        RACE_WAVE(4, t4 - t3); RACE_WAVE(5, t5 - t4); RACE_WAVE(6, t6 - t5); RACE_WAVE(7, t6 - t0);
#elif defined(ADRP_RACE_GJK_STATS)   // the "contacts" slot: this workgroup's GJK iterations
        RACE_WAVE(4, t4 - t3); RACE_WAVE(5, g_gjk_wave_iters); RACE_WAVE(6, t6 - t5); RACE_WAVE(7, t6 - t0);
#else
        RACE_WAVE(4, t4 - t3); RACE_WAVE(5, t5 - t4); RACE_WAVE(6, t6 - t5); RACE_WAVE(7, t6 - t0);
#endif
#endif
    }
#endif
    // ---- coalesced copy-out of the block's rows ----
    __syncthreads();
    const int e0 = lb * (kQuadDrones / G);
    const int ne = a.E - e0 < kQuadDrones / G ? a.E - e0 : kQuadDrones / G;
    const int total = ne * N * C.D;
    float* dst = a.obs + size_t(e0) * N * C.D;
    constexpr int kCopyStride = kRaceBlock;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        float4* dst4 = reinterpret_cast<float4*>(dst);
        const int n4 = total >> 2;
        for (int i = tl; i < n4; i += kCopyStride) store_out(dst4 + i, rows4[i]);
        for (int i = 4 * n4 + tl; i < total; i += kCopyStride) dst[i] = rows[i];
    } else {
        for (int i = tl; i < total; i += kCopyStride) dst[i] = rows[i];
    }
}

}  // namespace adrp
