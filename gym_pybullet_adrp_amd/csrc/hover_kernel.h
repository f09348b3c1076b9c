// hover_kernel.h — fused HoverAviary env.step for gfx950: one lane per env, all
// PYB_FREQ/CTRL_FREQ sub-steps in registers, then obs / reward / terminated /
// truncated and (optionally) the VecEnv auto-reset, in ONE launch.
//
// Reference path (FelixWaiblinger/gym-pybullet-adrp @ 2024-10-08):
//   BaseAviary.step            envs/BaseAviary.py:262-387 (sub-step loop 347-376)
//   _preprocessAction          envs/BaseRLAviary.py:160-239 (RPM 192, ONE_D_RPM 225)
//   _physics / _groundEffect / _drag / _downwash   envs/BaseAviary.py:683-818
//   p.stepSimulation (Bullet btMultiBody floating base)        BaseAviary.py:373-374
//   _dynamics / _integrateQ (Physics.DYN)          envs/BaseAviary.py:822-896
//   _computeObs                envs/BaseRLAviary.py:284-319
//   _computeReward / _computeTerminated / _computeTruncated    envs/HoverAviary.py:68-117
//
// Closed form used per Bullet sub-step (derivation in DESIGN.md §Kernel):
//   thrust axis  zs = Rs·ẑ  (Rs = link basis cached at the last forwardKinematics)
//   F_world      = Σf·zs + [Σg·R·ẑ] + B·f_link4 + m·g
//   n_body       = P × (Rᵀzs) + τz·(Rᵀzs) + [G × ẑ]          P = Σ f_i p_i, G = Σ g_i p_i
//   ω̇_b          = I⁻¹(n_b − k(1+|ω_b|) I∘ω_b − ω_b × I ω_b),   a_w = F_w/m − k(1+|v|) v
//   v, ω += dt(·) (clamped ±100);  x += dt v;  q ← normalize((ω̂ sin, cos) ⊗ q)
//
// Latency design (E = 4096 is 64 waves on 256 CUs: the kernel is one wave's critical
// path): no divides or IEEE sqrt in the sub-step chain (reciprocal constants, 1-ulp
// hardware rcp/sqrt/rsq), small-angle sin/cos polynomial, the lagged link basis is the
// previous sub-step's rotation matrix (carried, not recomputed), the action-ring loads
// are issued at entry independent of the ring head, rows are written with 16-byte
// per-lane stores straight from registers (no LDS, no barrier).
#pragma once

#include "adrp_device.h"

namespace adrp {

// float-field indices of the HoverAviary state snapshot ([field][E], SoA)
enum HoverField {
    HF_POS = 0, HF_QUAT = 3, HF_VEL = 7, HF_OMEGA = 10, HF_LAST_RPM = 13, HF_ANGV = 17,
    HF_LINK_QUAT = 20, HF_NBASE = 24,
    // DSLPIDControl state (PID / VEL / ONE_D_PID handles only): last_rpy 3, integral_pos_e 3,
    // integral_rpy_e 3 (control/DSLPIDControl.py:65-79)
    HF_PID = 24, HF_NPID = 9
};
enum HoverInt { HI_STEP = 0, HI_EPISODE = 1, HI_RING_HEAD = 2, HI_N = 3 };

// Per-config constants.  Device-resident (one block per handle, written at create, warm
// in L2 across launches), or compiled in as literals for the reference's default drone
// (cf2x_consts: CF2X / cf2x_IROS.urdf at 240 Hz), where they fold into immediates.
template <typename Real>
struct HoverConst {
    int S, trunc_steps, link_lag, physics;   // truncated once step_counter >= trunc_steps
    Real dt, mass, inv_mass, gravity;
    Real ixx, iyy, izz, inv_ixx, inv_iyy, inv_izz;
    Real kf, km, hover_rpm;
    Real px[4], py[4], pz[4];                // prop link COM offsets (body)
    Real gnd_kf, prop_r4, gnd_clip;          // kf*GND_EFF_COEFF, PROP_RADIUS/4, GND_EFF_H_CLIP
    Real drag[3];
    Real dyn_arm;                            // L/sqrt(2) (Physics.DYN)
    Real coll_hh, coll_r, coll_zoff;         // collision cylinder half-height, radius, z offset
    Real ang_max;                            // ANGULAR_MOTION_THRESHOLD / dt
    Real target[3];
    // DSLPIDControl (PID / VEL / ONE_D_PID): GRAVITY = g*m (BaseControl.py:35, the env's own
    // URDF), 1/(4 KF), CTRL_TIMESTEP and its inverse, SPEED_LIMIT as the float32 NumPy uses
    Real pid_grav, pid_inv4kf, ctrl_dt, ctrl_hz;
    float speed_limit;
};

// HoverAviary defaults: cf2x_IROS.urdf, PYB_FREQ 240, CTRL_FREQ 30, target (0,0,1), 8 s.
// Derived values are the float64 results of BaseAviary.py:117-128's formulas; the host
// selects this path only when its computed block is bit-identical (adrp.hip).
template <typename Real>
__host__ __device__ constexpr HoverConst<Real> cf2x_consts(int physics) {
    HoverConst<Real> c{};
    c.S = 8; c.trunc_steps = 1921; c.link_lag = 1; c.physics = physics;
    c.dt = Real(0.004166666666666667);
    c.mass = Real(0.03454); c.inv_mass = Real(28.951939779965258); c.gravity = Real(9.8);
    c.ixx = Real(1.4e-5); c.iyy = Real(1.4e-5); c.izz = Real(2.17e-5);
    c.inv_ixx = Real(71428.57142857143); c.inv_iyy = Real(71428.57142857143); c.inv_izz = Real(46082.949308755764);
    c.kf = Real(3.16e-10); c.km = Real(7.94e-12); c.hover_rpm = Real(16364.421890108686);
    c.px[0] = Real(0.028); c.px[1] = Real(-0.028); c.px[2] = Real(-0.028); c.px[3] = Real(0.028);
    c.py[0] = Real(0.028); c.py[1] = Real(0.028); c.py[2] = Real(-0.028); c.py[3] = Real(-0.028);
    c.pz[0] = Real(0); c.pz[1] = Real(0); c.pz[2] = Real(0); c.pz[3] = Real(0);
    c.gnd_kf = Real(3.5924744399999996e-09); c.prop_r4 = Real(0.0057837); c.gnd_clip = Real(0.03776371349209501);
    c.drag[0] = Real(9.1785e-7); c.drag[1] = Real(9.1785e-7); c.drag[2] = Real(10.311e-7);
    c.dyn_arm = Real(0.028072139213105935);
    c.coll_hh = Real(0.0125); c.coll_r = Real(0.06); c.coll_zoff = Real(0);
    c.ang_max = Real(188.49555921538757);
    c.target[0] = Real(0); c.target[1] = Real(0); c.target[2] = Real(1);
    c.pid_grav = Real(0.338492); c.pid_inv4kf = Real(791139240.5063292);
    c.ctrl_dt = Real(0.03333333333333333); c.ctrl_hz = Real(30);
    c.speed_limit = 0.25f;
    return c;
}

// reset distribution (only the auto-reset / reset path reads it)
template <typename Real>
struct HoverReset {
    Real init_xyz[3], init_rpy[3], n_xyz[3], n_rpy[3], n_vel[3], n_om[3];
};

// kernel argument block: pointers and a few scalars only (it is rewritten for every
// launch, so it is cold in every cache: keep it to two 64-byte lines)
constexpr int kStepBlock = 64;   // envs per workgroup: one chain wave (E = 4096 -> 64 CUs)
constexpr int kResetFields = 16; // pos 3, quat 4, vel 3, w 3, angv 3 of a reset state (HELP)
// HELP kernels: two more helper waves beside the reset helper compute the obs row's pitch and yaw
// from the chain's final quaternion while the chain computes the roll (ADRP_HOVER_ANGLE_HELPERS=0:
// the chain computes all three, one helper wave)
#ifndef ADRP_PERSIST_SPLIT   // 0: a step of one env (launched or persistent) computes its three obs angles on one lane
#define ADRP_PERSIST_SPLIT 1
#endif
#ifndef ADRP_HOVER_ANGLE_HELPERS
#define ADRP_HOVER_ANGLE_HELPERS 1
#endif
// (float64 only: in float32 the two extra barriers cost more than the two atan2 they take off the
// chain, +1.2 % against -1.2 % in float64, A/B round 6)
template <typename Real>
constexpr bool angle_helpers() { return ADRP_HOVER_ANGLE_HELPERS != 0 && sizeof(Real) == 8; }
template <typename Real>
constexpr int help_waves() { return angle_helpers<Real>() ? 3 : 1; }   // helper waves of a HELP workgroup

template <typename Real>
struct HoverArgs {
    const HoverConst<Real>* c;   // device-resident constants (generic path)
    const HoverReset<Real>* r;
    Real* f;           // [HF_NBASE][E]
    float* ring;       // [B][E][A]  (slot-major, the A floats of one env contiguous)
    int32_t* ist;      // [HI_N][E]
    const float* act;  // [E][A]
    float* obs;        // [E][D]
    float* rew;
    uint8_t* term;
    uint8_t* trunc;
    float* tobs;       // [E][D] or null
    const uint8_t* mask;  // reset mask or null
    int32_t* contact_count;  // device counter of ground-model hits (diagnostics) or null
    uint64_t seed;
    int64_t env_offset;
    int E, B, D, autoreset;
};

template <typename Real>
struct Body {
    V3<Real> pos, vel, w;     // w: world ω (PYB) or body rpy_rates (DYN)
    Q4<Real> q, ql;           // pose quaternion, cached link basis
    V3<Real> angv;            // DYN: world ω reported by getBaseVelocity
    Real prev_rpm[4];
};

// Explicit fused multiply-adds of the PYB sub-step chain.  The hover TUs contract a*b+c only
// within one source expression (csrc/Makefile CONTRACT: the same bits in every dispatch variant),
// so the fusions across the V3 operators that the chain wants are written out here.
__device__ __forceinline__ float fmx(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmx(double a, double b, double c) { return __builtin_fma(a, b, c); }

// rot(q) with its products folded into FMAs (20 operations instead of 24)
template <typename Real>
__device__ __forceinline__ M3<Real> rot_fm(Q4<Real> q) {
    const Real x2 = q.x + q.x, y2 = q.y + q.y, z2 = q.z + q.z;
    const Real xx = q.x * x2, zz = q.z * z2;
    const Real wx = q.w * x2, wy = q.w * y2, wz = q.w * z2;
    return {Real(1) - fmx(q.y, y2, zz), fmx(q.x, y2, -wz), fmx(q.x, z2, wy),
            fmx(q.x, y2, wz), Real(1) - fmx(q.x, x2, zz), fmx(q.y, z2, -wx),
            fmx(q.x, z2, -wy), fmx(q.y, z2, wx), Real(1) - fmx(q.y, y2, xx)};
}

// float32 1 + 0.05 a, two roundings as NumPy does it (no FMA contraction)
__device__ __forceinline__ float rpm_gain(float a) {
#pragma clang fp contract(off)
    const float m = 0.05f * a;
    return 1.0f + m;
}

// One Bullet stepSimulation of one drone after the reference's force calls.
// R = rot(b.q) on entry; Rs = rotation of the cached link basis.  On exit R/Rs are the
// matrices the next sub-step needs.  wn = |b.w| on entry and on exit (the exp map's |w| is the
// next sub-step's |R^T w| of the damping term: a rotation keeps the norm, so the chain takes one
// square root per sub-step, not two; rounding-level difference).  Returns true if the plane
// contact model acted.
// K: the chain's literal constants (pinned into VGPRs by the fp64 caller, ChainK)
template <typename Real, int PH>
__device__ __forceinline__ bool pyb_substep(const HoverConst<Real>& a, Body<Real>& b, M3<Real>& R, M3<Real>& Rs,
                                            const Real rpm[4], Real sum_f, V3<Real> P, Real tau_z, Real& wn,
                                            const ChainK<Real>& K) {
    constexpr bool GND = (PH == ADRP_PHYS_PYB_GND || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    constexpr bool DRAG = (PH == ADRP_PHYS_PYB_DRAG || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    // _physics: 4 prop forces + z torque on link 4, LINK_FRAME, cached basis
    const V3<Real> zs = col2(Rs);
    V3<Real> Fw = v3(sum_f * zs.x, sum_f * zs.y, sum_f * zs.z - a.mass * a.gravity);
    const V3<Real> m3 = mulT(R, zs);
    // P x m3 + tau_z m3
    V3<Real> nb = v3(fmx(tau_z, m3.x, fmx(P.y, m3.z, -(P.z * m3.y))), fmx(tau_z, m3.y, fmx(P.z, m3.x, -(P.x * m3.z))),
                     fmx(tau_z, m3.z, fmx(P.x, m3.y, -(P.y * m3.x))));
    bool cur_basis = false;
    if constexpr (GND) {
        // getLinkStates(computeForwardKinematics=1) refreshes the cached basis first
        cur_basis = true;
        const Real sqx = b.q.x * b.q.x, sqy = b.q.y * b.q.y, sqz = b.q.z * b.q.z, squ = b.q.w * b.q.w;
        const Real sarg = Real(-2) * (b.q.x * b.q.z - b.q.w * b.q.y);
        const Real den = squ - sqx - sqy + sqz, num = Real(2) * (b.q.y * b.q.z + b.q.w * b.q.x);
        // |roll| < pi/2 and |pitch| < pi/2 of getEulerFromQuaternion (BaseAviary.py:749)
        const bool gate = fabs_(sarg) < Real(0.99999) && (den > Real(0) || (den == Real(0) && num == Real(0)));
        if (gate) {
            Real sg = 0;
            V3<Real> G = v3(Real(0), Real(0), Real(0));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                Real h = b.pos.z + R.a20 * a.px[i] + R.a21 * a.py[i] + R.a22 * a.pz[i];
                h = h < a.gnd_clip ? a.gnd_clip : h;
                const Real k = a.prop_r4 * rcp_(h);
                const Real g = a.gnd_kf * rpm[i] * rpm[i] * k * k;
                sg += g;
                G = G + v3(g * a.px[i], g * a.py[i], g * a.pz[i]);
            }
            Fw = Fw + sg * col2(R);
            nb = nb + v3(G.y, -G.x, Real(0));
        }
    }
    if constexpr (DRAG) {
        Real s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += b.prev_rpm[i];
        s = s * Real(0.10471975511965977);  // sum(2*pi*rpm/60)
        const V3<Real> dw = v3(-a.drag[0] * s * b.vel.x, -a.drag[1] * s * b.vel.y, -a.drag[2] * s * b.vel.z);
        const V3<Real> dl = mulT(R, dw);    // np.dot(base_rot.T, drag_factors * vel)
        Fw = Fw + (cur_basis ? dw : mul(Rs, dl));
    }
    // ---- Bullet: forwardKinematics, ABA of the floating base, semi-implicit Euler ----
    const V3<Real> wb = mulT(R, b.w);
    const V3<Real> Iw = v3(a.ixx * wb.x, a.iyy * wb.y, a.izz * wb.z);
    const Real kw = K.k004 + K.k004 * wn;
    // nb - kw Iw - wb x Iw
    const V3<Real> rhs = v3(fmx(wb.z, Iw.y, fmx(-wb.y, Iw.z, fmx(-kw, Iw.x, nb.x))),
                            fmx(wb.x, Iw.z, fmx(-wb.z, Iw.x, fmx(-kw, Iw.y, nb.y))),
                            fmx(wb.y, Iw.x, fmx(-wb.x, Iw.y, fmx(-kw, Iw.z, nb.z))));
    const V3<Real> wdot = mul(R, v3(rhs.x * a.inv_ixx, rhs.y * a.inv_iyy, rhs.z * a.inv_izz));
    const Real kv = K.k004 + K.k004 * hsqrt_nn_(dot(b.vel, b.vel), K);
    const V3<Real> acc = v3(fmx(-kv, b.vel.x, a.inv_mass * Fw.x), fmx(-kv, b.vel.y, a.inv_mass * Fw.y),
                            fmx(-kv, b.vel.z, a.inv_mass * Fw.z));
    b.w = v3(b.w.x + a.dt * wdot.x, b.w.y + a.dt * wdot.y, b.w.z + a.dt * wdot.z);
    b.vel = v3(b.vel.x + a.dt * acc.x, b.vel.y + a.dt * acc.y, b.vel.z + a.dt * acc.z);
    clamp100_wv(b.w, b.vel, K);
    b.pos = v3(fmx(a.dt, b.vel.x, b.pos.x), fmx(a.dt, b.vel.y, b.pos.y), fmx(a.dt, b.vel.z, b.pos.z));
    // exp-map quaternion update (btMultiBody::stepPositionsMultiDof)
    Real ang = hsqrt_nn_(dot(b.w, b.w), K);
    wn = ang;
    if (ang > a.ang_max) ang = a.ang_max;          // |w| dt > ANGULAR_MOTION_THRESHOLD
    // sin(|w| dt / 2) / |w| = (dt / 2) sinc(|w| dt / 2): no reciprocal, and Bullet's small-angle
    // form (|w| < 0.001: 0.5 dt - dt^3 |w|^2 / 48) is the same series to rounding
    Real sinc, ch;
    expmap_sinc_cos(Real(0.5) * ang * a.dt, &sinc, &ch, K);
    const Real sc = (Real(0.5) * a.dt) * sinc;
    const V3<Real> ax = sc * b.w;
    const Q4<Real> q0 = b.q;
    const Q4<Real> q1 = {ch * q0.x + ax.x * q0.w + ax.y * q0.z - ax.z * q0.y,
                         ch * q0.y + ax.y * q0.w + ax.z * q0.x - ax.x * q0.z,
                         ch * q0.z + ax.z * q0.w + ax.x * q0.y - ax.y * q0.x,
                         ch * q0.w - ax.x * q0.x - ax.y * q0.y - ax.z * q0.z};
    const Real inv = quat_inv_norm(q1.x * q1.x + q1.y * q1.y + q1.z * q1.z + q1.w * q1.w, K);
    // the basis cached by this step's forwardKinematics is the pre-integration pose
    if (a.link_lag) {
        b.ql = b.q;
        Rs = R;
    }
    b.q = {q1.x * inv, q1.y * inv, q1.z * inv, q1.w * inv};
    R = rot_fm(b.q);
    if (!a.link_lag) Rs = R;
    // plane contact model: non-penetration, no inward velocity.
    // lowest point of the body cylinder: cos(tilt) = R22, sin(tilt) = |(R02, R12)|.  It is at
    // least z + zoff - hh - r below the centre, so a wave whose drones are all higher than that
    // skips the exact test (same result)
    if (__builtin_expect(__any(b.pos.z + a.coll_zoff <= a.coll_hh + a.coll_r + Real(1e-6)), 0)) {
        const Real low = b.pos.z + a.coll_zoff - a.coll_hh * fabs_(R.a22) - a.coll_r * hsqrt_nn_(R.a02 * R.a02 + R.a12 * R.a12);
        if (low < Real(0)) {
            b.pos.z -= low;
            if (b.vel.z < Real(0)) b.vel.z = Real(0);
            return true;
        }
    }
    return false;
}

// Physics.DYN (BaseAviary.py:822-896): explicit model, forward Euler, _integrateQ
template <typename Real>
__device__ __forceinline__ void dyn_substep(const HoverConst<Real>& a, Body<Real>& b, const Real rpm[4]) {
    const M3<Real> R = rot(b.q);
    Real f[4], zt[4], sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[i] = rpm[i] * rpm[i] * a.kf;
        zt[i] = rpm[i] * rpm[i] * a.km;
        sum += f[i];
    }
    const V3<Real> zb = col2(R);
    const V3<Real> force_w = v3(sum * zb.x, sum * zb.y, sum * zb.z - a.gravity * a.mass);
    const Real tz = -zt[0] + zt[1] - zt[2] + zt[3];
    const Real tx = (f[0] + f[1] - f[2] - f[3]) * a.dyn_arm;
    const Real ty = (-f[0] + f[1] + f[2] - f[3]) * a.dyn_arm;
    const V3<Real> rr = b.w;
    const V3<Real> tq = v3(tx, ty, tz) - cross(rr, v3(a.ixx * rr.x, a.iyy * rr.y, a.izz * rr.z));
    const V3<Real> rdd = v3(tq.x * a.inv_ixx, tq.y * a.inv_iyy, tq.z * a.inv_izz);
    b.vel = b.vel + a.dt * (a.inv_mass * force_w);
    b.w = rr + a.dt * rdd;
    b.pos = b.pos + a.dt * b.vel;
    const V3<Real> w = b.w;
    const Real wn = hsqrt_(dot(w, w));
    if (!(wn <= Real(1e-8))) {  // np.isclose(omega_norm, 0)
        const Real th = wn * a.dt * Real(0.5);
        Real s, c;
        if (th <= Real(0.39269908169872414)) small_sincos(th, &s, &c);
        else sincos_(th, &s, &c);
        const Real k = s * rcp_(wn);
        const Q4<Real> q = b.q;
        b.q = {c * q.x + k * (w.z * q.y - w.y * q.z + w.x * q.w),
               c * q.y + k * (-w.z * q.x + w.x * q.z + w.y * q.w),
               c * q.z + k * (w.y * q.x - w.x * q.y + w.z * q.w),
               c * q.w + k * (-w.x * q.x - w.y * q.y - w.z * q.z)};
    }
    b.angv = mul(R, b.w);   // resetBaseVelocity(vel, rotation @ rpy_rates)
}

// BaseAviary.reset -> _housekeeping (+ the optional init_noise extension), Real precision
template <typename Real>
__device__ __forceinline__ void hover_reset_state(const HoverArgs<Real>& args, const HoverConst<Real>& C, int e,
                                                  Body<Real>& b, int32_t& sc, int32_t& ep) {
    const HoverReset<Real>& a = *args.r;
    const uint64_t gid = uint64_t(args.env_offset + e);
    const U4 r0 = draw(args.seed, gid, uint32_t(ep), TAG_HOVER_RESET, 0);
    const U4 r1 = draw(args.seed, gid, uint32_t(ep), TAG_HOVER_RESET, 1);
    const U4 r2 = draw(args.seed, gid, uint32_t(ep), TAG_HOVER_RESET, 2);
    const uint32_t w0[4] = {r0.a, r0.b, r0.c, r0.d}, w1[4] = {r1.a, r1.b, r1.c, r1.d},
                   w2[4] = {r2.a, r2.b, r2.c, r2.d};
    Real p[3], e_[3], v[3], om[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        p[k] = a.init_xyz[k] + a.n_xyz[k] * (Real(2) * u01r<Real>(w0[k]) - Real(1));
        e_[k] = a.init_rpy[k] + a.n_rpy[k] * (Real(2) * u01r<Real>(w1[k]) - Real(1));
        v[k] = a.n_vel[k] * (Real(2) * u01r<Real>(w2[k]) - Real(1));
    }
    om[0] = a.n_om[0] * (Real(2) * u01r<Real>(w0[3]) - Real(1));
    om[1] = a.n_om[1] * (Real(2) * u01r<Real>(w1[3]) - Real(1));
    om[2] = a.n_om[2] * (Real(2) * u01r<Real>(w2[3]) - Real(1));
    b.q = quat_from_euler_fast<Real>(e_[0], e_[1], e_[2]);
    b.pos = v3(p[0], p[1], p[2]);
    b.ql = b.q;
    b.vel = v3(v[0], v[1], v[2]);
    if (C.physics == ADRP_PHYS_DYN) {
        b.w = mulT(rot(b.q), v3(om[0], om[1], om[2]));
        b.angv = v3(om[0], om[1], om[2]);
    } else {
        b.w = v3(om[0], om[1], om[2]);
        b.angv = v3(Real(0), Real(0), Real(0));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) b.prev_rpm[i] = Real(0);
    sc = 0;
    ep += 1;
}

// euler_xyz_fast_u's angles one at a time: the same expressions (the same contraction, so the same
// bits) and the same wave-uniform gimbal-lock branch, for the HELP kernel's angle helpers
template <typename Real>
__device__ __forceinline__ Real euler_roll_u(Q4<Real> q) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) return euler_xyz_fast(q).x;
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    return fatan2_(Real(2) * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz);
}
template <typename Real>
__device__ __forceinline__ Real euler_pitch_u(Q4<Real> q) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) return euler_xyz_fast(q).y;
    return fasin_(sarg);
}
template <typename Real>
__device__ __forceinline__ Real euler_yaw_u(Q4<Real> q) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) return euler_xyz_fast(q).z;
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    return fatan2_(Real(2) * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz);
}

// E = 1 persistent step (SPLIT): lane L evaluates Euler angle min(L, 2) of the (duplicated) env with
// ONE atan2 -- roll (y0, x0), pitch (sarg, sqrt((1 - sarg)(1 + sarg)), the atan2 form of fasin_),
// yaw (y2, x2) -- and the three come back by readlane: the same expressions as euler_xyz_fast_u, so
// the same bits, for one atan2 on the chain instead of three
template <typename Real>
__device__ __forceinline__ Real euler_axis_u(Q4<Real> q, int ax) {
    const Real sarg = Real(-2) * (q.x * q.z - q.w * q.y);
    if (__builtin_expect(__any(fabs_(sarg) >= Real(0.99999)), 0)) {
        const V3<Real> r = euler_xyz_fast(q);
        return ax == 0 ? r.x : (ax == 1 ? r.y : r.z);
    }
    const Real sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    const Real y0 = Real(2) * (q.y * q.z + q.w * q.x), x0 = squ - sqx - sqy + sqz;
    const Real y2 = Real(2) * (q.x * q.y + q.w * q.z), x2 = squ + sqx - sqy - sqz;
    Real x1;
    if constexpr (sizeof(Real) == 8) x1 = f64::sqrt((1.0 - sarg) * (1.0 + sarg));
    else x1 = __builtin_amdgcn_sqrtf((1.0f - sarg) * (1.0f + sarg));
    const Real yy = ax == 0 ? y0 : (ax == 1 ? sarg : y2), xx = ax == 0 ? x0 : (ax == 1 ? x1 : x2);
    return fatan2_(yy, xx);
}
__device__ __forceinline__ float readlane_r(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_r(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// hover_obs12 with the angles dealt over lanes 0..2 (every lane holds the same env)
template <typename Real>
__device__ __forceinline__ V3<Real> hover_obs12_split(const HoverConst<Real>& a, const Body<Real>& b, float o[12]) {
    const int l = int(threadIdx.x) & 63;
    const Real ang = euler_axis_u(b.q, l < 2 ? l : 2);
    const V3<Real> rpy = v3(readlane_r(ang, 0), readlane_r(ang, 1), readlane_r(ang, 2));
    const V3<Real> w = a.physics == ADRP_PHYS_DYN ? b.angv : b.w;
    o[0] = float(b.pos.x); o[1] = float(b.pos.y); o[2] = float(b.pos.z);
    o[3] = float(rpy.x);   o[4] = float(rpy.y);   o[5] = float(rpy.z);
    o[6] = float(b.vel.x); o[7] = float(b.vel.y); o[8] = float(b.vel.z);
    o[9] = float(w.x);     o[10] = float(w.y);    o[11] = float(w.z);
    return rpy;
}

template <typename Real>
__device__ __forceinline__ V3<Real> hover_obs12(const HoverConst<Real>& a, const Body<Real>& b, float o[12]) {
    const V3<Real> rpy = euler_xyz_fast_u(b.q);
    const V3<Real> w = a.physics == ADRP_PHYS_DYN ? b.angv : b.w;
    o[0] = float(b.pos.x); o[1] = float(b.pos.y); o[2] = float(b.pos.z);
    o[3] = float(rpy.x);   o[4] = float(rpy.y);   o[5] = float(rpy.z);
    o[6] = float(b.vel.x); o[7] = float(b.vel.y); o[8] = float(b.vel.z);
    o[9] = float(w.x);     o[10] = float(w.y);    o[11] = float(w.z);
    return rpy;
}

// one obs row [12 kinematic | B x A action ring, oldest first] from registers
template <int A, int B>
__device__ __forceinline__ void write_row(float* row, const float o12[12], const float (&ring)[B][A], int head1) {
    if constexpr (A == 4) {
        float4* r4 = reinterpret_cast<float4*>(row);
        r4[0] = make_float4(o12[0], o12[1], o12[2], o12[3]);
        r4[1] = make_float4(o12[4], o12[5], o12[6], o12[7]);
        r4[2] = make_float4(o12[8], o12[9], o12[10], o12[11]);
#pragma unroll
        for (int p = 0; p < B; ++p) {          // physical slot p -> logical position k
            int k = p - head1;
            k += k < 0 ? B : 0;
            r4[3 + k] = make_float4(ring[p][0], ring[p][1], ring[p][2], ring[p][3]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) row[k] = o12[k];
#pragma unroll
        for (int p = 0; p < B; ++p) {
            int k = p - head1;
            k += k < 0 ? B : 0;
#pragma unroll
            for (int j = 0; j < A; ++j) row[12 + k * A + j] = ring[p][j];
        }
    }
}

// generic-B variant: the ring part is copied from HBM in logical order (slot head1 = oldest);
// the newest entry (logical B-1) is this step's action
template <int A>
__device__ __forceinline__ void write_row_generic(float* __restrict__ row, const float o12[12],
                                                  const float* __restrict__ ring, int B, int E, int e, int head1,
                                                  const float act[A], bool act_is_newest) {
#pragma unroll
    for (int k = 0; k < 12; ++k) row[k] = o12[k];
    // chunks of 8 slots: all loads of a chunk in flight before its stores
    constexpr int CH = 8;
    int slot = head1;
    for (int k0 = 0; k0 < B; k0 += CH) {
        float v[CH][A];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int k = k0 + c;
#pragma unroll
            for (int j = 0; j < A; ++j)
                v[c][j] = k < B ? ((act_is_newest && k == B - 1) ? act[j] : ring[(size_t(slot) * E + e) * A + j]) : 0.0f;
            slot = slot + 1 == B ? 0 : slot + 1;
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int k = k0 + c;
            if (k < B)
#pragma unroll
                for (int j = 0; j < A; ++j) row[12 + k * A + j] = v[c][j];
        }
    }
}

// DSLPIDControl.computeControl (control/DSLPIDControl.py:82-259) for the HoverAviary PID / VEL /
// ONE_D_PID action types (BaseRLAviary.py:193-235): once per env.step, on the state at the
// start of the step.  ctl = last_rpy 3, integral_pos_e 3, integral_rpy_e 3 (in/out).  The
// scipy Euler round trip of the target rotation (:205, :242-244) is the identity on a proper
// rotation, so the target basis is used directly (oracle/oracle.c orc_dslpid, pinned by
// tests/golden/pid_golden.npz).
template <typename Real, int CTL>
__device__ __forceinline__ void dslpid_rpm(const HoverConst<Real>& C, const Body<Real>& b, const float* act,
                                           Real ctl[HF_NPID], Real rpm[4]) {
    const M3<Real> R = rot(b.q);
    const V3<Real> rpy = euler_xyz(b.q);   // accurate: the D term scales its error by 6e5
    V3<Real> tp, tv = v3(Real(0), Real(0), Real(0));
    Real tyaw = 0;
    if constexpr (CTL == ADRP_ACT_PID) {
        // _calculateNextStep(pos, action, step_size=1) (BaseAviary.py:1112-1160)
        const V3<Real> d = v3(Real(act[0]) - b.pos.x, Real(act[1]) - b.pos.y, Real(act[2]) - b.pos.z);
        const Real dist = sqrt_(dot(d, d));
        tp = dist <= Real(1) ? v3(Real(act[0]), Real(act[1]), Real(act[2])) : b.pos + (Real(1) / dist) * d;
    } else if constexpr (CTL == ADRP_ACT_VEL) {
        // target_vel = SPEED_LIMIT*|a3|*a[0:3]/|a[0:3]| in float32 (float32 action, NEP 50)
#pragma clang fp contract(off)
        tp = b.pos;
        tyaw = rpy.z;
        // correctly rounded float32 sqrt / division through float64 (53 >= 2*24 + 2 bits)
        const float n = float(sqrt(double(act[0] * act[0] + act[1] * act[1] + act[2] * act[2])));
        const float s = C.speed_limit * fabsf(act[3]);
        if (n != 0.0f) {
            const double dn = double(n);
            tv = v3(Real(s * float(double(act[0]) / dn)), Real(s * float(double(act[1]) / dn)),
                    Real(s * float(double(act[2]) / dn)));
        }
    } else {   // ONE_D_PID: target_pos = pos + 0.1*[0, 0, a]
        tp = v3(b.pos.x, b.pos.y, b.pos.z + Real(0.1) * Real(act[0]));
    }
    // _dslPIDPositionControl (:149-208)
    constexpr Real PF[3] = {Real(.4), Real(.4), Real(1.25)}, IF[3] = {Real(.05), Real(.05), Real(.05)},
                   DF[3] = {Real(.2), Real(.2), Real(.5)};
    const Real pe[3] = {tp.x - b.pos.x, tp.y - b.pos.y, tp.z - b.pos.z};
    const Real ve[3] = {tv.x - b.vel.x, tv.y - b.vel.y, tv.z - b.vel.z};
    Real tt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        Real ip = ctl[3 + k] + pe[k] * C.ctrl_dt;
        ip = ip < Real(-2) ? Real(-2) : (ip > Real(2) ? Real(2) : ip);
        if (k == 2) ip = ip < Real(-0.15) ? Real(-0.15) : (ip > Real(0.15) ? Real(0.15) : ip);
        ctl[3 + k] = ip;
        tt[k] = PF[k] * pe[k] + IF[k] * ip + DF[k] * ve[k];
    }
    tt[2] += C.pid_grav;
    Real sc = tt[0] * R.a02 + tt[1] * R.a12 + tt[2] * R.a22;
    sc = sc < Real(0) ? Real(0) : sc;
    const Real thrust = (sqrt_(sc * C.pid_inv4kf) - Real(4070.3)) * Real(1.0 / 0.2685);
    const V3<Real> ttv = v3(tt[0], tt[1], tt[2]);
    const V3<Real> zax = rsqrt_(dot(ttv, ttv)) * ttv;
    Real sy, cy;
    sincos_(tyaw, &sy, &cy);
    const V3<Real> yc = cross(zax, v3(cy, sy, Real(0)));
    const V3<Real> yax = rsqrt_(dot(yc, yc)) * yc;
    const V3<Real> xax = cross(yax, zax);
    // _dslPIDAttitudeControl (:212-259): rot_e = vee(Rt^T R - R^T Rt)
    const V3<Real> c0 = v3(R.a00, R.a10, R.a20), c1 = v3(R.a01, R.a11, R.a21), c2 = v3(R.a02, R.a12, R.a22);
    const Real rot_e[3] = {dot(zax, c1) - dot(c2, yax), dot(xax, c2) - dot(c0, zax), dot(yax, c0) - dot(c1, xax)};
    const Real cur[3] = {rpy.x, rpy.y, rpy.z};
    constexpr Real PT[3] = {Real(70000), Real(70000), Real(60000)}, IT[3] = {Real(0), Real(0), Real(500)},
                   DT[3] = {Real(20000), Real(20000), Real(12000)};
    Real tq[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const Real rr_e = -(cur[k] - ctl[k]) * C.ctrl_hz;
        ctl[k] = cur[k];
        Real ir = ctl[6 + k] - rot_e[k] * C.ctrl_dt;
        ir = ir < Real(-1500) ? Real(-1500) : (ir > Real(1500) ? Real(1500) : ir);
        if (k < 2) ir = ir < Real(-1) ? Real(-1) : (ir > Real(1) ? Real(1) : ir);
        ctl[6 + k] = ir;
        const Real t = -PT[k] * rot_e[k] + DT[k] * rr_e + IT[k] * ir;
        tq[k] = t < Real(-3200) ? Real(-3200) : (t > Real(3200) ? Real(3200) : t);
    }
    // CF2X mixer [[-.5,-.5,-1],[-.5,.5,1],[.5,.5,-1],[.5,-.5,1]], PWM clip, PWM -> RPM
    const Real hr = Real(0.5) * tq[0], hp = Real(0.5) * tq[1];
    const Real pwm[4] = {thrust - hr - hp - tq[2], thrust - hr + hp + tq[2], thrust + hr + hp - tq[2],
                         thrust + hr - hp + tq[2]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const Real p = pwm[i] < Real(20000) ? Real(20000) : (pwm[i] > Real(65535) ? Real(65535) : pwm[i]);
        rpm[i] = Real(0.2685) * p + Real(4070.3);
    }
}

template <typename Real>
__device__ __forceinline__ void load_body(const HoverArgs<Real>& a, int e, Body<Real>& b, bool lag, bool drag,
                                          bool dyn) {
    const int E = a.E;
    const Real* f = a.f;
    b.pos = v3(f[(HF_POS + 0) * E + e], f[(HF_POS + 1) * E + e], f[(HF_POS + 2) * E + e]);
    b.q = {f[(HF_QUAT + 0) * E + e], f[(HF_QUAT + 1) * E + e], f[(HF_QUAT + 2) * E + e], f[(HF_QUAT + 3) * E + e]};
    b.vel = v3(f[(HF_VEL + 0) * E + e], f[(HF_VEL + 1) * E + e], f[(HF_VEL + 2) * E + e]);
    b.w = v3(f[(HF_OMEGA + 0) * E + e], f[(HF_OMEGA + 1) * E + e], f[(HF_OMEGA + 2) * E + e]);
    if (lag) b.ql = {f[(HF_LINK_QUAT + 0) * E + e], f[(HF_LINK_QUAT + 1) * E + e], f[(HF_LINK_QUAT + 2) * E + e],
                     f[(HF_LINK_QUAT + 3) * E + e]};
    else b.ql = b.q;
#pragma unroll
    for (int i = 0; i < 4; ++i) b.prev_rpm[i] = drag ? f[(HF_LAST_RPM + i) * E + e] : Real(0);
    if (dyn) b.angv = v3(f[(HF_ANGV + 0) * E + e], f[(HF_ANGV + 1) * E + e], f[(HF_ANGV + 2) * E + e]);
    else b.angv = v3(Real(0), Real(0), Real(0));
}

template <typename Real>
__device__ __forceinline__ void store_body(const HoverArgs<Real>& a, int e, const Body<Real>& b, bool lag,
                                           bool drag, bool dyn) {
    const int E = a.E;
    Real* f = a.f;
    f[(HF_POS + 0) * E + e] = b.pos.x; f[(HF_POS + 1) * E + e] = b.pos.y; f[(HF_POS + 2) * E + e] = b.pos.z;
    f[(HF_QUAT + 0) * E + e] = b.q.x; f[(HF_QUAT + 1) * E + e] = b.q.y;
    f[(HF_QUAT + 2) * E + e] = b.q.z; f[(HF_QUAT + 3) * E + e] = b.q.w;
    f[(HF_VEL + 0) * E + e] = b.vel.x; f[(HF_VEL + 1) * E + e] = b.vel.y; f[(HF_VEL + 2) * E + e] = b.vel.z;
    f[(HF_OMEGA + 0) * E + e] = b.w.x; f[(HF_OMEGA + 1) * E + e] = b.w.y; f[(HF_OMEGA + 2) * E + e] = b.w.z;
    if (lag) {
        f[(HF_LINK_QUAT + 0) * E + e] = b.ql.x; f[(HF_LINK_QUAT + 1) * E + e] = b.ql.y;
        f[(HF_LINK_QUAT + 2) * E + e] = b.ql.z; f[(HF_LINK_QUAT + 3) * E + e] = b.ql.w;
    }
    if (drag) {
#pragma unroll
        for (int i = 0; i < 4; ++i) f[(HF_LAST_RPM + i) * E + e] = b.prev_rpm[i];
    }
    if (dyn) {
        f[(HF_ANGV + 0) * E + e] = b.angv.x; f[(HF_ANGV + 1) * E + e] = b.angv.y; f[(HF_ANGV + 2) * E + e] = b.angv.z;
    }
}

// ------------------------------------------------------------------------------------------
// env.step kernel: lane = env; B (ring length) is a template parameter so the ring lives
// in registers
// ------------------------------------------------------------------------------------------
// obs rows staged in LDS, then written as one contiguous, fully coalesced block of
// 64 rows (the row-per-lane float4 stores leave partial 64-B lines: +18 % write traffic)
constexpr int kRowF4 = 18;        // 72 floats = 18 float4 per obs row (A = 4, B = 15)

template <int A, int B>
__device__ __forceinline__ void stage_row(float4* lds_row, const float o12[12], const float (&ring)[B][A], int head1) {
    lds_row[0] = make_float4(o12[0], o12[1], o12[2], o12[3]);
    lds_row[1] = make_float4(o12[4], o12[5], o12[6], o12[7]);
    lds_row[2] = make_float4(o12[8], o12[9], o12[10], o12[11]);
#pragma unroll
    for (int p = 0; p < B; ++p) {
        int k = p - head1;
        k += k < 0 ? B : 0;
        lds_row[3 + k] = make_float4(ring[p][0], ring[p][1], ring[p][2], ring[p][3]);
    }
}

// B == 0: runtime ring length a.B;  SC > 0: compile-time sub-step count (loop fully unrolled);
// STG: LDS-staged obs rows (needs A == 4, B == 15 and every lane of the block live);
// CTL: 0 (RPM / ONE_D_RPM actions) or ADRP_ACT_PID / _VEL / _ONE_D_PID (fused DSLPIDControl);
// HELP (STG + auto-reset only): a second wave per block computes the next-episode initial state
// of the first wave's envs (3 Philox draws, quaternion, Euler obs: ~1/4 of a wave's instruction
// stream at E = 4096, where nearly every wave has a done lane) on another SIMD, into LDS; the
// chain wave, issue-bound at one instruction per 4 cycles, only copies it for its done lanes.
// SYS: the action rows live in host-mapped memory written by the host while the kernel runs
// (hover_persist.h): 1 = they are read with system-scope loads, which no GPU cache serves; 2 = the
// caller already read them (pre[0..A-1], the persistent kernel's line mode).
template <typename Real, int PH, int A, int B, int SC, bool STG = false, int CTL = 0, bool HELP = false, int SYS = 0>
__device__ __forceinline__ void hover_step_body(const HoverArgs<Real>& a, const HoverConst<Real>& C,
                                                const float* pre = nullptr) {
    constexpr int BR = B > 0 ? B : 1;
    constexpr bool DRAG = (PH == ADRP_PHYS_PYB_DRAG || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    constexpr bool DYN = (PH == ADRP_PHYS_DYN);
    static_assert(!HELP || STG, "the reset helper wave pairs with the staged (all lanes live) kernel");
    __shared__ Real rs_body[HELP ? kResetFields * kStepBlock : 1];
    __shared__ float rs_obs[HELP ? 12 * kStepBlock : 1];
    __shared__ float4 rows[STG ? kStepBlock * kRowF4 : 1];
    // ANG: the obs row's pitch / yaw are computed by two more helper waves from the chain's final
    // quaternion (LDS) while the chain computes the roll: the chain's tail holds one of the three
    // float64 atan2-class evaluations instead of three
    constexpr bool ANG = HELP && angle_helpers<Real>();
    __shared__ Real ang_q[ANG ? 4 * kStepBlock : 1];
    __shared__ Real ang_p[ANG ? kStepBlock : 1];
    __shared__ float ang_y[ANG ? kStepBlock : 1];
    // the block's coalesced copy-out dealt over its waves: float4 columns [cb(w), cb(w + 1)) of the
    // rows; with the angle helpers the chain wave takes 3 of the 18, the helpers 5 each
    constexpr int kWaves = HELP ? 1 + help_waves<Real>() : 1;
    constexpr auto cb = [](int w) { return w == 0 ? 0 : (w >= kWaves ? kRowF4 : (kWaves == 2 ? kRowF4 / 2 : 5 * w - 2)); };
    if constexpr (HELP) {
        if (ANG && threadIdx.x >= 2 * kStepBlock) {   // angle helpers: pitch (wave 2), yaw (wave 3)
            const int tl = threadIdx.x & (kStepBlock - 1), wv = threadIdx.x / kStepBlock;
            __syncthreads();   // A: the chain's final quaternion
            const Q4<Real> q = {ang_q[tl], ang_q[kStepBlock + tl], ang_q[2 * kStepBlock + tl], ang_q[3 * kStepBlock + tl]};
            if (wv == 2) ang_p[tl] = euler_pitch_u(q);
            else ang_y[tl] = float(euler_yaw_u(q));
            __syncthreads();   // C: pitch and yaw
            __syncthreads();   // B: the final rows
            float4* dst = reinterpret_cast<float4*>(a.obs) + size_t(blockIdx.x) * kStepBlock * kRowF4;
            for (int k = cb(wv); k < cb(wv + 1); ++k) store_out(dst + tl + kStepBlock * k, rows[tl + kStepBlock * k]);
            return;
        }
        if (threadIdx.x >= kStepBlock) {
            const int tl = threadIdx.x - kStepBlock;
            const int he = blockIdx.x * kStepBlock + tl;
            const int E = a.E;
            // the action ring: its part of the obs row is independent of the physics, so this
            // wave loads it, stages it in LDS and appends the action (deque.append)
            const float4 av = reinterpret_cast<const float4*>(a.act)[he];
            float rg[BR][4];    // plain floats: float4 struct copies under a select went to scratch
#pragma unroll
            for (int p = 0; p < B; ++p) {
                const float4 v = reinterpret_cast<const float4*>(a.ring)[size_t(p) * E + he];
                rg[p][0] = v.x; rg[p][1] = v.y; rg[p][2] = v.z; rg[p][3] = v.w;
            }
            const int32_t head = a.ist[HI_RING_HEAD * E + he];
            int32_t hsc = 0, hep = a.ist[HI_EPISODE * E + he];
            Body<Real> rb;
            hover_reset_state(a, C, he, rb, hsc, hep);
            float o[12];
            hover_obs12(C, rb, o);
            const Real v[kResetFields] = {rb.pos.x, rb.pos.y, rb.pos.z, rb.q.x, rb.q.y, rb.q.z, rb.q.w,
                                          rb.vel.x, rb.vel.y, rb.vel.z, rb.w.x, rb.w.y, rb.w.z,
                                          rb.angv.x, rb.angv.y, rb.angv.z};
#pragma unroll
            for (int k = 0; k < kResetFields; ++k) rs_body[k * kStepBlock + tl] = v[k];
#pragma unroll
            for (int k = 0; k < 12; ++k) rs_obs[k * kStepBlock + tl] = o[k];
            // ring part of the obs row, oldest first; the appended action is the newest entry.
            // Every env appends once per env.step and resets keep the ring, so the head is the
            // same for every env in practice: then the slot -> row position map is scalar.
            float4* my = rows + tl * kRowF4;
            const int hu = __builtin_amdgcn_readfirstlane(head);
            if (__all(head == hu)) {
                const int h1 = hu + 1 == B ? 0 : hu + 1;
#pragma unroll
                for (int p = 0; p < B; ++p) {
                    const int k = p >= h1 ? p - h1 : p - h1 + B;
                    my[3 + k] = make_float4(rg[p][0], rg[p][1], rg[p][2], rg[p][3]);
                }
                my[3 + B - 1] = av;
            } else {
                const int h1 = head + 1 == B ? 0 : head + 1;
#pragma unroll
                for (int p = 0; p < B; ++p) {
                    int k = p - h1;
                    k += k < 0 ? B : 0;
                    const bool hit = p == head;
                    my[3 + k] = make_float4(hit ? av.x : rg[p][0], hit ? av.y : rg[p][1], hit ? av.z : rg[p][2],
                                            hit ? av.w : rg[p][3]);
                }
            }
            reinterpret_cast<float4*>(a.ring)[size_t(head) * E + he] = av;
            __syncthreads();   // A: reset states and ring rows in LDS
            if constexpr (ANG) __syncthreads();   // C
            __syncthreads();   // B: the chain wave's kinematic parts and reset rows
            // this wave's part of the block's coalesced copy-out
            float4* dst = reinterpret_cast<float4*>(a.obs) + size_t(blockIdx.x) * kStepBlock * kRowF4;
#pragma unroll
            for (int k = cb(1); k < cb(2); ++k) store_out(dst + tl + kStepBlock * k, rows[tl + kStepBlock * k]);
            return;
        }
    }
    const int E = a.E;
    // SPLIT (a step of ONE env, BASELINE config 1: launched or persistent): every lane of the wave runs
    // env 0 (the same inputs, the same code: the duplicate stores write the same values) so that three
    // lanes can take the three obs angles at once; contacts are counted by lane 0 alone
    const bool split = ADRP_PERSIST_SPLIT && !STG && !HELP && E == 1;
    const int e = split ? 0 : int(blockIdx.x) * kStepBlock + int(threadIdx.x);
    const int D = B > 0 ? 12 + B * A : a.D;
    if (e >= E) return;
    RACE_MARK(t0);
    // ---- issue every load up front: action, the whole ring, ints, state ----
    float act[A];
    if constexpr (SYS == 2) {
#pragma unroll
        for (int j = 0; j < A; ++j) act[j] = pre[j];
    } else if constexpr (SYS == 1) {
        uint32_t* sa = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(a.act)) + size_t(e) * A;
#pragma unroll
        for (int j = 0; j < A; ++j)
            act[j] = __uint_as_float(__hip_atomic_load(sa + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    } else if constexpr (A == 4) {
        const float4 v = reinterpret_cast<const float4*>(a.act)[e];
        act[0] = v.x; act[1] = v.y; act[2] = v.z; act[3] = v.w;
    } else {
#pragma unroll
        for (int j = 0; j < A; ++j) act[j] = a.act[e * A + j];
    }
    float ring[BR][A];
#pragma unroll
    for (int p = 0; p < (HELP ? 0 : B); ++p) {   // (no-op for B == 0; HELP: the helper wave's job)
        if constexpr (A == 4) {
            const float4 v = reinterpret_cast<const float4*>(a.ring)[size_t(p) * E + e];
            ring[p][0] = v.x; ring[p][1] = v.y; ring[p][2] = v.z; ring[p][3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < A; ++j) ring[p][j] = a.ring[(size_t(p) * E + e) * A + j];
        }
    }
    int32_t sc = a.ist[HI_STEP * E + e], ep = a.ist[HI_EPISODE * E + e];
    const int32_t head = a.ist[HI_RING_HEAD * E + e];
    const bool lag = C.link_lag && !DYN;
    Body<Real> b;
    load_body(a, e, b, lag, DRAG, DYN);
    // ---- _preprocessAction: RPM = HOVER_RPM * (1 + 0.05 a), the gain in float32 (NEP 50),
    //      or the DSLPIDControl output for the PID action types ----
    Real rpm[4];
    if constexpr (CTL != 0) {
        static_assert(A == (CTL == ADRP_ACT_PID ? 3 : CTL == ADRP_ACT_VEL ? 4 : 1), "PID action width");
        Real ctl[HF_NPID];
#pragma unroll
        for (int k = 0; k < HF_NPID; ++k) ctl[k] = a.f[(HF_PID + k) * E + e];
        dslpid_rpm<Real, CTL>(C, b, act, ctl, rpm);
#pragma unroll
        for (int k = 0; k < HF_NPID; ++k) a.f[(HF_PID + k) * E + e] = ctl[k];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) rpm[i] = C.hover_rpm * Real(rpm_gain(act[A == 1 ? 0 : i]));
    }
    // ---- sub-step loop (BaseAviary.py:347-376) ----
    bool touched = false;
#ifdef ADRP_RACE_TIMING
    // loads landed: the rpm gains and the state are consumed by the first sub-step
    __builtin_amdgcn_s_waitcnt(0);
#endif
    RACE_MARK(t1);
    if constexpr (DYN) {
        if constexpr (SC > 0) {
#pragma unroll
            for (int s = 0; s < SC; ++s) dyn_substep(C, b, rpm);
        } else {
            for (int s = 0; s < C.S; ++s) dyn_substep(C, b, rpm);
        }
    } else {
        Real sum_f = 0, t2 = 0;
        V3<Real> P = v3(Real(0), Real(0), Real(0));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const Real r2 = rpm[i] * rpm[i];
            const Real f = r2 * C.kf;
            sum_f += f;
            P = P + v3(f * C.px[i], f * C.py[i], f * C.pz[i]);
            t2 += (i & 1) ? -r2 : r2;
        }
        const Real tau_z = t2 * C.km;    // KM*(rpm0^2 - rpm1^2 + rpm2^2 - rpm3^2), IROS sign
        M3<Real> R = rot_fm(b.q);
        M3<Real> Rs = lag ? rot_fm(b.ql) : R;
        // the chain's constants in VGPRs for the whole loop (fp64: no 64-bit literal operands)
        ChainK<Real> K = chain_consts<Real>();
        HoverConst<Real> Cp = C;
        if constexpr (sizeof(Real) == 8) {
            pin_all(K);
            pin(Cp.dt); pin(Cp.mass); pin(Cp.gravity); pin(Cp.inv_mass); pin(Cp.ang_max);
            pin(Cp.ixx); pin(Cp.iyy); pin(Cp.izz); pin(Cp.inv_ixx); pin(Cp.inv_iyy); pin(Cp.inv_izz);
            pin(Cp.coll_hh); pin(Cp.coll_r); pin(Cp.coll_zoff);
        }
        Real wn = hsqrt_nn_(dot(b.w, b.w), K);
        auto substep = [&]() {
            touched |= pyb_substep<Real, PH>(Cp, b, R, Rs, rpm, sum_f, P, tau_z, wn, K);
#pragma unroll
            for (int i = 0; i < 4; ++i) b.prev_rpm[i] = rpm[i];  // last_clipped_action
        };
        if constexpr (SC > 0) {
#pragma unroll
            for (int s = 0; s < SC; ++s) substep();
        } else {
            for (int s = 0; s < C.S; ++s) substep();
        }
    }
    RACE_MARK(t2);
    if (touched && a.contact_count && (!split || threadIdx.x == 0)) atomicAdd(a.contact_count, 1);
    // ---- action ring: append this action at `head` (deque.append, BaseRLAviary.py:187) ----
    if constexpr (HELP) {
        // the helper wave appends
    } else if constexpr (A == 4)
        reinterpret_cast<float4*>(a.ring)[size_t(head) * E + e] = make_float4(act[0], act[1], act[2], act[3]);
    else
#pragma unroll
        for (int j = 0; j < A; ++j) a.ring[(size_t(head) * E + e) * A + j] = act[j];
    const int BB = B > 0 ? B : a.B;                    // ring length (runtime for the generic kernel)
    const int head1 = head + 1 == BB ? 0 : head + 1;
    // ---- obs / reward / terminated / truncated (HoverAviary.py:68-117) ----
    float o12[12];
    V3<Real> rpy;
    if constexpr (ANG) {
        const int tl = threadIdx.x;
        ang_q[tl] = b.q.x; ang_q[kStepBlock + tl] = b.q.y; ang_q[2 * kStepBlock + tl] = b.q.z;
        ang_q[3 * kStepBlock + tl] = b.q.w;
        __syncthreads();   // A: the quaternion out; the reset helper's states and ring rows in
        rpy.x = euler_roll_u(b.q);
        const V3<Real> w = C.physics == ADRP_PHYS_DYN ? b.angv : b.w;   // hover_obs12's row, pitch / yaw below
        o12[0] = float(b.pos.x); o12[1] = float(b.pos.y); o12[2] = float(b.pos.z); o12[3] = float(rpy.x);
        o12[6] = float(b.vel.x); o12[7] = float(b.vel.y); o12[8] = float(b.vel.z);
        o12[9] = float(w.x);     o12[10] = float(w.y);    o12[11] = float(w.z);
    } else if (split) {
        rpy = hover_obs12_split(C, b, o12);
    } else {
        rpy = hover_obs12(C, b, o12);
    }
    const Real dx = C.target[0] - b.pos.x, dy = C.target[1] - b.pos.y, dz = C.target[2] - b.pos.z;
    const Real d2 = dx * dx + dy * dy + dz * dz;
    const Real r = Real(2) - d2 * d2;
    a.rew[e] = float(r > Real(0) ? r : Real(0));
    const bool te = d2 < Real(1e-8);   // |target - pos| < 1e-4
    bool tr = fabs_(b.pos.x) > Real(1.5) || fabs_(b.pos.y) > Real(1.5) || b.pos.z > Real(2.0) ||
              fabs_(rpy.x) > Real(0.4) || sc >= C.trunc_steps;
    if constexpr (ANG) {
        __syncthreads();   // C: the helpers' pitch and yaw
        rpy.y = ang_p[threadIdx.x];
        o12[4] = float(rpy.y);
        o12[5] = ang_y[threadIdx.x];
    }
    tr = tr || fabs_(rpy.y) > Real(0.4);
    a.term[e] = te;
    a.trunc[e] = tr;
    sc += C.S;
    const bool done = a.autoreset && (te || tr);
    RACE_MARK(t3);
#ifdef ADRP_RACE_TIMING
    const unsigned long long dmask = __ballot(done);
    uint64_t t4 = 0;
#endif
    if constexpr (STG) {
        // The obs row is assembled in LDS (18 float4 per lane, no padding: the copy-out
        // reads contiguous float4s at immediate offsets) and leaves as one coalesced block.
        static_assert(A == 4 && B == 15, "staged rows: 72-float rows only");
        float4* my = rows + threadIdx.x * kRowF4;
        // Every env appends once per env.step and resets keep the ring, so the ring head is
        // the same for every env in practice: then the slot -> row position map is scalar
        // and the appended action simply overwrites the newest position.
        const int hu = __builtin_amdgcn_readfirstlane(head);
        if constexpr (HELP) {
            // the ring part of the row is staged by the helper wave
        } else if (__all(head == hu)) {
            const int h1 = hu + 1 == B ? 0 : hu + 1;
#pragma unroll
            for (int p = 0; p < B; ++p) {
                const int k = p >= h1 ? p - h1 : p - h1 + B;
                my[3 + k] = make_float4(ring[p][0], ring[p][1], ring[p][2], ring[p][3]);
            }
            my[3 + B - 1] = make_float4(act[0], act[1], act[2], act[3]);
        } else {
#pragma unroll
            for (int p = 0; p < B; ++p) {
                const bool hit = p == head;
#pragma unroll
                for (int j = 0; j < A; ++j) ring[p][j] = hit ? act[j] : ring[p][j];
            }
            stage_row<A, B>(my, o12, ring, head1);
        }
        my[0] = make_float4(o12[0], o12[1], o12[2], o12[3]);
        my[1] = make_float4(o12[4], o12[5], o12[6], o12[7]);
        my[2] = make_float4(o12[8], o12[9], o12[10], o12[11]);
        if constexpr (HELP && !ANG) __syncthreads();   // A: the helper wave's reset states
        if (done) {
            if (a.tobs) {   // terminal obs = the row just staged (this lane's own LDS row)
                float4 t[kRowF4];
#pragma unroll
                for (int k = 0; k < kRowF4; ++k) t[k] = my[k];
                float4* trow = reinterpret_cast<float4*>(a.tobs + size_t(e) * D);
#pragma unroll
                for (int k = 0; k < kRowF4; ++k) trow[k] = t[k];
            }
            if constexpr (HELP) {   // BaseAviary.reset from the helper's LDS copy
                const int t = threadIdx.x;
                Real v[kResetFields];
#pragma unroll
                for (int k = 0; k < kResetFields; ++k) v[k] = rs_body[k * kStepBlock + t];
                b.pos = v3(v[0], v[1], v[2]);
                b.q = {v[3], v[4], v[5], v[6]};
                b.ql = b.q;
                b.vel = v3(v[7], v[8], v[9]);
                b.w = v3(v[10], v[11], v[12]);
                b.angv = v3(v[13], v[14], v[15]);
#pragma unroll
                for (int i = 0; i < 4; ++i) b.prev_rpm[i] = Real(0);
                sc = 0;
                ep += 1;
#pragma unroll
                for (int k = 0; k < 12; ++k) o12[k] = rs_obs[k * kStepBlock + t];
            } else {
                hover_reset_state(a, C, e, b, sc, ep);
                hover_obs12(C, b, o12);      // the reset keeps the ring: only the kinematic part changes
            }
            my[0] = make_float4(o12[0], o12[1], o12[2], o12[3]);
            my[1] = make_float4(o12[4], o12[5], o12[6], o12[7]);
            my[2] = make_float4(o12[8], o12[9], o12[10], o12[11]);
        }
        RACE_SET(t4);
        // the state leaves first: its registers are free before the copy-out (holding both
        // spilled the copy-out buffer to scratch)
        store_body(a, e, b, lag, DRAG, DYN);
        a.ist[HI_STEP * E + e] = sc;
        a.ist[HI_EPISODE * E + e] = ep;
        a.ist[HI_RING_HEAD * E + e] = head1;
        __syncthreads();
        float4* dst = reinterpret_cast<float4*>(a.obs) + size_t(blockIdx.x) * kStepBlock * kRowF4;
        constexpr int KC = cb(1);   // HELP: the helper waves copy the other columns
#pragma unroll
        for (int k = 0; k < KC; ++k) store_out(dst + threadIdx.x + kStepBlock * k, rows[threadIdx.x + kStepBlock * k]);
    } else {
#pragma unroll
        for (int p = 0; p < B; ++p) {
            const bool hit = p == head;
#pragma unroll
            for (int j = 0; j < A; ++j) ring[p][j] = hit ? act[j] : ring[p][j];
        }
        if (done) {
            if (a.tobs) {
                if constexpr (B > 0) write_row<A, B>(a.tobs + size_t(e) * D, o12, ring, head1);
                else write_row_generic<A>(a.tobs + size_t(e) * D, o12, a.ring, a.B, E, e, head1, act, true);
            }
            hover_reset_state(a, C, e, b, sc, ep);
            if (split) hover_obs12_split(C, b, o12);
            else hover_obs12(C, b, o12);
        }
        RACE_SET(t4);
        if constexpr (B > 0) write_row<A, B>(a.obs + size_t(e) * D, o12, ring, head1);
        else write_row_generic<A>(a.obs + size_t(e) * D, o12, a.ring, a.B, E, e, head1, act, true);
    }
    RACE_MARK(t5);
    if constexpr (!STG) {
        store_body(a, e, b, lag, DRAG, DYN);
        a.ist[HI_STEP * E + e] = sc;
        a.ist[HI_EPISODE * E + e] = ep;
        a.ist[HI_RING_HEAD * E + e] = head1;
    }
#ifdef ADRP_RACE_TIMING
    RACE_MARK(t6);
    if (threadIdx.x == 0) {   // [loads, sub-steps, obs+flags, reset, obs row, state stores, total, -, waves]
        RACE_ACC(0, t1 - t0); RACE_ACC(1, t2 - t1); RACE_ACC(2, t3 - t2); RACE_ACC(3, t4 - t3);
        RACE_ACC(4, t5 - t4); RACE_ACC(5, t6 - t5); RACE_ACC(6, t6 - t0); RACE_ACC(8, 1);
        RACE_ACC(7, __popcll(dmask));
        if (dmask) atomicAdd(&g_race_phase[9], 1ull);
    }
#endif
}

// Arguments the step needs at wave start are separate scalars so the CP preloads them into
// SGPRs (-amdgpu-kernarg-preload-count); the rest (used at the end) is one aggregate.
template <typename Real>
struct HoverTail {
    const HoverConst<Real>* c;
    const HoverReset<Real>* r;
    uint8_t* term;
    uint8_t* trunc;
    float* tobs;
    int32_t* contact_count;
    uint64_t seed;
    int64_t env_offset;
    int B, D, autoreset;
};

// DEF: compiled-in cf2x_consts (the reference default) instead of the device block.
// STG: LDS-staged coalesced obs rows (host: only when E % kStepBlock == 0).
// Launch with kStepBlock threads per workgroup.
template <typename Real, int PH, int A, int B, bool DEF, bool STG = false, int CTL = 0, bool HELP = false>
__global__ void __launch_bounds__(256) hover_step_kernel(Real* f, float* ring, int32_t* ist, const float* act,
                                                         float* obs, float* rew, int E, HoverTail<Real> t) {
    HoverArgs<Real> a;
    a.c = t.c; a.r = t.r;
    a.f = f; a.ring = ring; a.ist = ist; a.act = act; a.obs = obs; a.rew = rew;
    a.term = t.term; a.trunc = t.trunc; a.tobs = t.tobs; a.mask = nullptr; a.contact_count = t.contact_count;
    a.seed = t.seed; a.env_offset = t.env_offset;
    a.E = E; a.B = t.B; a.D = t.D; a.autoreset = t.autoreset;
    if constexpr (DEF) {
        constexpr HoverConst<Real> C = cf2x_consts<Real>(PH);
        hover_step_body<Real, PH, A, B, C.S, STG, CTL, HELP>(a, C);
    } else {
        hover_step_body<Real, PH, A, B, 0, STG, CTL, HELP>(a, *a.c);
    }
}

// reset kernel (BaseAviary.reset -> _housekeeping -> _computeObs); ring is NOT cleared (Q21)
template <typename Real, int A>
__global__ void __launch_bounds__(256) hover_reset_kernel(HoverArgs<Real> a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.E || (a.mask && !a.mask[e])) return;
    const HoverConst<Real>& C = *a.c;
    const int E = a.E;
    const bool dyn = C.physics == ADRP_PHYS_DYN;
    const bool drag = C.physics == ADRP_PHYS_PYB_DRAG || C.physics == ADRP_PHYS_PYB_GND_DRAG_DW;
    Body<Real> b;
    int32_t sc = a.ist[HI_STEP * E + e], ep = a.ist[HI_EPISODE * E + e];
    const int head = a.ist[HI_RING_HEAD * E + e];
    hover_reset_state(a, C, e, b, sc, ep);
    store_body(a, e, b, C.link_lag && !dyn, drag, dyn);
    a.ist[HI_STEP * E + e] = sc;
    a.ist[HI_EPISODE * E + e] = ep;
    float o12[12];
    hover_obs12(C, b, o12);
    const float none[A] = {};
    write_row_generic<A>(a.obs + size_t(e) * a.D, o12, a.ring, a.B, E, e, head, none, false);
}

}  // namespace adrp
