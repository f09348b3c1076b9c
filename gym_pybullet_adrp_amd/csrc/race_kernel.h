// race_kernel.h — MultiRaceAviary env.step as one fused launch (gfx950).
//
// One lane per drone: lane = env * G + drone, G = next power of two >= N, so the drones of
// an env sit in G adjacent lanes of one wave and exchange poses with __shfl (ds_bpermute,
// no LDS allocation): downwash every sub-step; rays, COMPETE obs/contacts and the
// per-env termination reduction once per env.step.  Per lane and env.step:
//   S x [ forces (motor, ground effect, drag, downwash, level1-3 disturbance) -> Bullet
//         floating-base step -> MellingerControl wrapper + firmware controllerMellinger +
//         PWM chain (500 Hz) ]
//   -> _gate_progress rays -> _computeObs (GJK range tests) -> elimination / terminated /
//   truncated -> RewardWrapper -> auto-reset.
// Reference: envs/MultiRaceAviary.py:171-270 (see oracle/race.c for the line-by-line map).
#pragma once

#include "../../include/adrp.h"
#include "adrp_device.h"
#include "commander.h"

namespace adrp {

constexpr uint32_t TAG_RACE_TRACK = 0x52540000u;
constexpr uint32_t TAG_RACE_DRONE = 0x52440000u;
constexpr uint32_t TAG_RACE_NOISE = 0x524e0000u;
constexpr uint32_t TAG_RACE_DIST = 0x52460000u;
constexpr int kRaceBlock = 64;      // drone lanes per block (one wave runs the sub-step chain)
constexpr int kRaceHelpers = 3;     // helper waves per block: the sub-step disturbance draws
constexpr int kRacePreS = 32;       // sub-steps per env.step whose draws fit the LDS table

// GJK call counts (global atomics from every lane that runs a GJK: they inflate the phase times, so
// they are a separate opt-in of the timing build)
#if defined(ADRP_RACE_TIMING) && defined(ADRP_RACE_GJK_STATS)
// this workgroup's GJK iterations (the four-lane kernel reports them in its "contacts" wave slot)
__shared__ unsigned int g_gjk_wave_iters;
#define GJK_STAT(n) do { atomicAdd(&g_gjk_wave_iters, (unsigned int)(n)); \
        atomicAdd(&g_race_phase[9], 1ull); atomicAdd(&g_race_phase[18], (unsigned long long)(n)); \
        atomicMax(&g_race_phase[19], (unsigned long long)(n)); \
        if (cut < Real(1e-3)) { atomicAdd(&g_race_phase[20], 1ull); atomicMax(&g_race_phase[21], (unsigned long long)(n)); } \
        if ((n) >= 48) atomicAdd(&g_race_phase[22], 1ull); \
        if (nout) *nout = (n); } while (0)
#else
#define GJK_STAT(n)
#endif

// per-drone SoA fields ([field][E*N]); env fields are replicated in every drone slot
enum RaceField {
    RF_POS = 0, RF_QUAT = 3, RF_VEL = 7, RF_OMEGA = 10, RF_RPM = 13, RF_PREV_RPM = 17, RF_ANGV = 21,
    RF_LINK_QUAT = 24, RF_LINK_POS = 28, RF_KIN_POS = 31, RF_PREV_RPY = 34, RF_PREV_VEL = 37,
    RF_LPF_D1 = 40, RF_LPF_D2 = 43, RF_I_ERR = 46, RF_I_ERR_M = 49, RF_PREV_OMEGA_ROLL = 52,
    RF_PREV_OMEGA_PITCH = 53, RF_PREV_SP_ROLL = 54, RF_PREV_SP_PITCH = 55, RF_CTL = 56, RF_MASS = 60,
    RF_INERTIA = 61, RF_GATE = 64, RF_OBST = 80, RF_WR_TARGET = 92, RF_WR_PREV = 95, RF_N = 98
};
enum RaceInt { RI_STEP = 0, RI_EPISODE, RI_TICK, RI_LAST_ATT, RI_LAST_POS, RI_TUMBLE, RI_GATE, RI_FLAGS, RI_WR_GATE, RI_N };

template <typename Real>
struct RaceConst {
    int N, S, physics, link_lag, compete, num_gates, num_obstacles, trunc_steps;
    int disturbances, reward_wrapper, obs_wrapper, random_gates, random_state, random_inertia, D, autoreset;
    int refine;   // support-function bounds for the pairs the centre-distance bounds leave open (ADRP_RACE_REFINE)
    Real dt, gravity, kf, km, hover_unused;
    Real px[4], py[4], pz[4];
    Real gnd_kf, prop_r4, gnd_clip, drag[3], dw1, dw2, dw3, prop_r;
    Real dyn_mass, dyn_inv_mass, dyn_i[3], dyn_inv_i[3], dyn_arm;   // Physics.DYN uses the IROS URDF M, J
    Real coll_hh, coll_r, coll_zoff, ang_max;
    Real gate_nom[ADRP_MAX_GATES][4];
    int gate_type[ADRP_MAX_GATES];
    Real obst_nom[ADRP_MAX_OBSTACLES][3];
    Real bounds[3];
    Real noise_std, dist_lo[3], dist_hi[3];
    Real gate_off[2], obst_off[2], pos_off[3][2], rot_off[3][2], inertia_off[4][2];
    Real init_pos[ADRP_MAX_DRONES][3], init_rpy[ADRP_MAX_DRONES][3], init_vel[ADRP_MAX_DRONES][3],
        init_pqr[ADRP_MAX_DRONES][3];
    Real race_mass, race_inertia[3];
    float lpf[5];   // gyro lpf2p b0, b1, b2, a1, a2 (host float, as the firmware's filter.c computes them)
    // nominal (loadURDF) attitude of every drone: quat_from_euler_fast(init_rpy * d2r) and its
    // euler_xyz_fast, written on the device by race_const_init_kernel after each upload (the
    // kernels' own transcendentals, so every reset / command init reads the same bits)
    Real nom_q[ADRP_MAX_DRONES][4], nom_rpy[ADRP_MAX_DRONES][3];
};

template <typename Real>
struct RaceArgs {
    const RaceConst<Real>* c;
    Real* f;             // [RF_N][E*N]
    int32_t* ist;        // [RI_N][E*N]
    const float* act;    // [E][N][4]
    float* obs;          // [E][N][D]
    float* rew;          // [E]
    uint8_t* term;
    uint8_t* trunc;
    float* tobs;         // [E][N][D] or null
    const uint8_t* mask; // reset mask or null
    const uint32_t* ticks; // tick-schedule bit tables (kTickTableN ticks each: att, then pos)
    float* cf;           // command mode: [ADRP_CMD_NF][E*N] (commander.h), else null
    int32_t* ci;         // [ADRP_CMD_NI][E*N]
    const int32_t* cmd;  // race_command_kernel: [E*N] ADRP_CMD_*
    const double* cargs; // [E*N][ADRP_CMD_ARGS]
    const double* inj_act;    // parity mode (adrp_set_noise): [E*N][S][4] action noise, or null (Philox)
    const double* inj_force;  // [E*N][S][3] disturbance force, or null
    uint64_t seed;
    int64_t env_offset;
    int E;
    uint32_t* mom_hash;  // diagnostics (adrp_set_diagnostics): [E*N] fw_moment_hash of the step, or null
    int16_t* mom_log;    // diagnostics level 2 (one-lane kernel): [E*N][S][3] int16 moments of every
    int32_t* mom_log_n;  //   firmware call of the step, in call order; [E*N] the number of calls
    // next-reset images (race_quad.h, race_refill_q4): what the auto-reset at the end of episode
    // img_ep[e] writes for env e, computed ahead of time; null when off
    Real* img_f;         // [RF_N][E*N]
    int32_t* img_i;      // [RI_N][E*N]
    float* img_row;      // [E*N][D] the reset obs rows
    int32_t* img_ep;     // [E] the episode the image is for, -1 none
    int32_t* reset_count;  // diagnostics: [2] auto-resets from an image / computed inline (four-lane kernel)
};

// The physical constants of the reference's race drone (cf2x.urdf at PYB_FREQ 500, BaseAviary.py:
// 117-128, 792-818): the float64 results of the host's race_const for that drone, so the host can
// check its runtime block against them bit for bit (race_is_cf2x, adrp.hip) and the four-lane
// kernel then compiles them in as literals (no SGPRs held or spilled across the sub-step loop).
template <typename Real>
__host__ __device__ constexpr void race_cf2x_phys(RaceConst<Real>& k) {
    k.dt = Real(1.0 / 500); k.gravity = Real(9.8); k.kf = Real(3.16e-10); k.km = Real(7.94e-12);
    k.px[0] = Real(0.028); k.px[1] = Real(-0.028); k.px[2] = Real(-0.028); k.px[3] = Real(0.028);
    k.py[0] = Real(0.028); k.py[1] = Real(0.028); k.py[2] = Real(-0.028); k.py[3] = Real(-0.028);
    k.pz[0] = Real(0); k.pz[1] = Real(0); k.pz[2] = Real(0); k.pz[3] = Real(0);
    k.gnd_kf = Real(3.16e-10 * 11.36859); k.prop_r4 = Real(0.0231348 / 4); k.gnd_clip = Real(0.03776371349209501);
    k.drag[0] = Real(9.1785e-7); k.drag[1] = Real(9.1785e-7); k.drag[2] = Real(1.0311e-6);
    k.dw1 = Real(2267.18); k.dw2 = Real(0.16); k.dw3 = Real(-0.11); k.prop_r = Real(0.0231348);
    k.dyn_mass = Real(0.03454); k.dyn_inv_mass = Real(1.0 / 0.03454);
    k.dyn_i[0] = Real(1.4e-5); k.dyn_i[1] = Real(1.4e-5); k.dyn_i[2] = Real(2.17e-5);
    k.dyn_inv_i[0] = Real(1.0 / 1.4e-5); k.dyn_inv_i[1] = Real(1.0 / 1.4e-5); k.dyn_inv_i[2] = Real(1.0 / 2.17e-5);
    k.dyn_arm = Real(0.028072139213105935);
    k.coll_hh = Real(0.5 * 0.025); k.coll_r = Real(0.06); k.coll_zoff = Real(0);
    k.ang_max = Real(0.5 * (3.14159265358979323846 / 2) * 500);
    k.link_lag = 1;   // link_frame_lag: the reference's cached link basis (deviation 2)
}

// nominal attitude of drone k (RaceConst::nom_q / nom_rpy)
template <typename Real>
__device__ __forceinline__ Q4<Real> nominal_q(const RaceConst<Real>& C, int k) {
    return {C.nom_q[k][0], C.nom_q[k][1], C.nom_q[k][2], C.nom_q[k][3]};
}
template <typename Real>
__device__ __forceinline__ V3<Real> nominal_rpy(const RaceConst<Real>& C, int k) {
    return v3(C.nom_rpy[k][0], C.nom_rpy[k][1], C.nom_rpy[k][2]);
}
// fills RaceConst::nom_q / nom_rpy in the device copy of the constant block (one lane per drone)
template <typename Real>
__global__ void race_const_init_kernel(RaceConst<Real>* c) {
    const int k = threadIdx.x;
    if (k >= ADRP_MAX_DRONES) return;
    const Real d2r = Real(0.017453292519943295);
    const Q4<Real> q = quat_from_euler_fast(c->init_rpy[k][0] * d2r, c->init_rpy[k][1] * d2r, c->init_rpy[k][2] * d2r);
    const V3<Real> r = euler_xyz_fast(q);
    c->nom_q[k][0] = q.x; c->nom_q[k][1] = q.y; c->nom_q[k][2] = q.z; c->nom_q[k][3] = q.w;
    c->nom_rpy[k][0] = r.x; c->nom_rpy[k][1] = r.y; c->nom_rpy[k][2] = r.z;
}

// ---------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------
// MellingerControl._step_controller's float64 tick schedule (MellingerControl.py:393-411):
//   cur = tick / 500; att due if cur - last_att / 500 > 0.002; pos due if cur - last_pos / 500 > 0.01.
// In float64 these tests depend only on the tick differences, except at the boundaries: a difference
// >= 2 (att) / >= 6 (pos) is always due and <= 0 / <= 4 never (checked for every tick < 2^21); for a
// difference of exactly 1 / 5 the rounding of tick / 500 decides.  Those two decisions per tick are
// bit tables computed on the host in float64 (race_tick_tables), so the loop does no fp64 work: each
// lane keeps a 32-tick window of both tables in registers.
constexpr int kTickTableN = 1 << 17;                  // ticks covered (262 s of flight per episode)
constexpr int kTickWords = kTickTableN / 32 + 1;      // + 1 word of padding for the window read
inline void race_tick_tables(uint32_t* att, uint32_t* pos) {   // host: [kTickWords] each
    for (int w = 0; w < kTickWords; ++w) att[w] = pos[w] = 0;
    for (int n = 1; n < kTickTableN; ++n) {
        const double cur = n / 500.0;
        if (cur - (n - 1) / 500.0 > 0.002) att[n >> 5] |= 1u << (n & 31);
        if (n >= 5 && cur - (n - 5) / 500.0 > 0.01) pos[n >> 5] |= 1u << (n & 31);
    }
}
// bits (tick0 .. tick0 + 31) of both tables; past the table the float64 tests themselves
__device__ __forceinline__ void tick_window(const uint32_t* tab, int n, uint32_t& att, uint32_t& pos) {
    if (__builtin_expect(__any(n > kTickTableN - 32), 0)) {
        if (n > kTickTableN - 32) {
            att = pos = 0;
            for (int j = 0; j < 32; ++j) {
                const double cur = double(n + j) / 500.0;
                att |= (cur - double(n + j - 1) / 500.0 > 0.002 ? 1u : 0u) << j;
                pos |= (cur - double(n + j - 5) / 500.0 > 0.01 ? 1u : 0u) << j;
            }
            return;
        }
    }
    const int w = n >> 5, sh = n & 31;
    att = __builtin_amdgcn_alignbit(tab[w + 1], tab[w], sh);
    pos = __builtin_amdgcn_alignbit(tab[kTickWords + w + 1], tab[kTickWords + w], sh);
}

// clamps: v_med3_f32 (one instruction; the select form is four), in fp64 v_max_f64 + v_min_f64 (the
// double select form is a compare and two v_cndmask per side).  Equal to the reference's
// `v < lo ? lo : (v > hi ? hi : v)` for every non-NaN v, up to the sign of a zero v at a zero bound
// (the max returns +0 where the select keeps -0; every fp64 call site clamps the thrust chain,
// whose later clamp to [20000, 65535] or sqrt makes the two zeros the same value)
__device__ __forceinline__ float clampf_(float v, float lo, float hi) { return __builtin_amdgcn_fmed3f(v, lo, hi); }
__device__ __forceinline__ float clampr_(float v, float lo, float hi) { return __builtin_amdgcn_fmed3f(v, lo, hi); }
__device__ __forceinline__ double clampr_(double v, double lo, double hi) { return __builtin_fmin(__builtin_fmax(v, lo), hi); }
// one-sided clamps (`x > hi ? hi : x`, `x < lo ? lo : x`) as v_min/v_max for non-NaN x
__device__ __forceinline__ float minr_(float x, float hi) { return __builtin_fminf(x, hi); }
__device__ __forceinline__ double minr_(double x, double hi) { return __builtin_fmin(x, hi); }
__device__ __forceinline__ float maxr_(float x, float lo) { return __builtin_fmaxf(x, lo); }
__device__ __forceinline__ double maxr_(double x, double lo) { return __builtin_fmax(x, lo); }
// `a > b ? a : b`; in fp64 as v_max_f64 (equal for every pair but +0 / -0, which compare equal
// wherever the bounds use it)
template <typename Real>
__device__ __forceinline__ Real fmaxr_(Real a, Real b) {
    if constexpr (sizeof(Real) == 8) return __builtin_fmax(a, b);
    else return a > b ? a : b;
}
__device__ __forceinline__ float radf_(float d) { return (3.14159265358979323846f / 180.0f) * d; }
__device__ __forceinline__ float degf_(float r) { return (180.0f / 3.14159265358979323846f) * r; }

template <typename Real>
__device__ __forceinline__ Real shfl_(Real v, int src, int width) { return __shfl(v, src, width); }

// value of lane k of this lane's group of G adjacent lanes (the drones of one env).  G <= 4: a
// DPP quad_perm move (one VALU op, no LDS round trip); G = 8: ds_bpermute.  k must fold to a
// constant (unrolled loops).
template <int G>
__device__ __forceinline__ int grp_bcast_i(int v, int k) {
    if constexpr (G == 1) {
        return v;
    } else if constexpr (G == 2) {
        switch (k) {   // quad_perm [k, k, 2 + k, 2 + k]
            case 0: return __builtin_amdgcn_mov_dpp(v, 0 | (0 << 2) | (2 << 4) | (2 << 6), 0xf, 0xf, false);
            default: return __builtin_amdgcn_mov_dpp(v, 1 | (1 << 2) | (3 << 4) | (3 << 6), 0xf, 0xf, false);
        }
    } else if constexpr (G == 4) {
        switch (k) {   // quad_perm [k, k, k, k]
            case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false);
            case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false);
            case 2: return __builtin_amdgcn_mov_dpp(v, 0xaa, 0xf, 0xf, false);
            default: return __builtin_amdgcn_mov_dpp(v, 0xff, 0xf, 0xf, false);
        }
    } else {
        return __shfl(v, k, G);
    }
}
template <int G>
__device__ __forceinline__ float grp_bcast(float v, int k) {
    return __int_as_float(grp_bcast_i<G>(__float_as_int(v), k));
}
template <int G>
__device__ __forceinline__ double grp_bcast(double v, int k) {
    const int lo = grp_bcast_i<G>(__double2loint(v), k), hi = grp_bcast_i<G>(__double2hiint(v), k);
    return __hiloint2double(hi, lo);
}

// ---------------------------------------------------------------------------------------
// geometry: URDF collision shapes, GJK distance, ray vs cylinder
// ---------------------------------------------------------------------------------------
template <typename Real>
struct Shape {
    V3<Real> c;
    M3<Real> R;      // body -> world
    V3<Real> h;      // box half extents / cylinder (.z = half height)
    Real r;          // cylinder radius (0 for a box)
    int cyl;
};

template <typename Real>
__device__ __forceinline__ V3<Real> support(const Shape<Real>& s, V3<Real> d) {
    const V3<Real> dl = mulT(s.R, d);
    V3<Real> pl;
    if (s.cyl) {
        const Real n2 = dl.x * dl.x + dl.y * dl.y;
        const Real k = n2 > Real(0) ? s.r / sqrt_(n2) : Real(0);
        pl = v3(k * dl.x, k * dl.y, dl.z >= Real(0) ? s.h.z : -s.h.z);
    } else {
        pl = v3(dl.x >= Real(0) ? s.h.x : -s.h.x, dl.y >= Real(0) ? s.h.y : -s.h.y, dl.z >= Real(0) ? s.h.z : -s.h.z);
    }
    return s.c + mul(s.R, pl);
}

// closest point of triangle (a,b,c) to the origin (Ericson 5.1.5); the supporting
// vertices are written to o0..o2 (m of them)
template <typename Real>
__device__ __forceinline__ V3<Real> tri_closest(V3<Real> a, V3<Real> b, V3<Real> c, V3<Real>& o0, V3<Real>& o1,
                                               V3<Real>& o2, int& m) {
    const V3<Real> ab = b - a, ac = c - a;
    const Real d1 = -dot(ab, a), d2 = -dot(ac, a);
    if (d1 <= Real(0) && d2 <= Real(0)) { o0 = a; m = 1; return a; }
    const Real d3 = -dot(ab, b), d4 = -dot(ac, b);
    if (d3 >= Real(0) && d4 <= d3) { o0 = b; m = 1; return b; }
    const Real vc = d1 * d4 - d3 * d2;
    if (vc <= Real(0) && d1 >= Real(0) && d3 <= Real(0)) {
        o0 = a; o1 = b; m = 2;
        return a + (d1 / (d1 - d3)) * ab;
    }
    const Real d5 = -dot(ab, c), d6 = -dot(ac, c);
    if (d6 >= Real(0) && d5 <= d6) { o0 = c; m = 1; return c; }
    const Real vb = d5 * d2 - d1 * d6;
    if (vb <= Real(0) && d2 >= Real(0) && d6 <= Real(0)) {
        o0 = a; o1 = c; m = 2;
        return a + (d2 / (d2 - d6)) * ac;
    }
    const Real va = d3 * d6 - d5 * d4;
    if (va <= Real(0) && (d4 - d3) >= Real(0) && (d5 - d6) >= Real(0)) {
        o0 = b; o1 = c; m = 2;
        return b + ((d4 - d3) / ((d4 - d3) + (d5 - d6))) * (c - b);
    }
    const Real den = Real(1) / (va + vb + vc);
    o0 = a; o1 = b; o2 = c; m = 3;
    return a + (vb * den) * ab + (vc * den) * ac;
}

// "distance(A, B) < cut" for two convex shapes, by GJK with the simplex kept in named
// registers (no dynamic indexing -> no scratch). Every iterate v is a point of the
// Minkowski difference, so |v| >= distance, and v.w / |v| <= distance for the support point
// w: the loop stops as soon as either bound decides against `cut`, else on convergence.
// v0 (optional): the first search direction, a point of A - B (e.g. A's centre minus B's point
// closest to it, gjk_seed): near a long part it starts the iteration next to the closest features
// instead of along the centre difference
template <typename Real>
__device__ __forceinline__ bool gjk_within_body(const Shape<Real>& A0, const Shape<Real>& B0, Real cut,
                                                bool* undecided, const V3<Real>* v0, int max_it,
                                                int* nout) {
    // in A's centre frame: support points stay O(shape size), so the fp32 termination test
    // is not swamped by rounding of world coordinates (which stalled convergence)
    Shape<Real> A = A0, B = B0;
    B.c = B0.c - A0.c;
    A.c = v3(Real(0), Real(0), Real(0));
    const Real eps = sizeof(Real) == 4 ? Real(4e-6) : Real(1e-13);
    const Real tol2 = sizeof(Real) == 4 ? Real(1e-14) : Real(1e-26);   // (1e-7 m)^2, (1e-13 m)^2
    V3<Real> W0, W1, W2, W3;
    int n = 0;
    V3<Real> v = A.c - B.c;
    if (v0 != nullptr) v = *v0;
    const Real cut2 = cut * cut;
    if (dot(v, v) < Real(1e-20)) v = v3(Real(1), Real(0), Real(0));
    Real vv_prev = Real(3.0e38);
    for (int it = 0; it < max_it; ++it) {
        const V3<Real> w = support(A, Real(-1) * v) - support(B, v);
        const Real vv = dot(v, v), vw = dot(v, w);
        // cycling: the same |v| twice in a row is the same simplex again (fp32 near contact: a support
        // point equal to a simplex vertex up to rounding, far above the 1e-10 m duplicate test, brings
        // back the same triangle every iteration; tools/gjk_replay.py).  The 48-iteration cap then
        // returned this same |v|'s answer.  (|v| may grow once: from the centre difference to the
        // first support point, and out of a flat tetrahedron, so only equality is a cycle.)
        if (vv == vv_prev) {
            GJK_STAT(it + 1);
            if (undecided) *undecided = true;
            return vv < cut2;
        }
        vv_prev = vv;
        if (vw > Real(0) && vw * vw >= cut2 * vv) { GJK_STAT(it + 1); return false; }   // lower bound
        if (vv - vw <= eps * vv) { GJK_STAT(it + 1); return vv < cut2; }
        // absolute gap: the distance is known to within tol (|v| - vw/|v| <= tol).  Near contact
        // (cut = 1 um, touching or penetrating shapes) |v| is tiny and the relative test above can
        // not pass under the rounding of O(0.1 m) support points, which ran such queries to the cap
        if ((vv - vw) * (vv - vw) <= tol2 * vv) { GJK_STAT(it + 1); return vv < cut2; }
        const V3<Real> dw0 = W0 - w, dw1 = W1 - w, dw2 = W2 - w;
        if ((n > 0 && dot(dw0, dw0) < Real(1e-20)) || (n > 1 && dot(dw1, dw1) < Real(1e-20)) ||
            (n > 2 && dot(dw2, dw2) < Real(1e-20))) {
            GJK_STAT(it + 1);
            return vv < cut2;
        }
        if (n == 0) { W0 = w; n = 1; v = w; }
        else if (n == 1) {
            W1 = w;
            const V3<Real> ab = W1 - W0;
            const Real t = -dot(W0, ab) / dot(ab, ab);
            if (t <= Real(0)) { n = 1; v = W0; }
            else if (t >= Real(1)) { W0 = W1; n = 1; v = W0; }
            else { n = 2; v = W0 + t * ab; }
        } else if (n == 2) {
            int m;
            v = tri_closest(W0, W1, w, W0, W1, W2, m);
            n = m;
        } else {
            W3 = w;
            // faces (0,1,2|3) (0,2,3|1) (0,3,1|2) (1,3,2|0)
            Real best = Real(3.0e38);
            V3<Real> bv = v, b0 = W0, b1 = W1, b2 = W2;
            int bm = 0;
            bool outside = false;
            // a flat (degenerate) tetrahedron -- two level discs at one height -- encloses
            // nothing: every face is then a candidate
            const V3<Real> e1 = W1 - W0, e2 = W2 - W0, e3 = W3 - W0;
            const Real vol = dot(e1, cross(e2, e3));
            const Real scl = sqrt_(dot(e1, e1) * dot(e2, e2) * dot(e3, e3));
            const bool flat = fabs_(vol) <= (sizeof(Real) == 4 ? Real(1e-5) : Real(1e-12)) * scl;
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const V3<Real> p0 = f == 3 ? W1 : W0;
                const V3<Real> p1 = f == 0 ? W1 : (f == 1 ? W2 : W3);
                const V3<Real> p2 = f == 0 ? W2 : (f == 1 ? W3 : (f == 2 ? W1 : W2));
                const V3<Real> po = f == 0 ? W3 : (f == 1 ? W1 : (f == 2 ? W2 : W0));
                const V3<Real> nrm = cross(p1 - p0, p2 - p0);
                const Real so = -dot(nrm, p0), sd = dot(nrm, po - p0);
                if (flat || so * sd < Real(0)) {
                    outside = true;
                    V3<Real> q0, q1, q2;
                    int m;
                    const V3<Real> vf = tri_closest(p0, p1, p2, q0, q1, q2, m);
                    const Real dd = dot(vf, vf);
                    if (dd < best) { best = dd; bv = vf; b0 = q0; b1 = q1; b2 = q2; bm = m; }
                }
            }
            if (!outside) { GJK_STAT(it + 1); return true; }
            v = bv; W0 = b0; W1 = b1; W2 = b2; n = bm;
        }
        if (dot(v, v) < cut2) { GJK_STAT(it + 1); return true; }   // upper bound
    }
    GJK_STAT(max_it);
    if (undecided) *undecided = true;
    return dot(v, v) < cut2;
}

template <typename Real>
__device__ __forceinline__ bool gjk_within_impl(const Shape<Real>& A0, const Shape<Real>& B0, Real cut,
                                                bool* undecided = nullptr, const V3<Real>* v0 = nullptr,
                                                int max_it = 48) {
#if defined(ADRP_RACE_TIMING) && defined(ADRP_RACE_GJK_STATS)
    int n = 0;
    const bool r = gjk_within_body<Real>(A0, B0, cut, undecided, v0, max_it, &n);
    if (n >= ADRP_GJK_DUMP_MIN_IT) {   // the query, for a CPU replay (tools/gjk_slow.py)
        const unsigned int k = atomicAdd(&g_gjk_dump_n, 1u);
        if (k < unsigned(kGjkDumps)) {
            double* o = g_gjk_dump + size_t(k) * kGjkDumpF;
            const Shape<Real>* sh[2] = {&A0, &B0};
            for (int j = 0; j < 2; ++j) {
                const Shape<Real>& q = *sh[j];
                double* p = o + 17 * j;
                p[0] = q.c.x; p[1] = q.c.y; p[2] = q.c.z;
                p[3] = q.R.a00; p[4] = q.R.a01; p[5] = q.R.a02; p[6] = q.R.a10; p[7] = q.R.a11; p[8] = q.R.a12;
                p[9] = q.R.a20; p[10] = q.R.a21; p[11] = q.R.a22;
                p[12] = q.h.x; p[13] = q.h.y; p[14] = q.h.z; p[15] = q.r; p[16] = q.cyl;
            }
            o[34] = cut; o[35] = 0.0; o[36] = double(sizeof(Real)); o[37] = n; o[38] = r ? 1.0 : 0.0;
            o[39] = v0 ? double(v0->x) : 0.0; o[40] = v0 ? double(v0->y) : 0.0; o[41] = v0 ? double(v0->z) : 0.0;
            o[42] = v0 ? 1.0 : 0.0; o[43] = double(max_it);
        }
    }
    return r;
#else
    return gjk_within_body<Real>(A0, B0, cut, undecided, v0, max_it, nullptr);
#endif
}

template <typename Real>
__device__ __forceinline__ Shape<double> shape_f64(const Shape<Real>& s) {
    Shape<double> d;
    d.c = v3(double(s.c.x), double(s.c.y), double(s.c.z));
    d.R = {double(s.R.a00), double(s.R.a01), double(s.R.a02), double(s.R.a10), double(s.R.a11), double(s.R.a12),
           double(s.R.a20), double(s.R.a21), double(s.R.a22)};
    d.h = v3(double(s.h.x), double(s.h.y), double(s.h.z));
    d.r = double(s.r);
    d.cyl = s.cyl;
    return d;
}

// "distance(A, B) < cut".  A contact query (cut 1 um) that the fp32 iteration leaves undecided is
// run again by the float64 GJK on the same float shapes: near contact the float iteration can not
// resolve |v| against the O(0.1 m) support points and cycles one triangle (|v| 1e-6 .. 4e-4 m where
// the oracle's distance was 0 .. 2e-4 m; tools/gjk_slow.py, tools/gjk_replay.py), so those
// queries are decided as the oracle decides them.  Decided queries (the lower bound, the enclosed
// origin, the upper bound, convergence) keep the float answer, and range queries (0.45 m) stay
// float.
// out of line: one copy per code object for the rare rerun (inlined at the three query sites it
// grew the fp32 kernels by ~10 % of code and made them no faster; a round-3 A/B)
__device__ __noinline__ bool gjk_within_f64_call(Shape<double> A, Shape<double> B, double cut, V3<double> v0, bool seeded) {
    return gjk_within_impl<double>(A, B, cut, nullptr, seeded ? &v0 : nullptr);
}

#ifndef ADRP_GJK_CAP_F32
#define ADRP_GJK_CAP_F32 24
#endif
#ifndef ADRP_GJK_CONTACT_F64   // 0: the float contact iteration first, float64 only for undecided queries
#define ADRP_GJK_CONTACT_F64 1
#endif
constexpr int kGjkContactCapF32 = ADRP_GJK_CAP_F32;
template <typename Real>
__device__ __forceinline__ bool gjk_within(const Shape<Real>& A0, const Shape<Real>& B0, Real cut,
                                           const V3<Real>* v0 = nullptr) {
    if constexpr (sizeof(Real) == 4) {
        if (cut < Real(1e-3)) {
#if ADRP_GJK_CONTACT_F64
            // contact queries (cut 1 um) run in float64 from the start: near contact the float
            // iteration stalls (|v| not resolvable against O(0.1 m) support points) and was rerun in
            // float64 after up to 24 float iterations; the slow actor-driven queries (tools/gjk_slow.py:
            // 691 of >= 8 iterations in 400 launches) take 8.8 float64 iterations on average, at most 14,
            // against 10.7 / 31 for the float iteration plus its rerun (CPU replay, tools/gjk_replay.py)
            const V3<double> v0d = v0 ? v3(double(v0->x), double(v0->y), double(v0->z)) : v3(0.0, 0.0, 0.0);
            return gjk_within_f64_call(shape_f64(A0), shape_f64(B0), double(cut), v0d, v0 != nullptr);
#else
            // a float contact query still open after 24 iterations goes to the float64 rerun (which
            // decides as the oracle does) instead of running the float iteration to 48: the actor-driven
            // tail was one such query per few hundred launches (48 fp32 iterations + the rerun)
            bool undecided = false;
            const bool r = gjk_within_impl<Real>(A0, B0, cut, &undecided, v0, kGjkContactCapF32);
            if (__builtin_expect(!undecided, 1)) return r;
            const V3<double> v0d = v0 ? v3(double(v0->x), double(v0->y), double(v0->z)) : v3(0.0, 0.0, 0.0);
            return gjk_within_f64_call(shape_f64(A0), shape_f64(B0), double(cut), v0d, v0 != nullptr);
#endif
        }
    }
    return gjk_within_impl<Real>(A0, B0, cut, nullptr, v0);
}

// entry fraction of the segment p0 -> p1 into a cylinder, > 1 on a miss
template <typename Real>
__device__ __forceinline__ Real ray_cylinder(const Shape<Real>& s, V3<Real> p0, V3<Real> p1) {
    const V3<Real> a = mulT(s.R, p0 - s.c), d = mulT(s.R, p1 - p0);
    Real lo = Real(-3.0e38), hi = Real(3.0e38);
    if (d.z == Real(0)) {
        if (fabs_(a.z) > s.h.z) return Real(2);
    } else {
        Real t1 = (-s.h.z - a.z) / d.z, t2 = (s.h.z - a.z) / d.z;
        if (t1 > t2) { const Real t = t1; t1 = t2; t2 = t; }
        lo = t1; hi = t2;
    }
    const Real qa = d.x * d.x + d.y * d.y, qb = Real(2) * (a.x * d.x + a.y * d.y),
               qc = a.x * a.x + a.y * a.y - s.r * s.r;
    if (qa == Real(0)) {
        if (qc > Real(0)) return Real(2);
    } else {
        const Real disc = qb * qb - Real(4) * qa * qc;
        if (disc < Real(0)) return Real(2);
        const Real sq = sqrt_(disc);
        const Real t3 = (-qb - sq) / (Real(2) * qa), t4 = (-qb + sq) / (Real(2) * qa);
        if (t3 > lo) lo = t3;
        if (t4 < hi) hi = t4;
    }
    if (lo > hi || hi < Real(0) || lo > Real(1)) return Real(2);
    return lo < Real(0) ? Real(0) : lo;
}

template <typename Real>
__device__ __forceinline__ M3<Real> rotz_(Real yaw) {
    Real s, c;
    sincos_f_(yaw, &s, &c);
    return {c, -s, Real(0), s, c, Real(0), Real(0), Real(0), Real(1)};
}
template <typename Real>
__device__ __forceinline__ M3<Real> mmul_(const M3<Real>& a, const M3<Real>& b) {
    return {a.a00 * b.a00 + a.a01 * b.a10 + a.a02 * b.a20, a.a00 * b.a01 + a.a01 * b.a11 + a.a02 * b.a21,
            a.a00 * b.a02 + a.a01 * b.a12 + a.a02 * b.a22, a.a10 * b.a00 + a.a11 * b.a10 + a.a12 * b.a20,
            a.a10 * b.a01 + a.a11 * b.a11 + a.a12 * b.a21, a.a10 * b.a02 + a.a11 * b.a12 + a.a12 * b.a22,
            a.a20 * b.a00 + a.a21 * b.a10 + a.a22 * b.a20, a.a20 * b.a01 + a.a21 * b.a11 + a.a22 * b.a21,
            a.a20 * b.a02 + a.a21 * b.a12 + a.a22 * b.a22};
}

// part k of a gate (portal.urdf / low_portal.urdf) or obstacle (obstacle.urdf), own frame
template <typename Real>
__device__ __forceinline__ void gate_part(int k, int low, V3<Real>& off, M3<Real>& R, V3<Real>& h, Real& r, int& cyl) {
    const Real c157 = Real(0.0007963267107332633), s157 = Real(0.9999996829318346);   // cos/sin(1.57)
    const M3<Real> I = {Real(1), Real(0), Real(0), Real(0), Real(1), Real(0), Real(0), Real(0), Real(1)};
    const M3<Real> Ry = {c157, Real(0), s157, Real(0), Real(1), Real(0), -s157, Real(0), c157};
    h = v3(Real(0.25), Real(0.025), Real(0.025)); r = Real(0); cyl = 0; R = I;
    if (k == 0) off = v3(Real(0), Real(0), Real(-0.225));
    else if (k == 1) off = v3(Real(0), Real(0), Real(0.225));
    else if (k == 2) { off = v3(Real(0.225), Real(0), Real(0)); R = Ry; }
    else if (k == 3) { off = v3(Real(-0.225), Real(0), Real(0)); R = Ry; }
    else if (low) { off = v3(Real(0), Real(0), Real(-0.4)); h = v3(Real(0.075), Real(0.075), Real(0.125)); }
    else { off = v3(Real(0), Real(0), Real(-0.6)); h = v3(Real(0), Real(0), Real(0.4)); r = Real(0.05); cyl = 1; }
}
template <typename Real>
__device__ __forceinline__ void obst_part(int k, V3<Real>& off, V3<Real>& h, Real& r, int& cyl) {
    if (k == 0) { off = v3(Real(0), Real(0), Real(0)); h = v3(Real(0), Real(0), Real(0.4)); r = Real(0.05); cyl = 1; }
    else { off = v3(Real(0), Real(0), Real(-0.4)); h = v3(Real(0.075), Real(0.075), Real(0.125)); r = Real(0); cyl = 0; }
}

template <typename Real>
__device__ __forceinline__ Shape<Real> drone_shape(const RaceConst<Real>& C, V3<Real> pos, Q4<Real> q) {
    const M3<Real> R = rot(q);
    return Shape<Real>{pos + C.coll_zoff * col2(R), R, v3(Real(0), Real(0), C.coll_hh), C.coll_r, 1};
}

// ---------------------------------------------------------------------------------------
// lane state
// ---------------------------------------------------------------------------------------
// Diagnostics (the causal fp64 closed-loop bar, tests/test_race_gpu.py): an FNV-1a style hash of the
// int16 (roll, pitch, yaw) moments of every firmware call of one env.step, in call order.  The
// oracle computes the same hash (oracle/race.c fw_moment_hash), so equal hashes mean the kernel and
// the oracle truncated every moment of the step to the same integers.
constexpr uint32_t kMomHashSeed = 2166136261u;
__device__ __forceinline__ uint32_t fw_moment_hash(uint32_t h, float r, float p, float y) {
    h = (h ^ uint32_t(int32_t(r))) * 16777619u;
    h = (h ^ uint32_t(int32_t(p))) * 16777619u;
    return (h ^ uint32_t(int32_t(y))) * 16777619u;
}

template <typename Real>
struct RDrone {
    V3<Real> pos, vel, w, angv, lpos, kpos;
    Q4<Real> q, ql;
    Real rpm[4], prev[4];
    Real prev_rpy[3], prev_vel[3];
    float lpf1[3], lpf2[3], ierr[3], ierrm[3];
    float pw_roll, pw_pitch, psp_roll, psp_pitch;
    float ctl[4];
    Real mass, inertia[3];
    Real inv_mass, inv_i[3];        // per env.step
    int tick, last_att, last_pos, tumble, gate, flags;   // last_*: the ticks of last_{att,pos}_pid_call
    int tick_base;                  // tick of bit 0 of the tick-schedule windows
    uint32_t att_bits, pos_bits;    // tick_window(tick_base)
    uint32_t mh;                    // fw_moment_hash over this env.step's firmware calls (diagnostics)
};

template <typename Real>
__device__ __forceinline__ Real ld(const Real* f, int field, size_t EN, size_t slot) { return f[size_t(field) * EN + slot]; }
template <typename Real>
__device__ __forceinline__ void st(Real* f, int field, size_t EN, size_t slot, Real v) { f[size_t(field) * EN + slot] = v; }

// TW: also load the tick-schedule window (a caller that issued it early passes false and sets it);
// ANGV: load the DYN world angular velocity (the other physics modes never change it: the four-lane
// kernel then neither loads nor stores it, so it holds no registers through the sub-steps)
template <typename Real, bool TW = true, bool ANGV = true>
__device__ __forceinline__ void load_drone(const RaceArgs<Real>& a, size_t EN, size_t slot, RDrone<Real>& d) {
    const Real* f = a.f;
#define L_(k) ld(f, (k), EN, slot)
    d.pos = v3(L_(RF_POS), L_(RF_POS + 1), L_(RF_POS + 2));
    d.q = {L_(RF_QUAT), L_(RF_QUAT + 1), L_(RF_QUAT + 2), L_(RF_QUAT + 3)};
    d.vel = v3(L_(RF_VEL), L_(RF_VEL + 1), L_(RF_VEL + 2));
    d.w = v3(L_(RF_OMEGA), L_(RF_OMEGA + 1), L_(RF_OMEGA + 2));
    if constexpr (ANGV) d.angv = v3(L_(RF_ANGV), L_(RF_ANGV + 1), L_(RF_ANGV + 2));
    else d.angv = v3(Real(0), Real(0), Real(0));
    d.ql = {L_(RF_LINK_QUAT), L_(RF_LINK_QUAT + 1), L_(RF_LINK_QUAT + 2), L_(RF_LINK_QUAT + 3)};
    d.lpos = v3(L_(RF_LINK_POS), L_(RF_LINK_POS + 1), L_(RF_LINK_POS + 2));
    d.kpos = v3(L_(RF_KIN_POS), L_(RF_KIN_POS + 1), L_(RF_KIN_POS + 2));
#pragma unroll
    for (int k = 0; k < 4; ++k) { d.rpm[k] = L_(RF_RPM + k); d.prev[k] = L_(RF_PREV_RPM + k); d.ctl[k] = float(L_(RF_CTL + k)); }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d.prev_rpy[k] = L_(RF_PREV_RPY + k); d.prev_vel[k] = L_(RF_PREV_VEL + k);
        d.lpf1[k] = float(L_(RF_LPF_D1 + k)); d.lpf2[k] = float(L_(RF_LPF_D2 + k));
        d.ierr[k] = float(L_(RF_I_ERR + k)); d.ierrm[k] = float(L_(RF_I_ERR_M + k));
        d.inertia[k] = L_(RF_INERTIA + k);
    }
    d.pw_roll = float(L_(RF_PREV_OMEGA_ROLL)); d.pw_pitch = float(L_(RF_PREV_OMEGA_PITCH));
    d.psp_roll = float(L_(RF_PREV_SP_ROLL)); d.psp_pitch = float(L_(RF_PREV_SP_PITCH));
    d.mass = L_(RF_MASS);
    d.mh = kMomHashSeed;
#undef L_
    const int32_t* ist = a.ist;
    d.tick = ist[RI_TICK * EN + slot]; d.last_att = ist[RI_LAST_ATT * EN + slot];
    d.last_pos = ist[RI_LAST_POS * EN + slot]; d.tumble = ist[RI_TUMBLE * EN + slot];
    d.gate = ist[RI_GATE * EN + slot]; d.flags = ist[RI_FLAGS * EN + slot];
    if constexpr (TW) {
        d.tick_base = d.tick;
        tick_window(a.ticks, d.tick, d.att_bits, d.pos_bits);
    }
    d.inv_mass = Real(1) / d.mass;
#pragma unroll
    for (int k = 0; k < 3; ++k) d.inv_i[k] = Real(1) / d.inertia[k];
}

// store_drone split in two for the four-lane kernel: everything the sub-step loop leaves final
// (stored right after the loop, so those registers are free for the post-loop queries), then the
// gate / flags the post-loop phases still change
template <typename Real, bool ANGV = true>
__device__ __forceinline__ void store_drone_body(const RaceArgs<Real>& a, size_t EN, size_t slot, const RDrone<Real>& d) {
    Real* f = a.f;
#define S_(k, v) st(f, (k), EN, slot, Real(v))
    S_(RF_POS, d.pos.x); S_(RF_POS + 1, d.pos.y); S_(RF_POS + 2, d.pos.z);
    S_(RF_QUAT, d.q.x); S_(RF_QUAT + 1, d.q.y); S_(RF_QUAT + 2, d.q.z); S_(RF_QUAT + 3, d.q.w);
    S_(RF_VEL, d.vel.x); S_(RF_VEL + 1, d.vel.y); S_(RF_VEL + 2, d.vel.z);
    S_(RF_OMEGA, d.w.x); S_(RF_OMEGA + 1, d.w.y); S_(RF_OMEGA + 2, d.w.z);
    if constexpr (ANGV) { S_(RF_ANGV, d.angv.x); S_(RF_ANGV + 1, d.angv.y); S_(RF_ANGV + 2, d.angv.z); }
    S_(RF_LINK_QUAT, d.ql.x); S_(RF_LINK_QUAT + 1, d.ql.y); S_(RF_LINK_QUAT + 2, d.ql.z); S_(RF_LINK_QUAT + 3, d.ql.w);
    S_(RF_LINK_POS, d.lpos.x); S_(RF_LINK_POS + 1, d.lpos.y); S_(RF_LINK_POS + 2, d.lpos.z);
    S_(RF_KIN_POS, d.kpos.x); S_(RF_KIN_POS + 1, d.kpos.y); S_(RF_KIN_POS + 2, d.kpos.z);
#pragma unroll
    for (int k = 0; k < 4; ++k) { S_(RF_RPM + k, d.rpm[k]); S_(RF_PREV_RPM + k, d.prev[k]); S_(RF_CTL + k, d.ctl[k]); }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        S_(RF_PREV_RPY + k, d.prev_rpy[k]); S_(RF_PREV_VEL + k, d.prev_vel[k]);
        S_(RF_LPF_D1 + k, d.lpf1[k]); S_(RF_LPF_D2 + k, d.lpf2[k]);
        S_(RF_I_ERR + k, d.ierr[k]); S_(RF_I_ERR_M + k, d.ierrm[k]);
    }
    S_(RF_PREV_OMEGA_ROLL, d.pw_roll); S_(RF_PREV_OMEGA_PITCH, d.pw_pitch);
    S_(RF_PREV_SP_ROLL, d.psp_roll); S_(RF_PREV_SP_PITCH, d.psp_pitch);
#undef S_
    int32_t* ist = a.ist;
    ist[RI_TICK * EN + slot] = d.tick; ist[RI_LAST_ATT * EN + slot] = d.last_att;
    ist[RI_LAST_POS * EN + slot] = d.last_pos; ist[RI_TUMBLE * EN + slot] = d.tumble;
    if (a.mom_hash) a.mom_hash[slot] = d.mh;
}
template <typename Real>
__device__ __forceinline__ void store_drone_flags(const RaceArgs<Real>& a, size_t EN, size_t slot, const RDrone<Real>& d) {
    a.ist[RI_GATE * EN + slot] = d.gate; a.ist[RI_FLAGS * EN + slot] = d.flags;
}

template <typename Real>
__device__ __forceinline__ void store_drone(const RaceArgs<Real>& a, size_t EN, size_t slot, const RDrone<Real>& d,
                                            bool params) {
    Real* f = a.f;
#define S_(k, v) st(f, (k), EN, slot, Real(v))
    S_(RF_POS, d.pos.x); S_(RF_POS + 1, d.pos.y); S_(RF_POS + 2, d.pos.z);
    S_(RF_QUAT, d.q.x); S_(RF_QUAT + 1, d.q.y); S_(RF_QUAT + 2, d.q.z); S_(RF_QUAT + 3, d.q.w);
    S_(RF_VEL, d.vel.x); S_(RF_VEL + 1, d.vel.y); S_(RF_VEL + 2, d.vel.z);
    S_(RF_OMEGA, d.w.x); S_(RF_OMEGA + 1, d.w.y); S_(RF_OMEGA + 2, d.w.z);
    S_(RF_ANGV, d.angv.x); S_(RF_ANGV + 1, d.angv.y); S_(RF_ANGV + 2, d.angv.z);
    S_(RF_LINK_QUAT, d.ql.x); S_(RF_LINK_QUAT + 1, d.ql.y); S_(RF_LINK_QUAT + 2, d.ql.z); S_(RF_LINK_QUAT + 3, d.ql.w);
    S_(RF_LINK_POS, d.lpos.x); S_(RF_LINK_POS + 1, d.lpos.y); S_(RF_LINK_POS + 2, d.lpos.z);
    S_(RF_KIN_POS, d.kpos.x); S_(RF_KIN_POS + 1, d.kpos.y); S_(RF_KIN_POS + 2, d.kpos.z);
#pragma unroll
    for (int k = 0; k < 4; ++k) { S_(RF_RPM + k, d.rpm[k]); S_(RF_PREV_RPM + k, d.prev[k]); S_(RF_CTL + k, d.ctl[k]); }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        S_(RF_PREV_RPY + k, d.prev_rpy[k]); S_(RF_PREV_VEL + k, d.prev_vel[k]);
        S_(RF_LPF_D1 + k, d.lpf1[k]); S_(RF_LPF_D2 + k, d.lpf2[k]);
        S_(RF_I_ERR + k, d.ierr[k]); S_(RF_I_ERR_M + k, d.ierrm[k]);
    }
    S_(RF_PREV_OMEGA_ROLL, d.pw_roll); S_(RF_PREV_OMEGA_PITCH, d.pw_pitch);
    S_(RF_PREV_SP_ROLL, d.psp_roll); S_(RF_PREV_SP_PITCH, d.psp_pitch);
    if (params) {   // mass / inertia: written by the reset only
        S_(RF_MASS, d.mass);
        S_(RF_INERTIA, d.inertia[0]); S_(RF_INERTIA + 1, d.inertia[1]); S_(RF_INERTIA + 2, d.inertia[2]);
    } else if (a.mom_hash) {   // the step's store (not a reset's): the firmware-output hash
        a.mom_hash[slot] = d.mh;
    }
#undef S_
    int32_t* ist = a.ist;
    ist[RI_TICK * EN + slot] = d.tick; ist[RI_LAST_ATT * EN + slot] = d.last_att;
    ist[RI_LAST_POS * EN + slot] = d.last_pos; ist[RI_TUMBLE * EN + slot] = d.tumble;
    ist[RI_GATE * EN + slot] = d.gate; ist[RI_FLAGS * EN + slot] = d.flags;
}

// ---------------------------------------------------------------------------------------
// firmware controllerMellinger (C float) + MellingerControl wrapper
// ---------------------------------------------------------------------------------------
struct Lpf { float b0, b1, b2, a1, a2; };
__device__ __forceinline__ float lpf_apply(const Lpf& l, float& d1, float& d2, float sample) {
#pragma clang fp contract(off)   // the firmware is C float code built without FMA contraction
    float d0 = sample - d1 * l.a1 - d2 * l.a2;
    if (!isfinite(d0)) d0 = sample;
    const float out = d0 * l.b0 + d1 * l.b1 + d2 * l.b2;
    d2 = d1;
    d1 = d0;
    return out;
}

// FULLSTATE setpoint modes (MellingerControl.py:510-543): x,y,z,quat abs; rates 0
// FAST (fp32 kernel): hardware reciprocals for the firmware's divisions; the fp64 kernel
// keeps the C float divisions bit-for-bit
// CMD (command mode, commander.h): the setpoint comes from the command state cs: position, velocity,
// acceleration, attitude rates and the mode (SP_FULLSTATE: desiredYaw from the quaternion;
// SP_COMMANDER: attitude.yaw; SP_UNSET: the zeroed setpoint_t, every mode modeDisable -> thrust
// direction (-sin 0, -sin 0, 1), desiredYaw 0); xc_x / xc_y are then computed here.
template <typename Real, bool FAST = (sizeof(Real) == 4), bool CMD = false>
__device__ __forceinline__ void mellinger_fw(RDrone<Real>& d, const float sp[3], float xc_x, float xc_y,
                                             const float gyro[3], const float pos[3], const float vel[3],
                                             const float Rm[9], const CmdState* cs = nullptr) {
#pragma clang fp contract(off)
    const float dt = float(1.0f / 500);
    float rx, ry, rz, vx, vy, vz, tx, ty, tz;
    float spr = 0.0f, spp = 0.0f, spy = 0.0f;   // setpoint attitude rates [deg/s]
    if constexpr (CMD) {
        rx = cs->sp_pos[0] - pos[0]; ry = cs->sp_pos[1] - pos[1]; rz = cs->sp_pos[2] - pos[2];
        vx = cs->sp_vel[0] - vel[0]; vy = cs->sp_vel[1] - vel[1]; vz = cs->sp_vel[2] - vel[2];
        spr = cs->sp_rate[0]; spp = cs->sp_rate[1]; spy = cs->sp_rate[2];
    } else {
        rx = sp[0] - pos[0]; ry = sp[1] - pos[1]; rz = sp[2] - pos[2];
        vx = 0.0f - vel[0]; vy = 0.0f - vel[1]; vz = 0.0f - vel[2];
    }
    d.ierr[2] = clampf_(d.ierr[2] + rz * dt, -0.4f, 0.4f);
    d.ierr[0] = clampf_(d.ierr[0] + rx * dt, -2.0f, 2.0f);
    d.ierr[1] = clampf_(d.ierr[1] + ry * dt, -2.0f, 2.0f);
    if constexpr (CMD) {
        float yaw_deg = 0.0f;
        if (cs->mode != SP_UNSET) {
            tx = 0.027f * cs->sp_acc[0] + 0.4f * rx + 0.2f * vx + 0.05f * d.ierr[0];
            ty = 0.027f * cs->sp_acc[1] + 0.4f * ry + 0.2f * vy + 0.05f * d.ierr[1];
            tz = 0.027f * (cs->sp_acc[2] + 9.81f) + 1.25f * rz + 0.4f * vz + 0.05f * d.ierr[2];
        } else {
            tx = -sinf(radf_(0.0f)); ty = -sinf(radf_(0.0f)); tz = 1.0f;
        }
        if (cs->mode == SP_COMMANDER) {
            yaw_deg = cs->sp_yaw;
        } else if (cs->mode == SP_FULLSTATE) {
            const float qz = cs->sp_qz, qw = cs->sp_qw;
            yaw_deg = degf_(atan2f(2.0f * (qw * qz + 0.0f * 0.0f), 1 - 2 * (0.0f * 0.0f + qz * qz)));
        }
        xc_x = cosf(radf_(yaw_deg));
        xc_y = sinf(radf_(yaw_deg));
    } else {
        tx = 0.027f * 0.0f + 0.4f * rx + 0.2f * vx + 0.05f * d.ierr[0];
        ty = 0.027f * 0.0f + 0.4f * ry + 0.2f * vy + 0.05f * d.ierr[1];
        tz = 0.027f * (0.0f + 9.81f) + 1.25f * rz + 0.4f * vz + 0.05f * d.ierr[2];
    }
    // R columns
    const float Rx0 = Rm[0], Rx1 = Rm[3], Rx2 = Rm[6];
    const float Ry0 = Rm[1], Ry1 = Rm[4], Ry2 = Rm[7];
    const float Rz0 = Rm[2], Rz1 = Rm[5], Rz2 = Rm[8];
    const float current_thrust = tx * Rz0 + ty * Rz1 + tz * Rz2;
    const float tn = FAST ? __builtin_amdgcn_sqrtf(tx * tx + ty * ty + tz * tz) : sqrtf(tx * tx + ty * ty + tz * tz);
    const float itn = FAST ? __builtin_amdgcn_rcpf(tn) : 0.0f;
    // !FAST: the C float divisions, correctly rounded through one float64 reciprocal per divisor
    // (f64::fdiv_rcp: the same bits as x / y, a third of the instructions for three quotients)
#ifdef ADRP_EXP_FDIV_IEEE   // measurement-only: the plain IEEE float divisions (A/B of fdiv_rcp)
#define FDIV_(x, ry, y) ((x) / (y))
#else
#define FDIV_(x, ry, y) f64::fdiv_rcp((x), (ry))
#endif
    const double rtn = FAST ? 0.0 : f64::rcp(double(tn));
    const float zd0 = FAST ? tx * itn : FDIV_(tx, rtn, tn), zd1 = FAST ? ty * itn : FDIV_(ty, rtn, tn),
                zd2 = FAST ? tz * itn : FDIV_(tz, rtn, tn);
    // y_des = normalize(z_des x x_c), x_c = (cos yaw, sin yaw, 0)
    float yd0 = zd1 * 0.0f - zd2 * xc_y, yd1 = zd2 * xc_x - zd0 * 0.0f, yd2 = zd0 * xc_y - zd1 * xc_x;
    const float yn = FAST ? __builtin_amdgcn_sqrtf(yd0 * yd0 + yd1 * yd1 + yd2 * yd2) : sqrtf(yd0 * yd0 + yd1 * yd1 + yd2 * yd2);
    if (FAST) {
        const float iyn = __builtin_amdgcn_rcpf(yn);
        yd0 *= iyn; yd1 *= iyn; yd2 *= iyn;
    } else {
        const double ryn = f64::rcp(double(yn));
        yd0 = FDIV_(yd0, ryn, yn); yd1 = FDIV_(yd1, ryn, yn); yd2 = FDIV_(yd2, ryn, yn);
    }
    const float xd0 = yd1 * zd2 - yd2 * zd1, xd1 = yd2 * zd0 - yd0 * zd2, xd2 = yd0 * zd1 - yd1 * zd0;
    const float eRx = (zd0 * Ry0 + zd1 * Ry1 + zd2 * Ry2) - (Rz0 * yd0 + Rz1 * yd1 + Rz2 * yd2);
    const float eRy = -((xd0 * Rz0 + xd1 * Rz1 + xd2 * Rz2) - (Rx0 * zd0 + Rx1 * zd1 + Rx2 * zd2));
    const float eRz = (yd0 * Rx0 + yd1 * Rx1 + yd2 * Rx2) - (Ry0 * xd0 + Ry1 * xd1 + Ry2 * xd2);
    const float rate_roll = radf_(gyro[0]), rate_pitch = -radf_(gyro[1]), rate_yaw = radf_(gyro[2]);
    const float ewx = radf_(spr) - rate_roll, ewy = -radf_(spp) - rate_pitch, ewz = radf_(spy) - rate_yaw;
    float err_d_roll = 0, err_d_pitch = 0;
    if (d.pw_roll == d.pw_roll) {
        // !FAST: x / dt as fdiv_rcp by the correctly rounded float64 1 / dt (2^-52 relative: exact too)
        constexpr double kInvDt = 1.0 / double(float(1.0f / 500));
        err_d_roll = FAST ? ((radf_(spr) - d.psp_roll) - (rate_roll - d.pw_roll)) * 500.0f
                          : FDIV_((radf_(spr) - d.psp_roll) - (rate_roll - d.pw_roll), kInvDt, dt);
        err_d_pitch = FAST ? (-(radf_(spp) - d.psp_pitch) - (rate_pitch - d.pw_pitch)) * 500.0f
                           : FDIV_(-(radf_(spp) - d.psp_pitch) - (rate_pitch - d.pw_pitch), kInvDt, dt);
    }
    d.pw_roll = rate_roll;
    d.pw_pitch = rate_pitch;
    d.psp_roll = radf_(spr);
    d.psp_pitch = radf_(spp);
    d.ierrm[0] = clampf_(d.ierrm[0] + (-eRx) * dt, -1.0f, 1.0f);
    d.ierrm[1] = clampf_(d.ierrm[1] + (-eRy) * dt, -1.0f, 1.0f);
    d.ierrm[2] = clampf_(d.ierrm[2] + (-eRz) * dt, -1500.0f, 1500.0f);
    const float Mx = -70000.0f * eRx + 20000.0f * ewx + 0.0f * d.ierrm[0] + 200.0f * err_d_roll;
    const float My = -70000.0f * eRy + 20000.0f * ewy + 0.0f * d.ierrm[1] + 200.0f * err_d_pitch;
    const float Mz = -60000.0f * eRz + 12000.0f * ewz + 500.0f * d.ierrm[2];
    d.ctl[3] = 132000.0f * current_thrust;
    // thrust <= 0: moments and integrators zeroed.  Selects, not a branch: the branch form made the
    // compiler merge the two paths' stores into one dynamically addressed store, which put
    // ierrm[2] / ctl[2] in scratch memory (a scratch load + vmcnt(0) wait on every firmware call)
    const bool on = d.ctl[3] > 0;
    d.ctl[0] = on ? float(int16_t(clampf_(Mx, -32000.0f, 32000.0f))) : 0.0f;
    d.ctl[1] = on ? float(int16_t(clampf_(My, -32000.0f, 32000.0f))) : 0.0f;
    d.ctl[2] = on ? float(int16_t(clampf_(-Mz, -32000.0f, 32000.0f))) : 0.0f;
    d.mh = fw_moment_hash(d.mh, d.ctl[0], d.ctl[1], d.ctl[2]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d.ierr[k] = on ? d.ierr[k] : 0.0f;
        d.ierrm[k] = on ? d.ierrm[k] : 0.0f;
    }
}
#undef FDIV_

// MellingerControl.computeControl (154-262) -> rpm (float64 wrapper arithmetic in Real)
// CMD: command mode (commander.h) — _update_state into cs->st_*, and while the commander drives
// the setpoint (override off) _update_setpoint(tick / 500) before _step_controller (MellingerControl.py:
// 216-241); coef = the drone's polynomial block (CF_COEF).
template <typename Real, bool CMD = false>
__device__ __forceinline__ void mellinger_compute(RDrone<Real>& d, const Lpf& lpf, const float sp[3], float xc_x,
                                                  float xc_y, V3<Real> rpy, const Real noise[4],
                                                  CmdState* cs = nullptr, const float* coef = nullptr, size_t EN = 0,
                                                  size_t slot = 0, int16_t* mlog = nullptr, int* mcount = nullptr) {
#pragma clang fp contract(off)   // numpy / C arithmetic of the reference wrapper and firmware
    constexpr bool F32 = sizeof(Real) == 4;   // fp32 kernel: reciprocal multiplies; fp64: numpy's divisions
    const Real fdt = Real(0.002);
    const Real r2d = Real(57.29577951308232);
    Real rates[3];
    const Real rr[3] = {rpy.x, rpy.y, rpy.z};
    const Real vv[3] = {d.vel.x, d.vel.y, d.vel.z};
    Real acc_z = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        rates[k] = F32 ? (rr[k] - d.prev_rpy[k]) * Real(500) : divc_(rr[k] - d.prev_rpy[k], fdt);
        d.prev_rpy[k] = rr[k];
        if (k == 2)
            acc_z = F32 ? (vv[k] - d.prev_vel[k]) * Real(500.0 / 9.8) + Real(1)
                        : divc_(divc_(vv[k] - d.prev_vel[k], fdt), Real(9.8)) + Real(1);
        d.prev_vel[k] = vv[k];
    }
    float gyro[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) gyro[k] = lpf_apply(lpf, d.lpf1[k], d.lpf2[k], float(rates[k] * r2d));
    if constexpr (CMD) {
        cs->st_pos[0] = float(d.pos.x); cs->st_pos[1] = float(d.pos.y); cs->st_pos[2] = float(d.pos.z);
        cs->st_vel[0] = float(d.vel.x); cs->st_vel[1] = float(d.vel.y); cs->st_vel[2] = float(d.vel.z);
        cs->st_yaw = float(rpy.z * r2d);
        if (!cs->ovr) hl_update_setpoint(*cs, coef, EN, slot, float(double(d.tick) / 500.0));
    }
    Real pwm[4];
    if (float(acc_z) < -0.5f) d.tumble += 1; else d.tumble = 0;
    if (d.tumble >= 30) {
        d.tick += 1;
        pwm[0] = pwm[1] = pwm[2] = pwm[3] = Real(0);
    } else {
        // the float64 schedule from the tick differences and the host bit tables (tick_window)
        const int da = d.tick - d.last_att, dp = d.tick - d.last_pos, bit = d.tick - d.tick_base;
        const bool att_due = (da >= 2) | ((da == 1) & (((d.att_bits >> bit) & 1u) != 0));
        const bool pos_due = (dp >= 6) | ((dp == 5) & (((d.pos_bits >> bit) & 1u) != 0));
        // t = 0 (both due), 2 (attitude due), 1 (neither); selects, no branches
        d.last_pos = (att_due & pos_due) ? d.tick : d.last_pos;
        d.last_att = att_due ? d.tick : d.last_att;
        if (att_due) {   // t even: RATE_DO_EXECUTE(500 Hz, tick)
            // state.attitudeQuaternion = get_quaternion_from_euler(rpy) -> quat2rotmat: the body
            // rotation itself, except in getEulerFromQuaternion's gimbal branches
            float Rm[9];
            const Real sarg = Real(-2) * (d.q.x * d.q.z - d.q.w * d.q.y);
            const M3<Real> Rq = rot(d.q);
            Rm[0] = float(Rq.a00); Rm[1] = float(Rq.a01); Rm[2] = float(Rq.a02);
            Rm[3] = float(Rq.a10); Rm[4] = float(Rq.a11); Rm[5] = float(Rq.a12);
            Rm[6] = float(Rq.a20); Rm[7] = float(Rq.a21); Rm[8] = float(Rq.a22);
            // the gimbal-lock path (3 libm sincosf) sits behind a wave-uniform test, so it is
            // entered only when a lane needs it instead of being if-converted into every sub-step
            if (__builtin_expect(__any(!(fabs_(sarg) < Real(0.99999))), 0)) {
                if (!(fabs_(sarg) < Real(0.99999))) {
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
            mellinger_fw<Real, sizeof(Real) == 4, CMD>(d, sp, xc_x, xc_y, gyro, pos, vel, Rm, cs);
            if (mlog) {   // diagnostics level 2: this call's int16 moments (the oracle can replay them)
                const int c = *mcount;
                mlog[3 * c] = int16_t(d.ctl[0]); mlog[3 * c + 1] = int16_t(d.ctl[1]); mlog[3 * c + 2] = int16_t(d.ctl[2]);
                *mcount = c + 1;
            }
        }
        d.tick += 1;
        // _compute_pwms (423-442)
        const Real r = Real(d.ctl[0]) / Real(2), p = Real(d.ctl[1]) / Real(2), y = Real(d.ctl[2]), th = Real(d.ctl[3]);
        const Real m4[4] = {th - r + p + y, th - r - p - y, th + r - p + y, th + r + p - y};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const Real x = F32 ? clampr_(m4[k], Real(0), Real(65535)) * Real(60.0 / 65535)
                               : divc_(clampr_(m4[k], Real(0), Real(65535)), Real(65535)) * Real(60);
            const Real volts = Real(-0.0006239) * x * x + Real(0.088) * x;
            const Real pct = minr_(F32 ? volts * Real(1.0 / 3) : divc_(volts, Real(3)), Real(1));
            pwm[k] = pct * Real(65535);
        }
    }
    // clip -> thrust -> reorder [3,2,1,0] -> + noise -> _thr2pwm -> rpm (246-262)
    Real th[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const Real rp = Real(0.2685) * clampr_(pwm[k], Real(20000), Real(65535)) + Real(4070.3);
        th[k] = Real(3.16e-10) * rp * rp;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const Real t = maxr_(th[3 - k] + noise[k], Real(0));
        Real mp = F32 ? (hsqrt_(t * Real(1.0 / 3.16e-10)) - Real(4070.3)) * Real(1.0 / 0.2685)
                      : divc_(sqrt_(divc_(t, Real(3.16e-10))) - Real(4070.3), Real(0.2685));
        mp = clampr_(mp, Real(20000), Real(65535));
        d.prev[k] = d.rpm[k];
        d.rpm[k] = Real(0.2685) * mp + Real(4070.3);
    }
}

// ---------------------------------------------------------------------------------------
// one physics sub-step of one drone (Bullet floating-base step after the force calls)
// ---------------------------------------------------------------------------------------
// Rq = rot(d.q), Rl = rot(d.ql) on entry; on return Rq = rot(new q), Rl = rot(new ql) (= the entry
// Rq): a caller that carries both across sub-steps computes one rotation matrix per sub-step
template <typename Real, int PH>
__device__ __forceinline__ void race_pyb_substep_r(const RaceConst<Real>& C, RDrone<Real>& d, V3<Real> F_ext,
                                                   V3<Real> T_ext, M3<Real>& Rq, M3<Real>& Rl) {
    constexpr bool GND = (PH == ADRP_PHYS_PYB_GND || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    constexpr bool DRAG = (PH == ADRP_PHYS_PYB_DRAG || PH == ADRP_PHYS_PYB_GND_DRAG_DW);
    const M3<Real> R = Rq;
    // cached link basis: GND modes refresh it (getLinkStates(computeForwardKinematics=1))
    // before the ground-effect forces, after the motor forces (BaseAviary.py:739-744)
    const M3<Real> Rs = C.link_lag ? Rl : R;
    Real sum_f = 0, t2 = 0;
    V3<Real> P = v3(Real(0), Real(0), Real(0));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const Real r2 = d.rpm[i] * d.rpm[i];
        const Real f = r2 * C.kf;
        sum_f += f;
        // the reference drone's props sit in the body plane: a literal pz = 0 adds f * 0 = +0
        // (f >= 0) to +0, so P.z stays +0 without the 8 multiply-adds
        const bool pz0 = __builtin_constant_p(C.pz[i]) && C.pz[i] == Real(0);
        P = v3(P.x + f * C.px[i], P.y + f * C.py[i], pz0 ? P.z : P.z + f * C.pz[i]);
        t2 += (i & 1) ? -r2 : r2;
    }
    const Real tau_z = t2 * C.km;
    const V3<Real> zs = col2(Rs);
    V3<Real> Fw = v3(sum_f * zs.x, sum_f * zs.y, sum_f * zs.z - d.mass * C.gravity) + F_ext;
    const V3<Real> m3 = mulT(R, zs);
    V3<Real> nb = cross(P, m3) + tau_z * m3 + mulT(R, T_ext);
    if constexpr (GND) {
        const Real sqx = d.q.x * d.q.x, sqy = d.q.y * d.q.y, sqz = d.q.z * d.q.z, squ = d.q.w * d.q.w;
        const Real sarg = Real(-2) * (d.q.x * d.q.z - d.q.w * d.q.y);
        const Real den = squ - sqx - sqy + sqz, num = Real(2) * (d.q.y * d.q.z + d.q.w * d.q.x);
        const bool gate = fabs_(sarg) < Real(0.99999) && (den > Real(0) || (den == Real(0) && num == Real(0)));
        if (gate) {
            Real sg = 0;
            V3<Real> G = v3(Real(0), Real(0), Real(0));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                Real h = d.pos.z + R.a20 * C.px[i] + R.a21 * C.py[i] + R.a22 * C.pz[i];
                h = h < C.gnd_clip ? C.gnd_clip : h;
                const Real k = C.prop_r4 * rcp_(h);
                const Real g = C.gnd_kf * d.rpm[i] * d.rpm[i] * k * k;
                sg += g;
                G = G + v3(g * C.px[i], g * C.py[i], g * C.pz[i]);
            }
            Fw = Fw + sg * col2(R);
            nb = nb + v3(G.y, -G.x, Real(0));
        }
    }
    if constexpr (DRAG) {
        Real s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += d.prev[i];
        s = s * Real(0.10471975511965977);
        const V3<Real> dw = v3(-C.drag[0] * s * d.vel.x, -C.drag[1] * s * d.vel.y, -C.drag[2] * s * d.vel.z);
        Fw = Fw + (GND ? dw : mul(Rs, mulT(R, dw)));
    }
    const Real ixx = d.inertia[0], iyy = d.inertia[1], izz = d.inertia[2];
    (void)0;
    const V3<Real> wb = mulT(R, d.w);
    const V3<Real> Iw = v3(ixx * wb.x, iyy * wb.y, izz * wb.z);
    const Real kw = Real(0.04) + Real(0.04) * hsqrt_nn_(dot(wb, wb));
    const V3<Real> rhs = nb - kw * Iw - cross(wb, Iw);
    const V3<Real> wdot = mul(R, v3(rhs.x * d.inv_i[0], rhs.y * d.inv_i[1], rhs.z * d.inv_i[2]));
    const Real kv = Real(0.04) + Real(0.04) * hsqrt_nn_(dot(d.vel, d.vel));
    const V3<Real> acc = d.inv_mass * Fw - kv * d.vel;
    d.w = v3(d.w.x + C.dt * wdot.x, d.w.y + C.dt * wdot.y, d.w.z + C.dt * wdot.z);
    d.vel = v3(d.vel.x + C.dt * acc.x, d.vel.y + C.dt * acc.y, d.vel.z + C.dt * acc.z);
    clamp100_wv(d.w, d.vel);
    // forwardKinematics of this step caches the pre-integration pose
    d.ql = d.q;
    d.lpos = d.pos;
    d.pos = d.pos + C.dt * d.vel;
    Real ang = hsqrt_nn_(dot(d.w, d.w));
    if (ang > C.ang_max) ang = C.ang_max;
    // sin(|w| dt / 2) / |w| = (dt / 2) sinc(|w| dt / 2) (argument <= ANGULAR_MOTION_THRESHOLD / 2 = pi / 8):
    // no reciprocal, and Bullet's |w| < 0.001 form is the same series to rounding
    Real sinc, ch;
    expmap_sinc_cos_full(Real(0.5) * ang * C.dt, &sinc, &ch);
    const Real sc = (Real(0.5) * C.dt) * sinc;
    const V3<Real> ax = sc * d.w;
    const Q4<Real> q0 = d.q;
    const Q4<Real> q1 = {ch * q0.x + ax.x * q0.w + ax.y * q0.z - ax.z * q0.y,
                         ch * q0.y + ax.y * q0.w + ax.z * q0.x - ax.x * q0.z,
                         ch * q0.z + ax.z * q0.w + ax.x * q0.y - ax.y * q0.x,
                         ch * q0.w - ax.x * q0.x - ax.y * q0.y - ax.z * q0.z};
    // fp64: the refined v_rsq_f64 (<= 2 ulp) instead of 1 / IEEE sqrt (two correctly rounded
    // sequences on the chain); fp32 keeps the correctly rounded form.  (The wave-uniform short forms
    // of the hover step, the short exp-map series / quat_inv_norm / the plane-contact guard, measured slower
    // in this kernel: config 4 fp64 +1.3 us, A/B)
    const Real nq2 = q1.x * q1.x + q1.y * q1.y + q1.z * q1.z + q1.w * q1.w;
    const Real inv = sizeof(Real) == 8 ? hrsqrt_nc_(nq2) : rsqrt_(nq2);
    d.q = {q1.x * inv, q1.y * inv, q1.z * inv, q1.w * inv};
    const M3<Real> Rn = rot(d.q);
    const Real low = d.pos.z + C.coll_zoff - C.coll_hh * fabs_(Rn.a22) - C.coll_r * hsqrt_nn_(Rn.a02 * Rn.a02 + Rn.a12 * Rn.a12);
    if (low < Real(0)) {
        d.pos.z -= low;
        if (d.vel.z < Real(0)) d.vel.z = Real(0);
    }
    Rl = R;
    Rq = Rn;
}
template <typename Real, int PH>
__device__ __forceinline__ void race_pyb_substep(const RaceConst<Real>& C, RDrone<Real>& d, V3<Real> F_ext,
                                                 V3<Real> T_ext) {
    M3<Real> Rq = rot(d.q), Rl = rot(d.ql);
    race_pyb_substep_r<Real, PH>(C, d, F_ext, T_ext, Rq, Rl);
}

template <typename Real>
__device__ __forceinline__ void race_dyn_substep(const RaceConst<Real>& C, RDrone<Real>& d) {
    const M3<Real> R = rot(d.q);
    Real f[4], zt[4], sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[i] = d.rpm[i] * d.rpm[i] * C.kf;
        zt[i] = d.rpm[i] * d.rpm[i] * C.km;
        sum += f[i];
    }
    const V3<Real> zb = col2(R);
    const V3<Real> force_w = v3(sum * zb.x, sum * zb.y, sum * zb.z - C.gravity * C.dyn_mass);
    const Real tz = -zt[0] + zt[1] - zt[2] + zt[3];
    const Real tx = (f[0] + f[1] - f[2] - f[3]) * C.dyn_arm;
    const Real ty = (-f[0] + f[1] + f[2] - f[3]) * C.dyn_arm;
    const V3<Real> rr = d.w;
    const V3<Real> tq = v3(tx, ty, tz) - cross(rr, v3(C.dyn_i[0] * rr.x, C.dyn_i[1] * rr.y, C.dyn_i[2] * rr.z));
    const V3<Real> rdd = v3(tq.x * C.dyn_inv_i[0], tq.y * C.dyn_inv_i[1], tq.z * C.dyn_inv_i[2]);
    d.vel = d.vel + C.dt * (C.dyn_inv_mass * force_w);
    d.w = rr + C.dt * rdd;
    d.pos = d.pos + C.dt * d.vel;
    const V3<Real> w = d.w;
    const Real wn = hsqrt_(dot(w, w));
    if (!(wn <= Real(1e-8))) {
        const Real th = wn * C.dt * Real(0.5);
        Real s, c;
        if (th <= Real(0.39269908169872414)) small_sincos(th, &s, &c);
        else sincos_(th, &s, &c);
        const Real k = s * rcp_(wn);
        const Q4<Real> q = d.q;
        d.q = {c * q.x + k * (w.z * q.y - w.y * q.z + w.x * q.w), c * q.y + k * (-w.z * q.x + w.x * q.z + w.y * q.w),
               c * q.z + k * (w.y * q.x - w.x * q.y + w.z * q.w), c * q.w + k * (-w.x * q.x - w.y * q.y - w.z * q.z)};
    }
    d.angv = mul(R, d.w);
}

// ---------------------------------------------------------------------------------------
// drone <-> track queries: getClosestPoints(distance=0.45) in-range flags (_computeObs 591-651)
// and contacts (_collision 552-562) as decisions "min part distance < cut".
//
// Exact bounds decide almost every (drone, part) pair without GJK. With p the centre of the
// drone's collision cylinder and dr its bounding radius, dist(p, part) - dr <= dist(drone,
// part) <= dist(p, part); dist(p, part) to a box / cylinder is closed form. Only pairs whose
// bounds straddle a cut (by more than the rounding guard) are queued; each lane then walks
// its own queue, so a wave runs max-over-lanes GJKs instead of one per part any lane needs.
// ---------------------------------------------------------------------------------------
template <typename Real>
__device__ __forceinline__ Real point_part_dist(V3<Real> lp, V3<Real> h, Real r, int cyl) {
    if (cyl) {
        const Real dr = fmaxr_(hsqrt_(lp.x * lp.x + lp.y * lp.y) - r, Real(0));
        const Real dz = fmaxr_(fabs_(lp.z) - h.z, Real(0));
        return hsqrt_(dr * dr + dz * dz);
    }
    const Real dx = fmaxr_(fabs_(lp.x) - h.x, Real(0)), dy = fmaxr_(fabs_(lp.y) - h.y, Real(0)),
               dz = fmaxr_(fabs_(lp.z) - h.z, Real(0));
    return hsqrt_(dx * dx + dy * dy + dz * dz);
}

// closest point of a part (own frame: box half extents h / z-axis cylinder radius r, half height h.z)
template <typename Real>
__device__ __forceinline__ V3<Real> part_closest(V3<Real> x, V3<Real> h, Real r, int cyl) {
    if (cyl) {
        const Real rho = hsqrt_(x.x * x.x + x.y * x.y);
        const Real k = rho > r ? r * rcp_(rho) : Real(1);
        return v3(x.x * k, x.y * k, clampr_(x.z, -h.z, h.z));
    }
    return v3(clampr_(x.x, -h.x, h.x), clampr_(x.y, -h.y, h.y), clampr_(x.z, -h.z, h.z));
}

// GJK seed for a (drone, part) query: the drone's centre minus the part point closest to it (world
// frame), a point of drone - part
template <typename Real>
__device__ __forceinline__ V3<Real> gjk_seed(const Shape<Real>& drone, const Shape<Real>& part) {
    const V3<Real> x = mulT(part.R, drone.c - part.c);
    return mul(part.R, x - part_closest(x, part.h, part.r, part.cyl));
}

// Support-function bounds of one (drone cylinder, part) pair in the part's frame: lp = the centre of
// the drone's collision cylinder, ax = its axis (unit), dr / dhh = its radius / half height.  With q
// the part point closest to lp and n = (q - lp) / |q - lp|, the (convex) part lies beyond the plane
// through q normal to n, so every cylinder point x is at least |q - lp| - (x - lp).n from it:
//   lo = |q - lp| - (dr |n - (n.a) a| + dhh |n.a|)          (the cylinder's support in direction n),
// and the cylinder's support point x* in direction n is a point of the drone:  up = dist(x*, part).
// For a flat face both are the exact distance; near edges the band is second order.  The centre
// bounds (|q - lp| - sqrt(dr^2 + dhh^2), |q - lp|) leave every pair within 6 cm of a cut open.
template <typename Real>
__device__ __forceinline__ void part_bounds_refined(V3<Real> lp, V3<Real> ax, V3<Real> h, Real r, int cyl, Real dr,
                                                    Real dhh, Real& lo, Real& up) {
    // y: a point of the drone's cylinder (its centre first, then its support points); q = the part
    // point closest to y.  For every such y, n = (q - y) / |q - y| gives the lower bound
    // (q - lp).n - support(n) and the cylinder's support point in n the upper bound.  Three rounds
    // (alternating projections) narrow the band near edges and curved parts.
    V3<Real> y = lp;
    lo = Real(-1);
    up = Real(3.0e38);
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const V3<Real> q = part_closest(y, h, r, cyl);
        const V3<Real> d = q - y;
        const Real pd = hsqrt_(dot(d, d));
        up = pd < up ? pd : up;
        if (!(pd > Real(1e-6))) return;   // y in (or at) the part: only the upper bound is known
        const V3<Real> n = rcp_(pd) * d;
        const Real c = dot(n, ax);
        const V3<Real> sp = n - c * ax;
        const Real sn = hsqrt_(dot(sp, sp));
        lo = fmaxr_(lo, dot(q - lp, n) - (dr * sn + dhh * fabs_(c)));
        const Real k = sn > Real(1e-6) ? dr * rcp_(sn) : Real(0);
        y = lp + (c >= Real(0) ? dhh : -dhh) * ax + k * sp;
    }
    const Real fd = point_part_dist(y, h, r, cyl);
    up = fd < up ? fd : up;
}

constexpr int kGateParts = 5, kObstParts = 2, kObstBit0 = ADRP_MAX_GATES * kGateParts;
constexpr int kRaceMaxD = 49 + 6 * (ADRP_MAX_DRONES - 1);   // obs row floats (COMPETE, 8 drones)
constexpr int kTrackFields = RF_WR_TARGET - RF_GATE;   // the env's actual gates (16) + obstacles (12)

// Where a lane reads its env's actual gate / obstacle poses: the SoA fields in HBM, or (L) the
// block's LDS copy [field][kRaceBlock] that the helper waves load while the chain runs.
template <typename Real, bool L>
struct TrackSrc {
    const Real* f;
    size_t EN, slot;
    const float* lds;
    int tl;
    __device__ __forceinline__ Real operator()(int field) const {
        if constexpr (L) return Real(lds[(field - RF_GATE) * kRaceBlock + tl]);
        else return ld(f, field, EN, slot);
    }
    // the same source for block lane l (drone slots of G-lane groups, clamped like the kernel's)
    __device__ __forceinline__ TrackSrc lane(int l, int G, int N, int E) const {
        TrackSrc t = *this;
        if constexpr (L) {
            t.tl = l;
        } else {
            const int gl = int(blockIdx.x) * kRaceBlock + l;
            const int e = gl / G < E ? gl / G : E - 1, d = gl % G < N ? gl % G : 0;
            t.slot = size_t(e) * N + d;
        }
        return t;
    }
};

// placed collision shape of queue bit b (gate b / 5, part b % 5; obstacle bits from kObstBit0)
template <typename Real, class TS>
__device__ __forceinline__ Shape<Real> track_part_shape(const RaceConst<Real>& C, const TS& T, int b) {
    V3<Real> off, h;
    Real r;
    int cyl;
    if (b < kObstBit0) {
        const int g = b / kGateParts, k = b - g * kGateParts;
        M3<Real> R;
        gate_part(k, C.gate_type[g] > 0, off, R, h, r, cyl);
        const V3<Real> org = v3(T(RF_GATE + 4 * g), T(RF_GATE + 4 * g + 1), T(RF_GATE + 4 * g + 2));
        const M3<Real> Rg = rotz_(T(RF_GATE + 4 * g + 3));
        return Shape<Real>{org + mul(Rg, off), mmul_(Rg, R), h, r, cyl};
    }
    const int o = (b - kObstBit0) / kObstParts, k = (b - kObstBit0) - o * kObstParts;
    obst_part(k, off, h, r, cyl);
    const V3<Real> org = v3(T(RF_OBST + 3 * o), T(RF_OBST + 3 * o + 1), T(RF_OBST + 3 * o + 2));
    const M3<Real> I = {Real(1), Real(0), Real(0), Real(0), Real(1), Real(0), Real(0), Real(0), Real(1)};
    return Shape<Real>{org + off, I, h, r, cyl};
}

// bounds pass: in-range bits decided by the bounds (gate g -> bit g, obstacle k -> bit k) for
// `cut`, and the queue of pairs left to GJK (amb; camb_all: those queued for the contact cut)
template <typename Real, class TS>
__device__ __forceinline__ void track_bounds(const RaceConst<Real>& C, const TS& T, const Shape<Real>& ds, Real cut,
                                             bool want_contact, Real ccut, uint32_t& gin, uint32_t& oin,
                                             uint32_t& amb, uint32_t& camb_all, bool* ccert = nullptr) {
    const Real tol = sizeof(Real) == 4 ? Real(1e-5) : Real(1e-10);
    const Real dr = hsqrt_(ds.r * ds.r + ds.h.z * ds.h.z);
    const V3<Real> p = ds.c, ax = col2(ds.R);
    amb = 0; camb_all = 0;
    gin = 0; oin = 0;
#pragma unroll
    for (int g = 0; g < ADRP_MAX_GATES; ++g) {
        if (g < C.num_gates) {
            const V3<Real> dp = p - v3(T(RF_GATE + 4 * g), T(RF_GATE + 4 * g + 1), T(RF_GATE + 4 * g + 2));
            Real sn, cs;
            sincos_f_(T(RF_GATE + 4 * g + 3), &sn, &cs);
            const V3<Real> lg = v3(cs * dp.x + sn * dp.y, -sn * dp.x + cs * dp.y, dp.z);   // Rz(yaw)^T dp
            const V3<Real> ag = v3(cs * ax.x + sn * ax.y, -sn * ax.x + cs * ax.y, ax.z);
            const int low = C.gate_type[g] > 0;
            bool in = false;
            uint32_t gamb = 0, camb = 0;
#pragma unroll
            for (int k = 0; k < kGateParts; ++k) {
                V3<Real> off, h;
                M3<Real> R;
                Real r;
                int cyl;
                gate_part(k, low, off, R, h, r, cyl);
                const V3<Real> lp = mulT(R, lg - off);
                const Real pd = point_part_dist(lp, h, r, cyl);
                Real lo = pd - dr, up = pd;
                if (C.refine && ((!(pd < cut - tol) && lo < cut + tol) || (want_contact && lo < ccut + tol))) {
                    Real lo2, up2;
                    part_bounds_refined(lp, mulT(R, ag), h, r, cyl, ds.r, ds.h.z, lo2, up2);
                    lo = fmaxr_(lo, lo2);
                    up = up2 < up ? up2 : up;
                }
                in |= up < cut - tol;
                if (lo < cut + tol) gamb |= 1u << k;
                // a drone point inside the part (up == 0: the clamps are the identity; the centre or
                // a support point of part_bounds_refined) is a contact without GJK (an
                // intersecting pair is GJK's slowest case)
                if (want_contact && lo < ccut + tol) {
                    if (ccert && up == Real(0)) *ccert = true;   // a drone point in the part
                    else camb |= 1u << k;
                }
            }
            if (in) gin |= 1u << g;
            amb |= ((in ? 0u : gamb) | camb) << (g * kGateParts);
            camb_all |= camb << (g * kGateParts);
        }
    }
#pragma unroll
    for (int o = 0; o < ADRP_MAX_OBSTACLES; ++o) {
        if (o < C.num_obstacles) {
            const V3<Real> dp = p - v3(T(RF_OBST + 3 * o), T(RF_OBST + 3 * o + 1), T(RF_OBST + 3 * o + 2));
            bool in = false;
            uint32_t gamb = 0, camb = 0;
#pragma unroll
            for (int k = 0; k < kObstParts; ++k) {
                V3<Real> off, h;
                Real r;
                int cyl;
                obst_part(k, off, h, r, cyl);
                const Real pd = point_part_dist(dp - off, h, r, cyl);
                Real lo = pd - dr, up = pd;
                if (C.refine && ((!(pd < cut - tol) && lo < cut + tol) || (want_contact && lo < ccut + tol))) {
                    Real lo2, up2;
                    part_bounds_refined(dp - off, ax, h, r, cyl, ds.r, ds.h.z, lo2, up2);
                    lo = fmaxr_(lo, lo2);
                    up = up2 < up ? up2 : up;
                }
                in |= up < cut - tol;
                if (lo < cut + tol) gamb |= 1u << k;
                if (want_contact && lo < ccut + tol) {
                    if (ccert && up == Real(0)) *ccert = true;   // a drone point in the part
                    else camb |= 1u << k;
                }
            }
            if (in) oin |= 1u << o;
            amb |= ((in ? 0u : gamb) | camb) << (kObstBit0 + o * kObstParts);
            camb_all |= camb << (kObstBit0 + o * kObstParts);
        }
    }
}

// in-range bits for `cut` (gin, oin); returns the contact decision (distance < ccut) when
// want_contact.  Per lane: each lane walks its own GJK queue.
template <typename Real, class TS>
__device__ __forceinline__ bool track_query(const RaceConst<Real>& C, const TS& T, const Shape<Real>& ds, Real cut,
                                            bool want_contact, Real ccut, uint32_t& gin, uint32_t& oin) {
    uint32_t amb, camb_all;
    track_bounds(C, T, ds, cut, want_contact, ccut, gin, oin, amb, camb_all);
    // a contact-queued pair has its drone centre within dr of the part, so its body is
    // already in range by the upper bound: each queued pair needs exactly one of the cuts
    bool contact = false;
    while (amb) {
        const int b = __builtin_ctz(amb);
        amb &= amb - 1;
        const bool for_contact = (camb_all >> b) & 1u;
        const Shape<Real> s = track_part_shape(C, T, b);
        if (gjk_within(ds, s, for_contact ? ccut : cut)) {
            if (for_contact) contact = true;
            else if (b < kObstBit0) gin |= 1u << (b / kGateParts);
            else oin |= 1u << ((b - kObstBit0) / kObstParts);
        }
    }
    return want_contact && contact;
}

// track_query with contacts for the whole wave (all kRaceBlock lanes of the block's single chain
// wave reach it together): the lanes' GJK queues are pooled in LDS and dealt out one job per
// lane per round, so a wave runs ceil(jobs / 64) GJKs instead of max-over-lanes queue length.
// Same pairs, same GJK inputs (the owner lane's shape by cross-lane moves): same decisions.
struct TrackJobs {
    uint16_t job[kRaceBlock * (ADRP_MAX_GATES * kGateParts + ADRP_MAX_OBSTACLES * kObstParts)];
    uint32_t res[kRaceBlock];
};

// the GJK part of track_query_wave for the bounds pass's result (gin, oin, amb, camb_all).
// SH: lanes per drone = 1 << SH (race_quad.h: 4); every lane reads its drone's owner lane's result
template <typename Real, class TS, int SH = 0>
__device__ __forceinline__ bool track_gjk_pool(const RaceConst<Real>& C, const TS& T, const Shape<Real>& ds,
                                               bool live, Real cut, Real ccut, uint32_t& gin, uint32_t& oin,
                                               uint32_t amb, uint32_t camb_all, TrackJobs& q, int tl, int G, int N,
                                               int E) {
    if (!live) amb = 0;
    const int n = __popc(amb);
    int incl = n;   // inclusive scan of the queue lengths
#pragma unroll
    for (int o = 1; o < kRaceBlock; o <<= 1) {
        const int t = __shfl_up(incl, o, kRaceBlock);
        if (tl >= o) incl += t;
    }
    const int total = __shfl(incl, kRaceBlock - 1, kRaceBlock);
    int pos = incl - n;
    q.res[tl] = 0;
    for (uint32_t m = amb; m; m &= m - 1) {
        const int b = __builtin_ctz(m);
        q.job[pos++] = uint16_t((tl << 6) | (((camb_all >> b) & 1u) << 5) | b);
    }
    __syncthreads();
    for (int base = 0; base < total; base += kRaceBlock) {
        const int j = base + tl;
        const int job = q.job[j < total ? j : total - 1];
        const int L = job >> 6, b = job & 31;
        const bool fc = (job >> 5) & 1;
        Shape<Real> dl = ds;   // lane L's drone (h, r, cyl are the same for every drone)
        dl.c = v3(shfl_(ds.c.x, L, kRaceBlock), shfl_(ds.c.y, L, kRaceBlock), shfl_(ds.c.z, L, kRaceBlock));
        dl.R.a00 = shfl_(ds.R.a00, L, kRaceBlock); dl.R.a01 = shfl_(ds.R.a01, L, kRaceBlock);
        dl.R.a02 = shfl_(ds.R.a02, L, kRaceBlock); dl.R.a10 = shfl_(ds.R.a10, L, kRaceBlock);
        dl.R.a11 = shfl_(ds.R.a11, L, kRaceBlock); dl.R.a12 = shfl_(ds.R.a12, L, kRaceBlock);
        dl.R.a20 = shfl_(ds.R.a20, L, kRaceBlock); dl.R.a21 = shfl_(ds.R.a21, L, kRaceBlock);
        dl.R.a22 = shfl_(ds.R.a22, L, kRaceBlock);
        if (j < total) {
            const Shape<Real> s = track_part_shape(C, T.lane(L, G, N, E), b);
            // warm start (config 3 + actor 78.4 -> 77.3 us fp64, 58.7 -> 57.6 us fp32; config 4 unchanged)
            const V3<Real> v0 = gjk_seed(dl, s);
            if (gjk_within(dl, s, fc ? ccut : cut, &v0)) {
                const uint32_t bit = fc ? 1u << 8
                                        : b < kObstBit0 ? 1u << (b / kGateParts)
                                                        : 1u << (4 + (b - kObstBit0) / kObstParts);
                atomicOr(&q.res[L], bit);
            }
        }
    }
    __syncthreads();
    const uint32_t r = q.res[(tl >> SH) << SH];
    gin |= r & 15u;
    oin |= (r >> 4) & 15u;
    return (r >> 8) & 1u;
}
// want_contact: false for a drone already eliminated (its contact cannot change anything,
// _computeTerminated 684-692 ORs it into drones_eliminated)
template <typename Real, class TS>
__device__ __forceinline__ bool track_query_wave(const RaceConst<Real>& C, const TS& T, const Shape<Real>& ds,
                                                 bool live, bool want_contact, Real cut, Real ccut, uint32_t& gin,
                                                 uint32_t& oin, TrackJobs& q, int tl, int G, int N, int E) {
    uint32_t amb, camb_all;
    bool ccert = false;
    track_bounds(C, T, ds, cut, want_contact, ccut, gin, oin, amb, camb_all, &ccert);
    const bool c = track_gjk_pool<Real, TS, 0>(C, T, ds, live, cut, ccut, gin, oin, amb, camb_all, q, tl, G, N, E);
    return c || ccert;
}

// ---------------------------------------------------------------------------------------
// obs row (MultiRaceAviary._computeObs, 566-661) written straight to global memory
// ---------------------------------------------------------------------------------------
template <typename Real, class TS>
__device__ __forceinline__ void race_obs_row_rpy(const RaceConst<Real>& C, const TS& T, V3<Real> pos, V3<Real> rpy,
                                                 V3<Real> vel, V3<Real> w, int gate, float* row, bool write, Real* row0,
                                                 uint32_t gin, uint32_t oin);
// the obs row from the pose quaternion (its Euler angles computed here)
template <typename Real, class TS>
__device__ __forceinline__ void race_obs_row(const RaceConst<Real>& C, const TS& T,
                                             V3<Real> pos, Q4<Real> q, V3<Real> vel, V3<Real> w, int gate,
                                             float* row, bool write, Real* row0, uint32_t gin, uint32_t oin,
                                             V3<Real>* rpy_out = nullptr) {
    const V3<Real> rpy = euler_xyz_fast_u(q);
    if (rpy_out) *rpy_out = rpy;
    race_obs_row_rpy(C, T, pos, rpy, vel, w, gate, row, write, row0, gin, oin);
}
// the obs row from given Euler angles (a reset's nominal pose: RaceConst::nom_rpy, the same bits
// euler_xyz_fast gives for nom_q)
template <typename Real, class TS>
__device__ __forceinline__ void race_obs_row_rpy(const RaceConst<Real>& C, const TS& T, V3<Real> pos, V3<Real> rpy,
                                                 V3<Real> vel, V3<Real> w, int gate, float* row, bool write, Real* row0,
                                                 uint32_t gin, uint32_t oin) {
    const Real k12[12] = {pos.x, pos.y, pos.z, rpy.x, rpy.y, rpy.z, vel.x, vel.y, vel.z, w.x, w.y, w.z};
    if (write)
#pragma unroll
        for (int k = 0; k < 12; ++k) row[k] = float(k12[k]);
    if (row0)
#pragma unroll
        for (int k = 0; k < 3; ++k) row0[k] = k12[k];
#pragma unroll
    for (int g = 0; g < ADRP_MAX_GATES; ++g) {
        Real v4[4] = {Real(0), Real(0), Real(0), Real(0)};
        Real in = 0;
        if (g < C.num_gates) {
            const V3<Real> org = v3(T(RF_GATE + 4 * g), T(RF_GATE + 4 * g + 1), T(RF_GATE + 4 * g + 2));
            const Real yaw = T(RF_GATE + 4 * g + 3);
            in = (gin >> g) & 1u ? Real(1) : Real(0);
            if (in > Real(0)) { v4[0] = org.x; v4[1] = org.y; v4[2] = org.z; v4[3] = yaw; }
            else {
#pragma unroll
                for (int j = 0; j < 4; ++j) v4[j] = C.gate_nom[g][j];
            }
        }
        if (write) {
#pragma unroll
            for (int j = 0; j < 4; ++j) row[12 + 4 * g + j] = float(v4[j]);
            row[28 + g] = float(in);
        }
        if (row0 && g < C.num_gates)
#pragma unroll
            for (int j = 0; j < 3; ++j) row0[3 + 3 * g + j] = v4[j];
    }
#pragma unroll
    for (int k = 0; k < ADRP_MAX_OBSTACLES; ++k) {
        Real v3_[3] = {Real(0), Real(0), Real(0)};
        Real in = 0;
        if (k < C.num_obstacles) {
            const V3<Real> org = v3(T(RF_OBST + 3 * k), T(RF_OBST + 3 * k + 1), T(RF_OBST + 3 * k + 2));
            in = (oin >> k) & 1u ? Real(1) : Real(0);
            if (in > Real(0)) { v3_[0] = org.x; v3_[1] = org.y; v3_[2] = org.z; }
            else {
#pragma unroll
                for (int j = 0; j < 3; ++j) v3_[j] = C.obst_nom[k][j];
            }
        }
        if (write) {
#pragma unroll
            for (int j = 0; j < 3; ++j) row[32 + 3 * k + j] = float(v3_[j]);
            row[44 + k] = float(in);
        }
    }
    if (write) row[48] = float(gate);
}

// ---------------------------------------------------------------------------------------
// reset of one drone (+ its env's replicated fields) -> state + initial obs row
// (MultiRaceAviary.reset 127-167, _addObstacles 347-403, _drone_init 407-467)
// ---------------------------------------------------------------------------------------
template <typename Real>
__device__ __forceinline__ void race_reset_lane(const RaceArgs<Real>& a, const RaceConst<Real>& C, int e, int dn, size_t EN,
                                size_t slot, int episode, float* obs_row) {
    const uint64_t gid = uint64_t(a.env_offset + e);
    const uint32_t ep = uint32_t(episode);
    Real* f = a.f;
    // track (every drone lane of the env computes the same draws)
    for (int g = 0; g < ADRP_MAX_GATES; ++g) {
        Real gx = C.gate_nom[g][0], gy = C.gate_nom[g][1], gyaw = C.gate_nom[g][3];
        if (C.random_gates && g < C.num_gates) {
            const U4 u = draw(a.seed, gid, ep, TAG_RACE_TRACK, uint32_t(g));
            const Real lo = C.gate_off[0], hi = C.gate_off[1];
            gx += lo + (hi - lo) * Real(u01(u.a));
            gy += lo + (hi - lo) * Real(u01(u.b));
            gyaw += lo + (hi - lo) * Real(u01(u.c));
        }
        st(f, RF_GATE + 4 * g, EN, slot, gx); st(f, RF_GATE + 4 * g + 1, EN, slot, gy);
        st(f, RF_GATE + 4 * g + 2, EN, slot, C.gate_nom[g][2]); st(f, RF_GATE + 4 * g + 3, EN, slot, gyaw);
    }
    for (int k = 0; k < ADRP_MAX_OBSTACLES; ++k) {
        Real ox = C.obst_nom[k][0], oy = C.obst_nom[k][1];
        if (C.random_gates && k < C.num_obstacles) {
            const U4 u = draw(a.seed, gid, ep, TAG_RACE_TRACK, uint32_t(4 + k));
            const Real lo = C.obst_off[0], hi = C.obst_off[1];
            ox += lo + (hi - lo) * Real(u01(u.a));
            oy += lo + (hi - lo) * Real(u01(u.b));
        }
        st(f, RF_OBST + 3 * k, EN, slot, ox); st(f, RF_OBST + 3 * k + 1, EN, slot, oy);
        st(f, RF_OBST + 3 * k + 2, EN, slot, C.obst_nom[k][2]);
    }
    // initial obs at the nominal (loadURDF) poses, at rest
    const V3<Real> npos = v3(C.init_pos[dn][0], C.init_pos[dn][1], C.init_pos[dn][2]);
    const Q4<Real> nq = nominal_q(C, dn);
    Real row0[15];
    const V3<Real> zero = v3(Real(0), Real(0), Real(0));
    uint32_t gin, oin;
    const TrackSrc<Real, false> T{f, EN, slot, nullptr, 0};   // the fields just written above
    track_query(C, T, drone_shape(C, npos, nq), Real(0.45), false, Real(0), gin, oin);
    race_obs_row_rpy(C, T, npos, nominal_rpy(C, dn), zero, zero, 0, obs_row, obs_row != nullptr, row0, gin, oin);
    if (C.compete && obs_row) {   // other drones' nominal pos + rpy
        int idx = 0;
        for (int k = 0; k < C.N; ++k) {
            if (k == dn) continue;
            const V3<Real> orpy = nominal_rpy(C, k);
            float* p = obs_row + 49 + 6 * idx;
            p[0] = float(C.init_pos[k][0]); p[1] = float(C.init_pos[k][1]); p[2] = float(C.init_pos[k][2]);
            p[3] = float(orpy.x); p[4] = float(orpy.y); p[5] = float(orpy.z);
            ++idx;
        }
    }
    const V3<Real> nrpy = nominal_rpy(C, dn);
    // RewardWrapper.reset: current_target = obs[0, 12:15], previous_pos = obs[0, :3]
    for (int k = 0; k < 3; ++k) {   // per-env state, kept in drone 0's slot
        st(f, RF_WR_TARGET + k, EN, slot, dn == 0 && C.num_gates > 0 ? row0[3 + k] : Real(0));
        st(f, RF_WR_PREV + k, EN, slot, dn == 0 ? row0[k] : Real(0));
    }
    // controller reset with the initial obs; _drone_init
    RDrone<Real> d;
    d.prev_rpy[0] = nrpy.x; d.prev_rpy[1] = nrpy.y; d.prev_rpy[2] = nrpy.z;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d.prev_vel[k] = Real(0); d.lpf1[k] = d.lpf2[k] = 0.0f; d.ierr[k] = d.ierrm[k] = 0.0f;
    }
    d.tick = d.last_att = d.last_pos = d.tumble = 0;
    d.pw_roll = d.pw_pitch = __builtin_nanf("");
    d.psp_roll = d.psp_pitch = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { d.ctl[k] = 0.0f; d.rpm[k] = d.prev[k] = Real(0); }
    d.gate = 0; d.flags = 0;
    d.mass = C.race_mass;
    d.inertia[0] = C.race_inertia[0]; d.inertia[1] = C.race_inertia[1]; d.inertia[2] = C.race_inertia[2];
    const uint32_t dtag = TAG_RACE_DRONE | uint32_t(dn);
    if (C.random_inertia) {
        const U4 u = draw(a.seed, gid, ep, dtag, 2);
        const uint32_t uu[4] = {u.a, u.b, u.c, u.d};
        Real v[4] = {d.mass, d.inertia[0], d.inertia[1], d.inertia[2]};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const Real lo = C.inertia_off[k][0], hi = C.inertia_off[k][1];
            v[k] = clampr_(v[k] + lo + (hi - lo) * Real(u01(uu[k])), Real(0), Real(100));
        }
        d.mass = v[0]; d.inertia[0] = v[1]; d.inertia[1] = v[2]; d.inertia[2] = v[3];
    }
    Real po[3] = {0, 0, 0}, ro[3] = {0, 0, 0};
    if (C.random_state) {
        const U4 u = draw(a.seed, gid, ep, dtag, 0), u2 = draw(a.seed, gid, ep, dtag, 1);
        const uint32_t a1[3] = {u.a, u.b, u.c}, a2[3] = {u2.a, u2.b, u2.c};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            po[k] = C.pos_off[k][0] + (C.pos_off[k][1] - C.pos_off[k][0]) * Real(u01(a1[k]));
            ro[k] = C.rot_off[k][0] + (C.rot_off[k][1] - C.rot_off[k][0]) * Real(u01(a2[k]));
        }
    }
    d.pos = v3(npos.x + po[0], npos.y + po[1], npos.z + po[2]);
    d.q = quat_from_euler_fast(C.init_rpy[dn][0] + ro[0], C.init_rpy[dn][1] + ro[1], C.init_rpy[dn][2] + ro[2]);
    d.vel = v3(C.init_vel[dn][0], C.init_vel[dn][1], C.init_vel[dn][2]);
    d.w = v3(C.init_pqr[dn][0], C.init_pqr[dn][1], C.init_pqr[dn][2]);
    d.angv = d.w;
    if (C.physics == ADRP_PHYS_DYN) d.w = v3(Real(0), Real(0), Real(0));   // rpy_rates zeroed by _housekeeping
    d.ql = d.q;
    d.lpos = d.pos;
    d.kpos = C.physics == ADRP_PHYS_PYB ? npos : d.pos;   // self.pos: nominal until the first read
    store_drone(a, EN, slot, d, true);
    a.ist[RI_STEP * EN + slot] = 0;
    a.ist[RI_EPISODE * EN + slot] = episode + 1;
    a.ist[RI_WR_GATE * EN + slot] = 0;
    if (a.cf) {   // command mode: MellingerControl.reset with the initial obs row (commander.h hl_reset)
        CmdState cs;
        hl_reset(cs, float(npos.x), float(npos.y), float(npos.z), float(nrpy.z * Real(57.29577951308232)));
        cmd_store(a.cf, a.ci, EN, slot, cs);
        for (int k = 0; k < 32; ++k) a.cf[size_t(CF_COEF + k) * EN + slot] = 0.0f;
    }
}

// command state of every drone as reset() leaves it (adrp_enable_commands): the initial obs is taken
// at the nominal pose, so this is exact for envs that have not stepped since their reset
template <typename Real>
__global__ void __launch_bounds__(kRaceBlock) race_cmd_init_kernel(RaceArgs<Real> a) {
    const RaceConst<Real>& C = *a.c;
    const size_t EN = size_t(a.E) * C.N;
    const size_t slot = size_t(blockIdx.x) * kRaceBlock + threadIdx.x;
    if (slot >= EN) return;
    const int dn = int(slot % C.N);
    const V3<Real> nrpy = nominal_rpy(C, dn);
    CmdState cs;
    hl_reset(cs, float(C.init_pos[dn][0]), float(C.init_pos[dn][1]), float(C.init_pos[dn][2]),
             float(nrpy.z * Real(57.29577951308232)));
    cmd_store(a.cf, a.ci, EN, slot, cs);
    for (int k = 0; k < 32; ++k) a.cf[size_t(CF_COEF + k) * EN + slot] = 0.0f;
}

// one command message per drone before the sub-steps (MultiRaceAviary.py:190-210; eliminated
// drones get STOP [step_counter]): commander.h hl_command on the stored command state
template <typename Real>
__global__ void __launch_bounds__(kRaceBlock) race_command_kernel(RaceArgs<Real> a) {
    const RaceConst<Real>& C = *a.c;
    const size_t EN = size_t(a.E) * C.N;
    const size_t slot = size_t(blockIdx.x) * kRaceBlock + threadIdx.x;
    if (slot >= EN) return;
    CmdState cs;
    cmd_load(a.cf, a.ci, EN, slot, cs);
    const double* args = a.cargs + slot * ADRP_CMD_ARGS;
    if (a.ist[RI_FLAGS * EN + slot] & 1) {
        double st[ADRP_CMD_ARGS] = {};
        st[ADRP_CMD_TIME_SLOT] = double(a.ist[RI_STEP * EN + slot]);
        hl_command(cs, a.cf + size_t(CF_COEF) * EN, EN, slot, ADRP_CMD_STOP, st, false);
    } else {
        hl_command(cs, a.cf + size_t(CF_COEF) * EN, EN, slot, a.cmd[slot], args, C.obs_wrapper != 0);
    }
    cmd_store(a.cf, a.ci, EN, slot, cs);
}

// ---------------------------------------------------------------------------------------
// env.step kernel
// ---------------------------------------------------------------------------------------
// The 7 disturbance values of one drone and sub-step (MultiRaceAviary.py:222-228, 532-544): the
// world force U(lo, hi) on link 4 and the N(0, std) thrust noise per motor (Box-Muller pairs).
// The Gaussian samples come from the hardware log2 / sin / cos (float) in both precisions: they
// are random numbers of a documented Philox stream (DESIGN.md §6 deviation 5), not a computation
// of the reference's; the fp64 kernel widens them (its force draws stay in Real).
template <typename Real>
__device__ __forceinline__ void race_noise_draws(const RaceConst<Real>& H, uint64_t seed, uint64_t gid, uint32_t ep,
                                                 int dn, uint32_t idx, Real noise[4]) {
    const U4 v = draw(seed, gid, ep, TAG_RACE_NOISE | uint32_t(dn), idx);
    if constexpr (sizeof(Real) == 8) {   // the oracle's Box-Muller, bit for bit (normal_pair_f)
        float z[4];
        normal_pair_f(v.a, v.b, &z[0], &z[1]);
        normal_pair_f(v.c, v.d, &z[2], &z[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k) noise[k] = Real(z[k]) * H.noise_std;
        return;
    }
    // fp32: hardware log2 / sin / cos (the samples differ from the oracle's by float rounding)
    const uint32_t x[4] = {v.a, v.b, v.c, v.d};
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const float u1 = (float(x[2 * p] >> 8) + 1.0f) * float(1.0 / 16777216.0);
        const float u2 = float(x[2 * p + 1] >> 8) * float(1.0 / 16777216.0);
        // v_log_f32 is log2; v_sin / v_cos take turns
        const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
        const float sn = __builtin_amdgcn_sinf(u2), cs = __builtin_amdgcn_cosf(u2);
        noise[2 * p] = Real(r * cs) * H.noise_std;
        noise[2 * p + 1] = Real(r * sn) * H.noise_std;
    }
}

template <typename Real>
__device__ __forceinline__ void race_substep_draws(const RaceConst<Real>& H, uint64_t seed, uint64_t gid, uint32_t ep,
                                                   int dn, uint32_t idx, Real fd[3], Real noise[4]) {
    const U4 u = draw(seed, gid, ep, TAG_RACE_DIST | uint32_t(dn), idx);
    fd[0] = H.dist_lo[0] + (H.dist_hi[0] - H.dist_lo[0]) * u01r<Real>(u.a);
    fd[1] = H.dist_lo[1] + (H.dist_hi[1] - H.dist_lo[1]) * u01r<Real>(u.b);
    fd[2] = H.dist_lo[2] + (H.dist_hi[2] - H.dist_lo[2]) * u01r<Real>(u.c);
    race_noise_draws(H, seed, gid, ep, dn, idx, noise);
}

// parity mode (adrp_set_noise): the caller's draws of sub-step s of drone slot instead of Philox's
template <typename Real>
__device__ __forceinline__ void injected_draws(const RaceArgs<Real>& a, size_t slot, int S, int s, Real fd[3],
                                               Real noise[4]) {
    const double* pf = a.inj_force + (slot * S + s) * 3;
    const double* pa = a.inj_act + (slot * S + s) * 4;
#pragma unroll
    for (int k = 0; k < 3; ++k) fd[k] = Real(pf[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) noise[k] = Real(pa[k]);
}
// Block = kRaceBlock drone lanes.  Wave 0 runs the serial sub-step chain (physics -> controller ->
// physics ...; one wave per CU at the race batch sizes, one instruction per 4 cycles).  With
// disturbances on, kRaceHelpers more waves, on the CU's otherwise idle SIMDs, pre-compute every
// sub-step's draws into LDS while wave 0 loads its state; the chain then reads 7 values per
// sub-step instead of running two Philox4x32-10 draws and a Box-Muller pair (~200 instructions).
// PRE: helper waves present (fp32; the host then launches kRaceBlock * (1 + kRaceHelpers)
// threads per block): 2 = the sub-step draws (disturbances on, S <= kRacePreS), 1 = no draws to
// make, so they copy the env's actual track (28 fields per lane) into LDS for the post-loop
// queries instead (A/B: the copy pays without disturbances, but not on top of the draws).
// CMD: command mode (adrp_enable_commands): the setpoint comes from the command state (commander.h),
// with a non-null act first turned into a FULLSTATE command; no helper waves.
template <typename Real, int PH, int G, int PRE, bool CMD = false>
__global__ void __launch_bounds__(kRaceBlock * (PRE ? 1 + kRaceHelpers : 1)) race_step_kernel(RaceArgs<Real> a) {
    RACE_MARK(t0);
    const RaceConst<Real>& C = *a.c;
    static_assert(!PRE || sizeof(Real) == 4, "pre-computed draws: fp32 kernel only");
    static_assert(!(CMD && PRE), "command mode: no helper waves");
    __shared__ float pre_draws[PRE == 2 ? kRacePreS * 7 * kRaceBlock : 1];
    __shared__ float trk_lds[PRE == 1 ? kTrackFields * kRaceBlock : 1];
    // the block's obs rows, laid out as in global memory (its envs' rows are contiguous there),
    // so the copy-out is coalesced: direct per-lane row stores touch a line per lane per float
    __shared__ float4 rows4[kRaceBlock * kRaceMaxD / 4];
    __shared__ TrackJobs tjobs;
    constexpr bool pre = PRE == 2;
    const int tl = threadIdx.x % kRaceBlock;
    // Barrier protocol (every wave passes the same count before the helpers exit):
    //   PRE == 2: helpers  B1 after the draws of s < S/2, B2 after the rest;
    //             chain    B1 before the sub-step loop,  B2 at s == S/2 (reached once for every
    //                      1 <= S <= kRacePreS: S/2 < S; S = 1 puts it on s = 0, right after B1).
    //   PRE == 1: helpers  B2 after the track copy;  chain  B2 after the sub-step loop.
    // Later barriers (GJK pooling, copy-out) see only the chain wave: exited waves do not count.
    // test_helper_waves_bit_identical runs S = 20, 5 and 1 with and without the helpers.
    if (threadIdx.x >= kRaceBlock) {   // helper waves
        if constexpr (PRE) {
            const int hw = int(threadIdx.x / kRaceBlock) - 1;
            const int hl = blockIdx.x * kRaceBlock + tl;
            const int he = hl / G < a.E ? hl / G : a.E - 1, hd = hl % G < C.N ? hl % G : 0;
            const size_t hEN = size_t(a.E) * C.N, hslot = size_t(he) * C.N + hd;
            const int hsc0 = a.ist[RI_STEP * hEN + hslot];
            const uint32_t hep = uint32_t(a.ist[RI_EPISODE * hEN + hslot] - 1);
            const uint64_t hgid = uint64_t(a.env_offset + he);
            // PRE == 2: sub-steps [0, S/2) before the chain's loop starts, the rest by its middle
            const int half = C.S / 2;
            for (int part = 0; pre && part < 2; ++part) {
                for (int s = hw; s < C.S; s += kRaceHelpers) {
                    if ((s < half) != (part == 0)) continue;
                    Real fd[3], nz[4];
                    if (a.inj_force) injected_draws(a, hslot, C.S, s, fd, nz);
                    else race_substep_draws(C, a.seed, hgid, hep, hd, uint32_t(hsc0 + s), fd, nz);
                    float* dst = pre_draws + s * 7 * kRaceBlock + tl;
#pragma unroll
                    for (int k = 0; k < 3; ++k) dst[k * kRaceBlock] = float(fd[k]);
#pragma unroll
                    for (int k = 0; k < 4; ++k) dst[(3 + k) * kRaceBlock] = float(nz[k]);
                }
                if (part == 0) __syncthreads();   // first half in LDS
            }
            // PRE == 1: the track copy, off the chain's critical path (read after the loop)
            for (int k = hw; PRE == 1 && k < kTrackFields; k += kRaceHelpers)
                trk_lds[k * kRaceBlock + tl] = float(ld(a.f, RF_GATE + k, hEN, hslot));
            __syncthreads();   // draws (before the chain's loop) / track (after it) in LDS
        }
        return;
    }
    // register copy of the constants the sub-step loop reads (uniform -> SGPRs; no reloads
    // behind the state stores, which the compiler cannot prove do not alias a.c)
    RaceConst<Real> H;
    H.S = C.S; H.link_lag = C.link_lag; H.disturbances = C.disturbances;
    H.dt = C.dt; H.gravity = C.gravity; H.kf = C.kf; H.km = C.km;
#pragma unroll
    for (int i = 0; i < 4; ++i) { H.px[i] = C.px[i]; H.py[i] = C.py[i]; H.pz[i] = C.pz[i]; }
    H.gnd_kf = C.gnd_kf; H.prop_r4 = C.prop_r4; H.gnd_clip = C.gnd_clip;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        H.drag[i] = C.drag[i]; H.dist_lo[i] = C.dist_lo[i]; H.dist_hi[i] = C.dist_hi[i];
        H.dyn_i[i] = C.dyn_i[i]; H.dyn_inv_i[i] = C.dyn_inv_i[i];
    }
    H.dw1 = C.dw1; H.dw2 = C.dw2; H.dw3 = C.dw3; H.prop_r = C.prop_r;
    H.dyn_mass = C.dyn_mass; H.dyn_inv_mass = C.dyn_inv_mass; H.dyn_arm = C.dyn_arm;
    H.coll_hh = C.coll_hh; H.coll_r = C.coll_r; H.coll_zoff = C.coll_zoff; H.ang_max = C.ang_max;
    H.noise_std = C.noise_std;
    const int lane = blockIdx.x * kRaceBlock + tl;
    const int e_raw = lane / G, d_raw = lane % G;
    const int N = C.N;
    const bool active = e_raw < a.E && d_raw < N;
    const int e = e_raw < a.E ? e_raw : a.E - 1;
    const int dn = d_raw < N ? d_raw : 0;
    const size_t EN = size_t(a.E) * N;
    const size_t slot = size_t(e) * N + dn;
    const uint64_t gid = uint64_t(a.env_offset + e);
    RDrone<Real> d;
    load_drone(a, EN, slot, d);
    const int sc0 = a.ist[RI_STEP * EN + slot];
    const int episode = a.ist[RI_EPISODE * EN + slot];
    const uint32_t ep = uint32_t(episode - 1);
    // FULLSTATE setpoint (MultiRaceAviary.py:190-194; _sendFullStateCmd 510-543)
    const float4 av = CMD && !a.act ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : reinterpret_cast<const float4*>(a.act)[slot];
    CmdState cs;
    float* const coefp = CMD ? a.cf + size_t(CF_COEF) * EN : nullptr;
    if constexpr (CMD) {   // the step's command message (MultiRaceAviary.py:190-210)
        cmd_load(a.cf, a.ci, EN, slot, cs);
        double ca[ADRP_CMD_ARGS] = {};
        ca[ADRP_CMD_TIME_SLOT] = double(sc0);
        if (d.flags & 1) {
            hl_command(cs, coefp, EN, slot, ADRP_CMD_STOP, ca, false);
        } else if (a.act) {
            ca[0] = av.x; ca[1] = av.y; ca[2] = av.z; ca[9] = av.w;
            hl_command(cs, coefp, EN, slot, ADRP_CMD_FULLSTATE, ca, C.obs_wrapper != 0);
        }
    }
    const float sp[3] = {av.x, av.y, av.z};
    float xc_x, xc_y;
    {
#pragma clang fp contract(off)
        Real qs, qc;
        // get_quaternion_from_euler(0, 0, yaw); DroneObservationWrapper zeroes the yaw (wrapper.py:51-57)
        sincos_(Real(C.obs_wrapper ? 0.0f : av.w) * Real(0.5), &qs, &qc);
        const float qz = float(qs), qw = float(qc);
        const float yaw_deg = degf_(atan2f(2.0f * (qw * qz + 0.0f * 0.0f), 1 - 2 * (0.0f * 0.0f + qz * qz)));
        xc_x = cosf(radf_(yaw_deg));
        xc_y = sinf(radf_(yaw_deg));
    }
    const Lpf lpf = {C.lpf[0], C.lpf[1], C.lpf[2], C.lpf[3], C.lpf[4]};   // lpf2pInit(gyrolpf, 500, 30), host
    if constexpr (PRE == 2) __syncthreads();   // the helpers' first half of the draws is in LDS
    // diagnostics level 2: the step's firmware moments, call by call (adrp_race_moment_log)
    int16_t* mlog = a.mom_log ? a.mom_log + slot * size_t(3 * H.S) : nullptr;
    int mcount = 0;
    RACE_MARK(t1);
#ifdef ADRP_RACE_TIMING
    uint64_t acc_phys = 0;
#endif
    for (int s0 = 0; s0 < H.S; s0 += 32) {   // chunks of the 32-tick schedule windows (S > 32 only)
    if (s0 > 0) {
        d.tick_base = d.tick;
        tick_window(a.ticks, d.tick, d.att_bits, d.pos_bits);
    }
    const int s1 = H.S < s0 + 32 ? H.S : s0 + 32;
    for (int s = s0; s < s1; ++s) {
#ifdef ADRP_RACE_TIMING
        RACE_MARK(ta);
#endif
        if constexpr (PRE == 2) {
            if (s == H.S / 2) __syncthreads();   // the helpers' second half of the draws
        }
        const uint32_t idx = uint32_t(sc0 + s);
        if (PH != ADRP_PHYS_PYB) d.kpos = d.pos;          // KIN_PHYSICS read-back
        if constexpr (PH == ADRP_PHYS_DYN) {
            race_dyn_substep(H, d);
        } else {
            V3<Real> Fx = v3(Real(0), Real(0), Real(0)), Tx = v3(Real(0), Real(0), Real(0));
            if constexpr (PH == ADRP_PHYS_PYB_DW || PH == ADRP_PHYS_PYB_GND_DRAG_DW) {
                // _downwash (BaseAviary.py:792-818): every other drone above, LINK_FRAME on link 4
                Real fz = 0;
                constexpr bool F32 = sizeof(Real) == 4;
#pragma unroll
                for (int k = 0; k < G; ++k) {   // all shuffles in flight at once
                    const Real ox = grp_bcast<G>(d.pos.x, k), oy = grp_bcast<G>(d.pos.y, k), oz = grp_bcast<G>(d.pos.z, k);
                    const Real dz = oz - d.pos.z, dx = ox - d.pos.x, dy = oy - d.pos.y;
                    const Real dxy = hsqrt_(dx * dx + dy * dy);
                    if (k < N && dz > Real(0) && dxy < Real(10)) {
                        const Real kk = F32 ? H.prop_r * rcp_(Real(4) * dz) : H.prop_r / (Real(4) * dz);
                        const Real alpha = H.dw1 * kk * kk, beta = H.dw2 * dz + H.dw3;
                        const Real q = F32 ? dxy * rcp_(beta) : dxy / beta;
                        fz -= alpha * fexp_(Real(-0.5) * q * q);
                    }
                }
                const M3<Real> Rs = H.link_lag && !(PH == ADRP_PHYS_PYB_GND_DRAG_DW) ? rot(d.ql) : rot(d.q);
                Fx = fz * col2(Rs);
            }
            if (H.disturbances) {   // world-frame force on link 4 at posObj = self.pos (532-544)
                V3<Real> fd;
                if (pre) {
                    const float* src = pre_draws + s * 7 * kRaceBlock + tl;
                    fd = v3(Real(src[0]), Real(src[kRaceBlock]), Real(src[2 * kRaceBlock]));
                } else {
                    Real f3[3], nz[4];
                    if (a.inj_force) injected_draws(a, slot, H.S, s, f3, nz);
                    else race_substep_draws(H, a.seed, gid, ep, dn, idx, f3, nz);
                    fd = v3(f3[0], f3[1], f3[2]);
                }
                const V3<Real> lo = (PH == ADRP_PHYS_PYB_GND || PH == ADRP_PHYS_PYB_GND_DRAG_DW) ? d.pos : d.lpos;
                Fx = Fx + fd;
                Tx = cross(d.kpos - lo, fd);
            }
            race_pyb_substep<Real, PH>(H, d, Fx, Tx);
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
            Real noise[4] = {Real(0), Real(0), Real(0), Real(0)};
            if (H.disturbances) {
                if (pre) {
                    const float* src = pre_draws + (s * 7 + 3) * kRaceBlock + tl;
#pragma unroll
                    for (int k = 0; k < 4; ++k) noise[k] = Real(src[k * kRaceBlock]);
                } else {
                    Real f3[3];
                    if (a.inj_force) injected_draws(a, slot, H.S, s, f3, noise);
                    else race_substep_draws(H, a.seed, gid, ep, dn, idx, f3, noise);
                }
            }
            mellinger_compute<Real, CMD>(d, lpf, sp, xc_x, xc_y, euler_xyz_fast_u(d.q), noise, &cs, coefp, EN, slot,
                                         mlog, &mcount);
        }
    }
    }
    RACE_MARK(t2);
    if (mlog) a.mom_log_n[slot] = mcount;
    if constexpr (PRE == 1) __syncthreads();   // the helpers' track copy is in LDS
    const TrackSrc<Real, PRE == 1> T{a.f, EN, slot, trk_lds, tl};
    // ---- _gate_progress (471-506): rays of my current gate vs every drone of the env ----
    V3<Real> gpos[ADRP_MAX_DRONES];
    Q4<Real> gq[ADRP_MAX_DRONES];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        gpos[k] = v3(grp_bcast<G>(d.pos.x, k), grp_bcast<G>(d.pos.y, k), grp_bcast<G>(d.pos.z, k));
        gq[k] = {grp_bcast<G>(d.q.x, k), grp_bcast<G>(d.q.y, k), grp_bcast<G>(d.q.z, k), grp_bcast<G>(d.q.w, k)};
    }
    const int gate0 = d.gate;
    if (C.num_gates > 0 && gate0 < C.num_gates) {
        const Real gx = T(RF_GATE + 4 * gate0), gy = T(RF_GATE + 4 * gate0 + 1);
        const Real rotg = T(RF_GATE + 4 * gate0 + 3);
        const Real h = C.gate_type[gate0] == 0 ? Real(1.0) : Real(0.525), half = Real(0.1875);
        Real sn, cs;
        sincos_f_(rotg, &sn, &cs);
        const Real dx = Real(0.05) * cs, dy = Real(0.05) * sn;
        // the 7 rays span the rectangle {g + t u + z e_z : |t| <= 0.15, |z - h| <= half};
        // drones whose bounding sphere (about pos: |z offset| + cylinder radius) misses it
        // cannot be hit, and a pass needs this lane's own drone to be hit
        const Real br = fabs_(C.coll_zoff) + hsqrt_(C.coll_r * C.coll_r + C.coll_hh * C.coll_hh) +
                        (sizeof(Real) == 4 ? Real(1e-5) : Real(1e-10));
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
    float* row = rows + ((tl / G) * N + dn) * C.D;   // staged; inactive lanes write nothing
    Real row0[15];
    const Shape<Real> ds = drone_shape(C, d.pos, d.q);
    uint32_t gin, oin;
    bool crashed = track_query_wave(C, T, ds, active, !(d.flags & 1), Real(0.45), Real(1e-6), gin, oin, tjobs, tl, G, N, a.E);
    V3<Real> rpy;
    race_obs_row(C, T, d.pos, d.q, d.vel, wv, d.gate, row, active, row0, gin, oin, &rpy);
    if (C.compete) {   // other drones' pos + rpy (653-659): the rpy of their own obs rows
        V3<Real> grpy[ADRP_MAX_DRONES];
#pragma unroll
        for (int k = 0; k < G; ++k) grpy[k] = v3(grp_bcast<G>(rpy.x, k), grp_bcast<G>(rpy.y, k), grp_bcast<G>(rpy.z, k));
        int idx = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (active && k < N && k != dn) {
                const V3<Real> orpy = grpy[k];
                float* p = row + 49 + 6 * idx;
                p[0] = float(gpos[k].x); p[1] = float(gpos[k].y); p[2] = float(gpos[k].z);
                p[3] = float(orpy.x); p[4] = float(orpy.y); p[5] = float(orpy.z);
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
                if (k < N && k != dn && !crashed && !(d.flags & 1)) {
                    // bounding spheres first: GJK only for drones closer than 2 dr
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
    // per-env reduction over the drone lanes
    const int mydone = ((d.flags & 1) || (d.flags & 2)) ? 1 : 0, myfin = (d.flags & 2) ? 1 : 0;
    int all_done = 1, all_fin = 1;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        if (k < N) {
            all_done &= grp_bcast_i<G>(mydone, k);
            all_fin &= grp_bcast_i<G>(myfin, k);
        }
    }
    // DroneObservationWrapper: terminated once drone 0's current gate >= 2 (wrapper.py:61-63)
    const int gate_d0 = grp_bcast_i<G>(d.gate, 0);
    const bool te_env = all_done != 0;
    const bool te = te_env || (C.obs_wrapper && gate_d0 >= 2);
    const bool te_rw = C.obs_wrapper == 1 ? te : te_env;   // what the RewardWrapper sees
    const bool tr = sc0 >= C.trunc_steps;   // step_counter / PYB_FREQ > episode_len_sec, before += S
    // ---- RewardWrapper (wrapper.py:121-186), drone 0 ----
    float reward = 0.0f;
    int wr_gate = a.ist[RI_WR_GATE * EN + slot];
    if (C.reward_wrapper && dn == 0) {
        const int gate_id = d.gate;
        Real tgt[3] = {ld(a.f, RF_WR_TARGET, EN, slot), ld(a.f, RF_WR_TARGET + 1, EN, slot), ld(a.f, RF_WR_TARGET + 2, EN, slot)};
        const Real prv[3] = {ld(a.f, RF_WR_PREV, EN, slot), ld(a.f, RF_WR_PREV + 1, EN, slot), ld(a.f, RF_WR_PREV + 2, EN, slot)};
        Real r_passed = 0;
        if (gate_id > wr_gate % 4) {
            wr_gate = gate_id;
            if (gate_id < 4 && gate_id < C.num_gates) {
                // row0[3 + 3 gate_id + k] by selects: a lane-varying index would put row0 in scratch
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int k = 0; k < 3; ++k) tgt[k] = g == gate_id ? row0[3 + 3 * g + k] : tgt[k];
            }
            r_passed = Real(5);
        }
        const Real r_col = (te_rw && !all_fin) ? Real(-1) : Real(0), r_lab = (te_rw && all_fin) ? Real(10) : Real(0);
        const Real pxy = sqrt_((tgt[0] - prv[0]) * (tgt[0] - prv[0]) + (tgt[1] - prv[1]) * (tgt[1] - prv[1]));
        const Real cxy = sqrt_((tgt[0] - row0[0]) * (tgt[0] - row0[0]) + (tgt[1] - row0[1]) * (tgt[1] - row0[1]));
        const Real pz = fabs_(tgt[2] - prv[2]), cz = fabs_(tgt[2] - row0[2]);
        reward = float((pxy - cxy) + (pz - cz) + r_passed + r_col + r_lab);
        if (active)
            for (int k = 0; k < 3; ++k) { st(a.f, RF_WR_TARGET + k, EN, slot, tgt[k]); st(a.f, RF_WR_PREV + k, EN, slot, row0[k]); }
    }
#ifdef ADRP_RACE_TIMING
    RACE_MARK(t6);
    if (threadIdx.x == 0) {
        RACE_ACC(0, t1 - t0); RACE_ACC(1, acc_phys); RACE_ACC(2, (t2 - t1) - acc_phys); RACE_ACC(3, t3 - t2);
        RACE_ACC(4, t4 - t3); RACE_ACC(5, t5 - t4); RACE_ACC(6, t6 - t5); RACE_ACC(7, t6 - t0); RACE_ACC(8, 1);
    }
#endif
    if (active) {
        if (dn == 0) {
            a.rew[e] = reward;
            a.term[e] = te;
            a.trunc[e] = tr;
        }
        if (C.autoreset && (te || tr)) {
            if (a.tobs) {
                float* trow = a.tobs + slot * size_t(C.D);
                for (int k = 0; k < C.D; ++k) trow[k] = row[k];
            }
            race_reset_lane(a, C, e, dn, EN, slot, episode, row);
        } else {
            store_drone(a, EN, slot, d, false);
            a.ist[RI_STEP * EN + slot] = sc0 + C.S;
            if (dn == 0) a.ist[RI_WR_GATE * EN + slot] = wr_gate;
            if constexpr (CMD) cmd_store(a.cf, a.ci, EN, slot, cs);
        }
    }
    // ---- coalesced copy-out of the block's rows (envs e0 .. e0 + ne - 1) ----
    __syncthreads();   // (the helper waves have ended)
    const int e0 = blockIdx.x * (kRaceBlock / G);
    const int ne = a.E - e0 < kRaceBlock / G ? a.E - e0 : kRaceBlock / G;
    const int total = ne * N * C.D;
    float* dst = a.obs + size_t(e0) * N * C.D;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        float4* dst4 = reinterpret_cast<float4*>(dst);
        const int n4 = total >> 2;
        for (int i = tl; i < n4; i += kRaceBlock) store_out(dst4 + i, rows4[i]);
        for (int i = 4 * n4 + tl; i < total; i += kRaceBlock) dst[i] = rows[i];
    } else {
        for (int i = tl; i < total; i += kRaceBlock) dst[i] = rows[i];
    }
}

// reset kernel (MultiRaceAviary.reset): masked envs, one lane per drone
template <typename Real>
__global__ void __launch_bounds__(kRaceBlock) race_reset_kernel(RaceArgs<Real> a) {
    const RaceConst<Real>& C = *a.c;
    const int lane = blockIdx.x * kRaceBlock + threadIdx.x;
    const int e = lane / C.N, dn = lane % C.N;
    if (e >= a.E || (a.mask && !a.mask[e])) return;
    const size_t EN = size_t(a.E) * C.N, slot = size_t(e) * C.N + dn;
    const int episode = a.ist[RI_EPISODE * EN + slot];
    race_reset_lane(a, C, e, dn, EN, slot, episode, a.obs + slot * size_t(C.D));
}

}  // namespace adrp
