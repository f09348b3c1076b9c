/*
 * race.c — TEST INFRASTRUCTURE ONLY.  MultiRaceAviary part of the CPU oracle; textually
 * included at the end of oracle.c (it shares that file's static helpers and handle).
 *
 * One env.step (MultiRaceAviary.step, envs/MultiRaceAviary.py:171-270):
 *   per drone: FULLSTATE setpoint from the action (190-202);
 *   S = pyb_freq/ctrl_freq sub-steps, each:
 *     _apply_physics with the rpms of the previous controller call (510-548, incl. the
 *       level1-3 world-frame disturbance force at posObj = self.pos),
 *     Bullet step of all drones (the btMultiBody restatement in oracle.c),
 *     state read-back, action noise N(0, std) (223-228),
 *     per drone (eliminated drones get 0 rpm): MellingerControl.computeControl
 *       (control/MellingerControl.py:154-262) = wrapper in float64 + the Crazyflie
 *       firmware controllerMellinger / lpf2p in C float (restated, parity unpinned);
 *   _gate_progress (471-506): 7 vertical rays per drone, first hit;
 *   _computeObs (566-661), _computeTerminated (674-698), _computeTruncated (702-709),
 *   optional RewardWrapper (utils/wrapper.py:121-186), auto-reset.
 * Geometry (contacts, getClosestPoints range, rays) uses the URDF collision shapes
 * (assets/cf2x_IROS.urdf:32-37, portal.urdf, low_portal.urdf, obstacle.urdf) with a GJK
 * distance; gates and obstacles are static.
 */

/* ---------------------------------------------------------------------------------- */
/* constants                                                                          */
/* ---------------------------------------------------------------------------------- */
#define FIRMWARE_FREQ 500
#define FIRMWARE_DT (1.0 / 500)
#define RAD_TO_DEG (180 / PI)
#define DEG_TO_RAD (PI / 180)
#define VISIBILITY_RANGE 0.45
#define TAG_RACE_TRACK 0x52540000u   /* gate / obstacle offsets, idx = gate or 4 + obstacle */
#define TAG_RACE_DRONE 0x52440000u   /* | drone: idx 0 pos offsets + idx 1 rot offsets, 2 inertia */
#define TAG_RACE_NOISE 0x524e0000u   /* | drone: idx = step_counter + s, 4 normals */
#define TAG_RACE_DIST 0x52460000u    /* | drone: idx = step_counter + s, 3 uniforms */

/* Crazyflie firmware (controller_mellinger.c defaults, CF2 platform) */
#define MEL_MASS 0.027f
#define MEL_MASS_THRUST 132000.0f
#define MEL_KP_XY 0.4f
#define MEL_KD_XY 0.2f
#define MEL_KI_XY 0.05f
#define MEL_I_RANGE_XY 2.0f
#define MEL_KP_Z 1.25f
#define MEL_KD_Z 0.4f
#define MEL_KI_Z 0.05f
#define MEL_I_RANGE_Z 0.4f
#define MEL_KR_XY 70000.0f
#define MEL_KW_XY 20000.0f
#define MEL_KI_M_XY 0.0f
#define MEL_I_RANGE_M_XY 1.0f
#define MEL_KR_Z 60000.0f
#define MEL_KW_Z 12000.0f
#define MEL_KI_M_Z 500.0f
#define MEL_I_RANGE_M_Z 1500.0f
#define MEL_KD_OMEGA_RP 200.0f
#define GRAVITY_MAGNITUDE 9.81f
#define M_PI_F 3.14159265358979323846f

/* ---------------------------------------------------------------------------------- */
/* race state                                                                          */
/* ---------------------------------------------------------------------------------- */
typedef struct rdrone_s {
    double rpm[4], prev_rpm[4];      /* self.rpms / self.prev_rpms (MultiRaceAviary.py:120-121) */
    v3 kin_pos;                      /* self.pos as the env last read it (disturbance posObj) */
    double mass; v3 inertia;         /* changeDynamics after _drone_init (MultiRaceAviary.py:426-432) */
    /* MellingerControl wrapper (float64) */
    double prev_rpy[3], prev_vel[3];
    int tick, last_att_tick, last_pos_tick, tumble;
    /* firmware (C float) */
    float lpf_d1[3], lpf_d2[3];      /* gyro lpf2pData delay elements */
    float i_err[3], i_err_m[3];
    float prev_omega_roll, prev_omega_pitch, prev_sp_roll, prev_sp_pitch;
    float ctl[4];                    /* control_t roll, pitch, yaw (int16 values), thrust */
    float mom_margin;                /* diagnostic, not state: over this env.step's firmware calls, the
                                        smallest distance of a clamped moment to a point where its int16
                                        truncation changes (a nonzero integer) */
    uint32_t mom_hash;               /* diagnostic, not state: fw_moment_hash over this env.step's firmware
                                        calls (the kernel's adrp_race_moment_hash) */
    const int16_t* rp_mom;           /* diagnostic, not state: the kernel's int16 moments of this env.step's
                                        firmware calls to use instead of this restatement's truncation
                                        (orc_race_set_moment_replay), or NULL */
    int rp_n, rp_call;               /* calls recorded, calls made so far this env.step */
    /* race progress */
    int gate, elim, fin;
    /* command state (adrp.h ADRP_CMD_NF / ADRP_CMD_NI order): setpoint_t fields the controller
       reads, the high-level commander's pos / vel / yaw, the firmware state_t of the last
       _update_state, the planner's single-piece trajectory */
    float sp_pos[3], sp_vel[3], sp_acc[3], sp_rate[3], sp_qz, sp_qw, sp_yaw;
    float c_pos[3], c_vel[3], c_yaw;
    float st_pos[3], st_vel[3], st_yaw;
    float plan_t0, plan_dur, coef[4][8];
    int plan_state, override, sp_mode;
} rdrone_t;

typedef struct renv_s {
    double gate[ADRP_MAX_GATES][4];      /* actual x, y, z, yaw */
    double obst[ADRP_MAX_OBSTACLES][3];  /* actual x, y, z */
    int wr_gate;                          /* RewardWrapper.current_gate_id */
    double wr_target[3], wr_prev[3];      /* RewardWrapper.current_target / previous_pos */
} renv_t;

/* lpf2p coefficients (firmware filter.c lpf2pSetCutoffFreq), float */
typedef struct { float b0, b1, b2, a1, a2; } lpf_t;
static lpf_t lpf_coeffs(float sample_freq, float cutoff_freq) {
    lpf_t l;
    float fr = sample_freq / cutoff_freq;
    float ohm = tanf(M_PI_F / fr);
    float c = 1.0f + 2.0f * cosf(M_PI_F / 4.0f) * ohm + ohm * ohm;
    l.b0 = ohm * ohm / c;
    l.b1 = 2.0f * l.b0;
    l.b2 = l.b0;
    l.a1 = 2.0f * (ohm * ohm - 1.0f) / c;
    l.a2 = (1.0f - 2.0f * cosf(M_PI_F / 4.0f) * ohm + ohm * ohm) / c;
    return l;
}
static float lpf_apply(const lpf_t* l, float* d1, float* d2, float sample) {
    float d0 = sample - *d1 * l->a1 - *d2 * l->a2;
    if (!isfinite(d0)) d0 = sample;
    float out = d0 * l->b0 + *d1 * l->b1 + *d2 * l->b2;
    *d2 = *d1;
    *d1 = d0;
    return out;
}

/* ---------------------------------------------------------------------------------- */
/* firmware controllerMellinger (restated; C float arithmetic)                         */
/* ---------------------------------------------------------------------------------- */
static float clampf_(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static float radiansf_(float d) { return (M_PI_F / 180.0f) * d; }
static float degreesf_(float r) { return (180.0f / M_PI_F) * r; }

typedef struct { float x, y, z; } f3;
static f3 F3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static float f3dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static f3 f3cross(f3 a, f3 b) { return F3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static f3 f3norm(f3 a) {
    float m = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return F3(a.x / m, a.y / m, a.z / m);
}

/* the int16 moments of one firmware call folded into the step's hash (FNV-1a over the int32 values;
   include/adrp.h adrp_race_moment_hash, race_kernel.h fw_moment_hash) */
#define MOM_HASH_SEED 2166136261u
static uint32_t fw_moment_hash(uint32_t h, float r, float p, float y) {
    h = (h ^ (uint32_t)(int32_t)r) * 16777619u;
    h = (h ^ (uint32_t)(int32_t)p) * 16777619u;
    return (h ^ (uint32_t)(int32_t)y) * 16777619u;
}

static void mellinger_reset(rdrone_t* d) {   /* controllerMellingerReset */
    for (int k = 0; k < 3; ++k) { d->i_err[k] = 0; d->i_err_m[k] = 0; }
}

enum { SP_UNSET = 0, SP_FULLSTATE = 1, SP_COMMANDER = 2 };   /* setpoint_t modes the controller sees */

/* controllerMellinger(control, setpoint, sensors, state, tick).  Setpoint modes:
 *   SP_FULLSTATE (MellingerControl._sendFullStateCmd, MellingerControl.py:510-543): x,y,z,quat
 *     modeAbs, roll/pitch/yaw modeDisable -> desiredYaw from the quaternion;
 *   SP_COMMANDER (crtpCommanderHighLevelGetSetpoint): x,y,z,yaw modeAbs, quat modeDisable ->
 *     desiredYaw = attitude.yaw;
 *   SP_UNSET (the zeroed setpoint_t of reset(), MellingerControl.py:121, before any command):
 *     every mode modeDisable -> thrust direction (-sin(pitch), -sin(roll), 1) with roll = pitch = 0
 *     and desiredYaw 0. */
static void mellinger_fw(rdrone_t* d, const float gyro[3], const float st_pos[3], const float st_vel[3],
                         const float st_q[4], int tick) {
    if (tick % 2 != 0) return;   /* RATE_DO_EXECUTE(ATTITUDE_RATE = 500, tick), RATE_MAIN_LOOP = 1000 */
    const float dt = (float)(1.0f / 500);
    f3 r_error = F3(d->sp_pos[0] - st_pos[0], d->sp_pos[1] - st_pos[1], d->sp_pos[2] - st_pos[2]);
    f3 v_error = F3(d->sp_vel[0] - st_vel[0], d->sp_vel[1] - st_vel[1], d->sp_vel[2] - st_vel[2]);
    d->i_err[2] += r_error.z * dt;
    d->i_err[2] = clampf_(d->i_err[2], -MEL_I_RANGE_Z, MEL_I_RANGE_Z);
    d->i_err[0] += r_error.x * dt;
    d->i_err[0] = clampf_(d->i_err[0], -MEL_I_RANGE_XY, MEL_I_RANGE_XY);
    d->i_err[1] += r_error.y * dt;
    d->i_err[1] = clampf_(d->i_err[1], -MEL_I_RANGE_XY, MEL_I_RANGE_XY);
    f3 target;
    float desired_yaw = 0;
    if (d->sp_mode != SP_UNSET) {
        target.x = MEL_MASS * d->sp_acc[0] + MEL_KP_XY * r_error.x + MEL_KD_XY * v_error.x + MEL_KI_XY * d->i_err[0];
        target.y = MEL_MASS * d->sp_acc[1] + MEL_KP_XY * r_error.y + MEL_KD_XY * v_error.y + MEL_KI_XY * d->i_err[1];
        target.z = MEL_MASS * (d->sp_acc[2] + GRAVITY_MAGNITUDE) + MEL_KP_Z * r_error.z + MEL_KD_Z * v_error.z +
                   MEL_KI_Z * d->i_err[2];
    } else {
        target.x = -sinf(radiansf_(0.0f));
        target.y = -sinf(radiansf_(0.0f));
        target.z = 1;
    }
    if (d->sp_mode == SP_COMMANDER) {
        desired_yaw = d->sp_yaw;
    } else if (d->sp_mode == SP_FULLSTATE) {
        /* quat2rpy(setpoint quaternion).z in degrees (the quaternion's x = y = 0) */
        float qx = 0.0f, qy = 0.0f, qz = d->sp_qz, qw = d->sp_qw;
        desired_yaw = degreesf_(atan2f(2.0f * (qw * qz + qx * qy), 1 - 2 * (qy * qy + qz * qz)));
    }
    /* state attitude quaternion -> rotation matrix (quat2rotmat) */
    float x = st_q[0], y = st_q[1], z = st_q[2], w = st_q[3];
    float R[3][3];
    R[0][0] = 1 - 2 * y * y - 2 * z * z; R[0][1] = 2 * x * y - 2 * z * w;     R[0][2] = 2 * x * z + 2 * y * w;
    R[1][0] = 2 * x * y + 2 * z * w;     R[1][1] = 1 - 2 * x * x - 2 * z * z; R[1][2] = 2 * y * z - 2 * x * w;
    R[2][0] = 2 * x * z - 2 * y * w;     R[2][1] = 2 * y * z + 2 * x * w;     R[2][2] = 1 - 2 * x * x - 2 * y * y;
    f3 Rx = F3(R[0][0], R[1][0], R[2][0]), Ry = F3(R[0][1], R[1][1], R[2][1]), Rz = F3(R[0][2], R[1][2], R[2][2]);
    float current_thrust = f3dot(target, Rz);
    f3 z_des = f3norm(target);
    f3 x_c = F3(cosf(radiansf_(desired_yaw)), sinf(radiansf_(desired_yaw)), 0);
    f3 y_des = f3norm(f3cross(z_des, x_c));
    f3 x_des = f3cross(y_des, z_des);
    /* eR = vee(Rdes^T R - R^T Rdes), pitch in the legacy (inverted) convention */
    f3 eR;
    eR.x = f3dot(z_des, Ry) - f3dot(Rz, y_des);
    eR.y = -(f3dot(x_des, Rz) - f3dot(Rx, z_des));
    eR.z = f3dot(y_des, Rx) - f3dot(Ry, x_des);
    /* ew: gyro in deg/s, pitch inverted; setpoint attitude rates in deg/s */
    float rate_roll = radiansf_(gyro[0]);
    float rate_pitch = -radiansf_(gyro[1]);
    float rate_yaw = radiansf_(gyro[2]);
    const float spr = d->sp_rate[0], spp = d->sp_rate[1], spy = d->sp_rate[2];
    f3 ew = F3(radiansf_(spr) - rate_roll, -radiansf_(spp) - rate_pitch, radiansf_(spy) - rate_yaw);
    float err_d_roll = 0, err_d_pitch = 0;
    if (d->prev_omega_roll == d->prev_omega_roll) {   /* d part initialised (not NaN) */
        err_d_roll = ((radiansf_(spr) - d->prev_sp_roll) - (rate_roll - d->prev_omega_roll)) / dt;
        err_d_pitch = (-(radiansf_(spp) - d->prev_sp_pitch) - (rate_pitch - d->prev_omega_pitch)) / dt;
    }
    d->prev_omega_roll = rate_roll;
    d->prev_omega_pitch = rate_pitch;
    d->prev_sp_roll = radiansf_(spr);
    d->prev_sp_pitch = radiansf_(spp);
    d->i_err_m[0] += (-eR.x) * dt;
    d->i_err_m[0] = clampf_(d->i_err_m[0], -MEL_I_RANGE_M_XY, MEL_I_RANGE_M_XY);
    d->i_err_m[1] += (-eR.y) * dt;
    d->i_err_m[1] = clampf_(d->i_err_m[1], -MEL_I_RANGE_M_XY, MEL_I_RANGE_M_XY);
    d->i_err_m[2] += (-eR.z) * dt;
    d->i_err_m[2] = clampf_(d->i_err_m[2], -MEL_I_RANGE_M_Z, MEL_I_RANGE_M_Z);
    f3 M;
    M.x = -MEL_KR_XY * eR.x + MEL_KW_XY * ew.x + MEL_KI_M_XY * d->i_err_m[0] + MEL_KD_OMEGA_RP * err_d_roll;
    M.y = -MEL_KR_XY * eR.y + MEL_KW_XY * ew.y + MEL_KI_M_XY * d->i_err_m[1] + MEL_KD_OMEGA_RP * err_d_pitch;
    M.z = -MEL_KR_Z * eR.z + MEL_KW_Z * ew.z + MEL_KI_M_Z * d->i_err_m[2];
    d->ctl[3] = MEL_MASS_THRUST * current_thrust;
    if (d->ctl[3] > 0) {   /* control_t roll/pitch/yaw are int16: C float->int truncation */
        const float mc[3] = {clampf_(M.x, -32000, 32000), clampf_(M.y, -32000, 32000), clampf_(-M.z, -32000, 32000)};
        for (int k = 0; k < 3; ++k) {
            const float a = fabsf(mc[k]);
            const float dist = a < 1.0f ? 1.0f - a : fabsf(a - rintf(a));
            if (dist < d->mom_margin) d->mom_margin = dist;
        }
        d->ctl[0] = (float)(int16_t)mc[0];
        d->ctl[1] = (float)(int16_t)mc[1];
        d->ctl[2] = (float)(int16_t)mc[2];
        if (d->rp_mom && d->rp_call < d->rp_n) {   /* replay: the kernel's integers for this call */
            const int16_t* m = d->rp_mom + 3 * d->rp_call;
            d->ctl[0] = (float)m[0];
            d->ctl[1] = (float)m[1];
            d->ctl[2] = (float)m[2];
        }
    } else {
        d->ctl[0] = d->ctl[1] = d->ctl[2] = 0;
        mellinger_reset(d);
    }
    d->rp_call += 1;
    d->mom_hash = fw_moment_hash(d->mom_hash, d->ctl[0], d->ctl[1], d->ctl[2]);
}

/* ---------------------------------------------------------------------------------- */
/* MellingerControl wrapper (float64), MellingerControl.py:99-262, 378-442             */
/* ---------------------------------------------------------------------------------- */
static void mellinger_wrapper_reset(rdrone_t* d, const double init_rpy[3], const double init_vel[3]) {
    for (int k = 0; k < 3; ++k) {
        d->prev_rpy[k] = init_rpy[k];
        d->prev_vel[k] = init_vel[k];
        d->lpf_d1[k] = d->lpf_d2[k] = 0;
    }
    d->tick = d->last_att_tick = d->last_pos_tick = d->tumble = 0;
    mellinger_reset(d);
    d->prev_omega_roll = d->prev_omega_pitch = NAN;   /* first call has no D term */
    d->prev_sp_roll = d->prev_sp_pitch = 0;
    d->ctl[0] = d->ctl[1] = d->ctl[2] = d->ctl[3] = 0;
}

/* ---------------------------------------------------------------------------------- */
/* Crazyflie high-level commander + planner: restated from the published   */
/* firmware algorithm (crtp_commander_high_level.c, planner.c, pptraj.c, math3d.h; C float). */
/* Not in /root/reference (pycffirmware is an un-vendored dependency): parity unpinned.      */
/* Call sites: low_level_control (MellingerControl.py:17-61), process_command_queue         */
/* (292-303), _update_setpoint (369-374), the send*Cmd / _send*Cmd pairs (491-699), reset's  */
/* crtpCommanderHighLevelInit + TellState (145-150).                                        */
/* ---------------------------------------------------------------------------------- */
enum { PLAN_IDLE = 0, PLAN_FLYING = 1, PLAN_LANDING = 2 };
#define HL_GRAV 9.81f                  /* pptraj.c GRAV */
#define HL_DEFAULT_VELOCITY 0.5f       /* defaultTakeoffVelocity / defaultLandingVelocity */

static f3 f3scl(float s, f3 v) { return F3(s * v.x, s * v.y, s * v.z); }
static f3 f3normr(f3 v) {   /* math3d vnormalize = vdiv(v, vmag(v)) = vscl(1 / |v|, v) */
    return f3scl(1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z), v);
}
static float shortest_signed_angle_radians(float start, float goal) {
    float diff = goal - start;
    float signed_diff = fmodf(diff + M_PI_F, 2 * M_PI_F) - M_PI_F;
    if (signed_diff < -M_PI_F) signed_diff += 2 * M_PI_F;
    return signed_diff;
}
/* poly7_nojerk: 7th-order polynomial with x, x', x'' given and x''' = 0 at both ends */
static void poly7_nojerk(float p[8], float T, float x0, float dx0, float ddx0, float xf, float dxf, float ddxf) {
    if (T <= 0.0f) {
        p[0] = xf; p[1] = dxf; p[2] = ddxf / 2;
        for (int i = 3; i < 8; ++i) p[i] = 0;
        return;
    }
    const float T2 = T * T, T3 = T2 * T, T4 = T3 * T, T5 = T4 * T, T6 = T5 * T, T7 = T6 * T;
    p[0] = x0; p[1] = dx0; p[2] = ddx0 / 2; p[3] = 0;
    p[4] = -(5 * (14 * x0 - 14 * xf + 8 * T * dx0 + 6 * T * dxf + 2 * T2 * ddx0 - T2 * ddxf)) / (2 * T4);
    p[5] = (84 * x0 - 84 * xf + 45 * T * dx0 + 39 * T * dxf + 10 * T2 * ddx0 - 7 * T2 * ddxf) / T5;
    p[6] = -(140 * x0 - 140 * xf + 72 * T * dx0 + 68 * T * dxf + 15 * T2 * ddx0 - 13 * T2 * ddxf) / (2 * T6);
    p[7] = (2 * (10 * x0 - 10 * xf + 5 * T * dx0 + 5 * T * dxf + T2 * ddx0 - T2 * ddxf)) / T7;
    (void)T3;
}
static float polyval7(const float p[8], float t) {   /* Horner from the top coefficient */
    float x = 0.0f;
    for (int i = 7; i >= 0; --i) x = x * t + p[i];
    return x;
}
static void polyder7(float p[8]) {
    for (int i = 1; i <= 7; ++i) p[i - 1] = i * p[i];
    p[7] = 0;
}
typedef struct { f3 pos, vel, acc, omega; float yaw; } traj_eval_t;
/* poly4d_eval: flat outputs -> pos, vel, acc, yaw and the body rates of the differential flatness map */
static traj_eval_t poly4d_eval(const float coef[4][8], float t) {
    float d[4][8];
    memcpy(d, coef, sizeof d);
    traj_eval_t o;
    o.pos = F3(polyval7(d[0], t), polyval7(d[1], t), polyval7(d[2], t));
    o.yaw = polyval7(d[3], t);
    for (int k = 0; k < 4; ++k) polyder7(d[k]);
    o.vel = F3(polyval7(d[0], t), polyval7(d[1], t), polyval7(d[2], t));
    const float dyaw = polyval7(d[3], t);
    for (int k = 0; k < 4; ++k) polyder7(d[k]);
    o.acc = F3(polyval7(d[0], t), polyval7(d[1], t), polyval7(d[2], t));
    for (int k = 0; k < 4; ++k) polyder7(d[k]);
    const f3 jerk = F3(polyval7(d[0], t), polyval7(d[1], t), polyval7(d[2], t));
    const f3 thrust = F3(o.acc.x + 0.0f, o.acc.y + 0.0f, o.acc.z + HL_GRAV);
    const f3 z_body = f3normr(thrust);
    const f3 x_world = F3(cosf(o.yaw), sinf(o.yaw), 0);
    const f3 y_body = f3normr(f3cross(z_body, x_world));
    const f3 x_body = f3cross(y_body, z_body);
    const float jz = f3dot(jerk, z_body);   /* vorthunit(jerk, z_body) */
    const f3 jerk_orth = F3(jerk.x - jz * z_body.x, jerk.y - jz * z_body.y, jerk.z - jz * z_body.z);
    const f3 h_w = f3scl(1.0f / sqrtf(f3dot(thrust, thrust)), jerk_orth);
    o.omega = F3(-f3dot(h_w, y_body), f3dot(h_w, x_body), z_body.z * dyaw);
    return o;
}
/* piecewise_eval of the planner's one-piece trajectory (timescale 1, shift 0); past its end the
   end point with zero derivatives.  Before t_begin the polynomial is extrapolated, as the firmware
   does (no clamp at t < t_begin). */
static traj_eval_t plan_eval(const rdrone_t* d, float t) {
    const float tr = t - d->plan_t0;
    if (tr <= d->plan_dur * 1.0f) return poly4d_eval(d->coef, tr);
    traj_eval_t ev = poly4d_eval(d->coef, d->plan_dur);
    ev.vel = ev.acc = ev.omega = F3(0, 0, 0);
    return ev;
}
/* piecewise_plan_7th_order_no_jerk into the planner, state -> FLYING / LANDING from t */
static void plan_7th(rdrone_t* d, int state, float t, float dur, f3 p0, float y0, f3 v0, float dy0, f3 a0,
                     f3 p1, float y1) {
    d->plan_dur = dur;
    poly7_nojerk(d->coef[0], dur, p0.x, v0.x, a0.x, p1.x, 0, 0);
    poly7_nojerk(d->coef[1], dur, p0.y, v0.y, a0.y, p1.y, 0, 0);
    poly7_nojerk(d->coef[2], dur, p0.z, v0.z, a0.z, p1.z, 0, 0);
    poly7_nojerk(d->coef[3], dur, y0, dy0, 0, y1, 0, 0);
    d->plan_state = state;
    d->plan_t0 = t;
}
static f3 cpos_(const rdrone_t* d) { return F3(d->c_pos[0], d->c_pos[1], d->c_pos[2]); }
/* plan_takeoff / plan_land (planner.c): takeoff only from IDLE, land not from IDLE / LANDING */
static void plan_takeoff(rdrone_t* d, float height, float hover_yaw, float dur, float t) {
    if (d->plan_state != PLAN_IDLE) return;
    const f3 p = cpos_(d), z = F3(0, 0, 0);
    plan_7th(d, PLAN_FLYING, t, dur, p, d->c_yaw, z, 0, z, F3(p.x, p.y, height), hover_yaw);
}
static void plan_land(rdrone_t* d, float height, float hover_yaw, float dur, float t) {
    if (d->plan_state == PLAN_IDLE || d->plan_state == PLAN_LANDING) return;
    const f3 p = cpos_(d), z = F3(0, 0, 0);
    plan_7th(d, PLAN_LANDING, t, dur, p, d->c_yaw, z, 0, z, F3(p.x, p.y, height), hover_yaw);
}
/* go_to from a stopped planner (the only case here: process_command_queue stops the planner
   before every command): plan_go_to_from the commander's last pos / vel / yaw, zero acc / rates */
static void plan_go_to(rdrone_t* d, f3 hover_pos, float hover_yaw, float dur, int relative, float t) {
    const f3 p0 = cpos_(d), v0 = F3(d->c_vel[0], d->c_vel[1], d->c_vel[2]), z = F3(0, 0, 0);
    const float y0 = d->c_yaw;
    if (relative) {
        hover_pos = F3(hover_pos.x + p0.x, hover_pos.y + p0.y, hover_pos.z + p0.z);
        hover_yaw += y0;
    }
    const float end_yaw = y0 + shortest_signed_angle_radians(y0, hover_yaw);
    plan_7th(d, PLAN_FLYING, t, dur, p0, y0, v0, 0, z, hover_pos, end_yaw);
}
/* crtpCommanderHighLevelTellState(state) */
static void hl_tell_state(rdrone_t* d) {
    for (int k = 0; k < 3; ++k) { d->c_pos[k] = d->st_pos[k]; d->c_vel[k] = d->st_vel[k]; }
    d->c_yaw = d->st_yaw * M_PI_F / 180.0f;
}
/* MellingerControl._update_setpoint (369-374) while full_state_cmd_override is off:
   TellState(state), UpdateTime(t), GetSetpoint(setpoint, state) */
static void hl_update_setpoint(rdrone_t* d, float t) {
    hl_tell_state(d);
    traj_eval_t ev;
    int valid = 0;
    if (d->plan_state != PLAN_IDLE) {   /* plan_current_goal */
        if (d->plan_state == PLAN_LANDING && t - d->plan_t0 >= d->plan_dur * 1.0f) d->plan_state = PLAN_IDLE;
        ev = plan_eval(d, t);
        valid = 1;
    }
    if (!valid || d->plan_state == PLAN_IDLE) {   /* plan_stop; plan_is_stopped: keep the setpoint */
        for (int k = 0; k < 3; ++k) { d->c_pos[k] = d->st_pos[k]; d->c_vel[k] = d->st_vel[k]; }
        d->c_yaw = radiansf_(d->st_yaw);
        return;
    }
    d->sp_pos[0] = ev.pos.x; d->sp_pos[1] = ev.pos.y; d->sp_pos[2] = ev.pos.z;
    d->sp_vel[0] = ev.vel.x; d->sp_vel[1] = ev.vel.y; d->sp_vel[2] = ev.vel.z;
    d->sp_acc[0] = ev.acc.x; d->sp_acc[1] = ev.acc.y; d->sp_acc[2] = ev.acc.z;
    d->sp_yaw = degreesf_(ev.yaw);
    d->sp_rate[0] = degreesf_(ev.omega.x); d->sp_rate[1] = degreesf_(ev.omega.y); d->sp_rate[2] = degreesf_(ev.omega.z);
    d->sp_mode = SP_COMMANDER;
    d->c_pos[0] = ev.pos.x; d->c_pos[1] = ev.pos.y; d->c_pos[2] = ev.pos.z;
    d->c_vel[0] = ev.vel.x; d->c_vel[1] = ev.vel.y; d->c_vel[2] = ev.vel.z;
    d->c_yaw = ev.yaw;
}
/* reset (MellingerControl.py:119-150): zeroed setpoint_t, override on, crtpCommanderHighLevelInit
   (planner IDLE), _update_state from the initial obs row, TellState */
static void hl_reset(rdrone_t* d, const double pos[3], const double rpy[3]) {
    for (int k = 0; k < 3; ++k) {
        d->sp_pos[k] = d->sp_vel[k] = d->sp_acc[k] = d->sp_rate[k] = 0;
        d->st_pos[k] = (float)pos[k];
        d->st_vel[k] = 0.0f;
    }
    d->sp_qz = d->sp_qw = d->sp_yaw = 0;
    d->st_yaw = (float)(rpy[2] * RAD_TO_DEG);
    d->plan_t0 = d->plan_dur = 0;
    memset(d->coef, 0, sizeof d->coef);
    d->plan_state = PLAN_IDLE;
    d->override = 1;
    d->sp_mode = SP_UNSET;
    hl_tell_state(d);
}
/* _sendFullStateCmd (510-543): float setpoint fields from the float64 arguments */
static void hl_fullstate(rdrone_t* d, const double pos[3], const double vel[3], const double acc[3], double yaw,
                         const double rate[3]) {
    double q[4], e3[3] = {0, 0, yaw};
    orc_quat_from_euler(e3, q);   /* get_quaternion_from_euler(0, 0, yaw) */
    for (int k = 0; k < 3; ++k) {
        d->sp_pos[k] = (float)pos[k];
        d->sp_vel[k] = (float)vel[k];
        d->sp_acc[k] = (float)acc[k];
        d->sp_rate[k] = (float)(rate[k] * RAD_TO_DEG);
    }
    d->sp_qz = (float)q[2];
    d->sp_qw = (float)q[3];
    d->sp_mode = SP_FULLSTATE;
    d->override = 1;
}
/* one command message: low_level_control (17-61) -> send*Cmd -> process_command_queue(args[-1])
   (292-303): crtpCommanderHighLevelStop, UpdateTime(args[-1]), then the queued _send*Cmd */
static void hl_command(rdrone_t* d, int code, const double* a, int obs_wrapper) {
    if (code <= ADRP_CMD_NONE || code > ADRP_CMD_NOTIFY) return;
    d->plan_state = PLAN_IDLE;
    const float t = (float)a[ADRP_CMD_TIME_SLOT];
    switch (code) {
        case ADRP_CMD_FULLSTATE:   /* DroneObservationWrapper zeroes the tuple's yaw (wrapper.py:56-57) */
            hl_fullstate(d, a, a + 3, a + 6, obs_wrapper ? 0.0 : a[9], a + 10);
            return;
        case ADRP_CMD_TAKEOFF:     /* takeoff2, useCurrentYaw */
            plan_takeoff(d, (float)a[0], d->c_yaw, (float)a[1], t);
            break;
        case ADRP_CMD_TAKEOFFYAW:
            plan_takeoff(d, (float)a[0], (float)a[2], (float)a[1], t);
            break;
        case ADRP_CMD_TAKEOFFVEL: {  /* takeoff_with_velocity */
            float h = (float)a[0];
            if (a[2] != 0) h += d->c_pos[2];
            const float v = (float)a[1] > 0 ? (float)a[1] : HL_DEFAULT_VELOCITY;
            plan_takeoff(d, h, d->c_yaw, fabsf(h - d->c_pos[2]) / v, t);
            break;
        }
        case ADRP_CMD_LAND:
            plan_land(d, (float)a[0], d->c_yaw, (float)a[1], t);
            break;
        case ADRP_CMD_LANDYAW:
            plan_land(d, (float)a[0], (float)a[2], (float)a[1], t);
            break;
        case ADRP_CMD_LANDVEL: {   /* land_with_velocity */
            float h = (float)a[0];
            if (a[2] != 0) h = d->c_pos[2] - h;
            const float v = (float)a[1] > 0 ? (float)a[1] : HL_DEFAULT_VELOCITY;
            plan_land(d, h, d->c_yaw, fabsf(h - d->c_pos[2]) / v, t);
            break;
        }
        case ADRP_CMD_STOP:
            break;
        case ADRP_CMD_GOTO:
            plan_go_to(d, F3((float)a[0], (float)a[1], (float)a[2]), (float)a[3], (float)a[4], a[5] != 0, t);
            break;
        case ADRP_CMD_NOTIFY:
            hl_tell_state(d);
            break;
    }
    d->override = 0;
}

/* computeControl(t, pos, rpy, vel, ang_vel, disturbance) -> rpm[4] */
static lpf_t g_gyro_lpf;   /* written once in orc_create, before any (threaded) step */
static void race_init_consts(void) { g_gyro_lpf = lpf_coeffs(FIRMWARE_FREQ, 30); }

static void mellinger_compute(rdrone_t* d, const double pos[3], const double rpy[3], const double vel[3],
                              const double noise[4], double rpm[4]) {
    const lpf_t gyro_lpf = g_gyro_lpf;   /* ACCEL_LPF_CUTOFF_FREQ (swapped); set by orc_create */
    double rates[3], acc[3];
    for (int k = 0; k < 3; ++k) {
        rates[k] = (rpy[k] - d->prev_rpy[k]) / FIRMWARE_DT;
        d->prev_rpy[k] = rpy[k];
        acc[k] = (vel[k] - d->prev_vel[k]) / FIRMWARE_DT / 9.8 + (k == 2 ? 1.0 : 0.0);
        d->prev_vel[k] = vel[k];
    }
    /* _update_state: quaternion from rpy (deg -> rad round trip), position, velocity, acc */
    double rpy_rt[3], qd[4];
    for (int k = 0; k < 3; ++k) rpy_rt[k] = (rpy[k] * RAD_TO_DEG) * DEG_TO_RAD;
    orc_quat_from_euler(rpy_rt, qd);
    float st_q[4] = {(float)qd[0], (float)qd[1], (float)qd[2], (float)qd[3]};
    float st_pos[3] = {(float)pos[0], (float)pos[1], (float)pos[2]};
    float st_vel[3] = {(float)vel[0], (float)vel[1], (float)vel[2]};
    float st_acc_z = (float)acc[2];
    /* _update_sensorData: gyro = lpf2p(rates in deg/s); the acc channel only feeds the
       firmware's log variable and is not modelled */
    for (int k = 0; k < 3; ++k) { d->st_pos[k] = st_pos[k]; d->st_vel[k] = st_vel[k]; }
    d->st_yaw = (float)(rpy[2] * RAD_TO_DEG);   /* state.attitude.yaw [deg] */
    float gyro[3];
    for (int k = 0; k < 3; ++k) gyro[k] = lpf_apply(&gyro_lpf, &d->lpf_d1[k], &d->lpf_d2[k], (float)(rates[k] * RAD_TO_DEG));
    /* _update_setpoint(self.tick / FIRMWARE_FREQ) (369-374) */
    if (!d->override) hl_update_setpoint(d, (float)(d->tick / (double)FIRMWARE_FREQ));
    /* _step_controller */
    double pwm[4];
    if (st_acc_z < -0.5f) d->tumble += 1; else d->tumble = 0;
    if (d->tumble >= 30) {
        d->tick += 1;
        pwm[0] = pwm[1] = pwm[2] = pwm[3] = 0;
    } else {
        double cur = d->tick / (double)FIRMWARE_FREQ;
        double last_att = d->last_att_tick / (double)FIRMWARE_FREQ, last_pos = d->last_pos_tick / (double)FIRMWARE_FREQ;
        int t;
        if ((cur - last_att > 0.002) && (cur - last_pos > 0.01)) {
            t = 0; d->last_pos_tick = d->tick; d->last_att_tick = d->tick;
        } else if (cur - last_att > 0.002) {
            d->last_att_tick = d->tick; t = 2;
        } else {
            t = 1;
        }
        mellinger_fw(d, gyro, st_pos, st_vel, st_q, t);
        d->tick += 1;
        double c[4] = {d->ctl[0], d->ctl[1], d->ctl[2], d->ctl[3]};
        orc_compute_pwms(c, pwm);
    }
    orc_pwms_to_rpms(pwm, noise, rpm);
}

/* ---------------------------------------------------------------------------------- */
/* geometry: URDF collision shapes, GJK distance, ray vs cylinder                       */
/* ---------------------------------------------------------------------------------- */
enum { SH_BOX = 0, SH_CYL = 1 };
typedef struct { int type; v3 c; m33 R; v3 h; double r; } shape_t;   /* CYL: radius r, half height h.z, axis R[:,2] */

static m33 m_mul(m33 a, m33 b) {
    m33 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return r;
}
static m33 rot_z(double a) {
    m33 r = {{{cos(a), -sin(a), 0}, {sin(a), cos(a), 0}, {0, 0, 1}}};
    return r;
}
static m33 rot_y(double a) {
    m33 r = {{{cos(a), 0, sin(a)}, {0, 1, 0}, {-sin(a), 0, cos(a)}}};
    return r;
}
static m33 m_eye(void) { m33 r = {{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}}; return r; }

static v3 support(const shape_t* s, v3 d) {
    v3 dl = mtv(s->R, d), pl;
    if (s->type == SH_BOX) {
        pl = V(dl.x >= 0 ? s->h.x : -s->h.x, dl.y >= 0 ? s->h.y : -s->h.y, dl.z >= 0 ? s->h.z : -s->h.z);
    } else {
        double n = sqrt(dl.x * dl.x + dl.y * dl.y);
        pl = n > 1e-300 ? V(s->r * dl.x / n, s->r * dl.y / n, 0) : V(0, 0, 0);
        pl.z = dl.z >= 0 ? s->h.z : -s->h.z;
    }
    return vadd(s->c, mv(s->R, pl));
}

/* closest point to the origin on conv(W[0..n-1]); reduces W to the supporting subset.
   Returns 1 if the origin is inside a tetrahedron. */
static int simplex_closest(v3* W, int* n, v3* out) {
    if (*n == 1) { *out = W[0]; return 0; }
    if (*n == 2) {
        v3 a = W[0], b = W[1], ab = vsub(b, a);
        double t = -vdot(a, ab) / vdot(ab, ab);
        if (t <= 0) { *n = 1; *out = a; return 0; }
        if (t >= 1) { W[0] = b; *n = 1; *out = b; return 0; }
        *out = vadd(a, vscale(ab, t));
        return 0;
    }
    if (*n == 3) {   /* Ericson, Real-Time Collision Detection 5.1.5, p = origin */
        v3 a = W[0], b = W[1], c = W[2];
        v3 ab = vsub(b, a), ac = vsub(c, a), ap = vscale(a, -1);
        double d1 = vdot(ab, ap), d2 = vdot(ac, ap);
        if (d1 <= 0 && d2 <= 0) { *n = 1; *out = a; return 0; }
        v3 bp = vscale(b, -1);
        double d3 = vdot(ab, bp), d4 = vdot(ac, bp);
        if (d3 >= 0 && d4 <= d3) { W[0] = b; *n = 1; *out = b; return 0; }
        double vc = d1 * d4 - d3 * d2;
        if (vc <= 0 && d1 >= 0 && d3 <= 0) {
            double v = d1 / (d1 - d3);
            *n = 2; *out = vadd(a, vscale(ab, v)); return 0;
        }
        v3 cp = vscale(c, -1);
        double d5 = vdot(ab, cp), d6 = vdot(ac, cp);
        if (d6 >= 0 && d5 <= d6) { W[0] = c; *n = 1; *out = c; return 0; }
        double vb = d5 * d2 - d1 * d6;
        if (vb <= 0 && d2 >= 0 && d6 <= 0) {
            double w = d2 / (d2 - d6);
            W[1] = c; *n = 2; *out = vadd(a, vscale(ac, w)); return 0;
        }
        double va = d3 * d6 - d5 * d4;
        if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
            double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
            W[0] = b; W[1] = c; *n = 2; *out = vadd(b, vscale(vsub(c, b), w)); return 0;
        }
        double den = 1.0 / (va + vb + vc);
        double v = vb * den, w = vc * den;
        *out = vadd(a, vadd(vscale(ab, v), vscale(ac, w)));
        return 0;
    }
    /* tetrahedron: origin inside?  else the closest of the faces that see the origin.  A
       degenerate (flat) tetrahedron -- e.g. two level discs at the same height -- encloses
       nothing: then every face is a candidate. */
    v3 a = W[0], b = W[1], c = W[2], d = W[3];
    v3 faces[4][3] = {{a, b, c}, {a, c, d}, {a, d, b}, {b, d, c}};
    v3 opp[4] = {d, b, c, a};
    double vol = vdot(vsub(b, a), vcross(vsub(c, a), vsub(d, a)));
    double scale = vnorm(vsub(b, a)) * vnorm(vsub(c, a)) * vnorm(vsub(d, a));
    int flat = fabs(vol) <= 1e-12 * scale;
    double best = INFINITY;
    v3 bestW[3], bestv = V(0, 0, 0);
    int bestn = 0, outside = 0;
    for (int f = 0; f < 4; ++f) {
        v3 p0 = faces[f][0], p1 = faces[f][1], p2 = faces[f][2];
        v3 nrm = vcross(vsub(p1, p0), vsub(p2, p0));
        double so = -vdot(nrm, p0), sd = vdot(nrm, vsub(opp[f], p0));
        if (flat || so * sd < 0) {   /* origin and the opposite vertex on different sides */
            outside = 1;
            v3 Wf[3] = {p0, p1, p2};
            int nf = 3;
            v3 vf;
            simplex_closest(Wf, &nf, &vf);
            double dd = vdot(vf, vf);
            if (dd < best) { best = dd; bestv = vf; bestn = nf; memcpy(bestW, Wf, sizeof Wf); }
        }
    }
    if (!outside) return 1;
    memcpy(W, bestW, sizeof(v3) * bestn);
    *n = bestn;
    *out = bestv;
    return 0;
}

/* Euclidean distance between two convex shapes (0 when they overlap). */
static double gjk_distance(const shape_t* A, const shape_t* B) {
    v3 W[4];
    int n = 0;
    v3 v = vsub(A->c, B->c);
    if (vdot(v, v) < 1e-24) v = V(1, 0, 0);
    for (int it = 0; it < 96; ++it) {
        v3 w = vsub(support(A, vscale(v, -1)), support(B, v));
        double vv = vdot(v, v);
        if (vv - vdot(v, w) <= 1e-13 * vv + 1e-30) break;      /* converged */
        int dup = 0;
        for (int k = 0; k < n; ++k)
            if (vdot(vsub(W[k], w), vsub(W[k], w)) < 1e-26) dup = 1;
        if (dup) break;
        W[n++] = w;
        if (simplex_closest(W, &n, &v)) return 0;
        if (vdot(v, v) < 1e-24) return 0;
    }
    return vnorm(v);
}

/* Part lists in the body's own frame (URDF <collision> origins / rpy / sizes). */
typedef struct { int type; v3 off; m33 R; v3 h; double r; } part_t;
static int gate_parts(int low, part_t* p) {   /* portal.urdf (tall, type 0) / low_portal.urdf (type 1) */
    m33 I = m_eye(), Ry = rot_y(1.57);
    part_t bar = {SH_BOX, V(0, 0, -0.225), I, V(0.25, 0.025, 0.025), 0};
    p[0] = bar;                                  /* grey_edge */
    p[1] = bar; p[1].off = V(0, 0, 0.225);       /* blue_edge */
    p[2] = bar; p[2].off = V(0.225, 0, 0); p[2].R = Ry;    /* green_edge, rpy (0, 1.57, 0) */
    p[3] = bar; p[3].off = V(-0.225, 0, 0); p[3].R = Ry;   /* red_edge */
    if (low) { part_t bx = {SH_BOX, V(0, 0, -0.4), I, V(0.075, 0.075, 0.125), 0}; p[4] = bx; }
    else { part_t cy = {SH_CYL, V(0, 0, -0.6), I, V(0, 0, 0.4), 0.05}; p[4] = cy; }
    return 5;
}
static int obstacle_parts(part_t* p) {   /* obstacle.urdf */
    m33 I = m_eye();
    part_t cy = {SH_CYL, V(0, 0, 0), I, V(0, 0, 0.4), 0.05};
    part_t bx = {SH_BOX, V(0, 0, -0.4), I, V(0.075, 0.075, 0.125), 0};
    p[0] = cy; p[1] = bx;
    return 2;
}
static shape_t place(const part_t* p, v3 origin, m33 Rb) {
    shape_t s = {p->type, vadd(origin, mv(Rb, p->off)), m_mul(Rb, p->R), p->h, p->r};
    return s;
}
static shape_t drone_shape(const orc_t* o, const body_t* b) {   /* cf2x_IROS.urdf:32-37 */
    m33 R = mat_from_quat(qconj(b->q_wtb));
    shape_t s = {SH_CYL, vadd(b->pos, mv(R, V(0, 0, o->cfg.drone.collision_z_offset))), R,
                 V(0, 0, 0.5 * o->cfg.drone.collision_h), o->cfg.drone.collision_r};
    return s;
}
/* minimum distance drone <-> one gate / obstacle body */
static double body_distance(const shape_t* drone, const part_t* parts, int np, v3 origin, m33 Rb) {
    double best = INFINITY;
    for (int k = 0; k < np; ++k) {
        shape_t s = place(&parts[k], origin, Rb);
        double dd = gjk_distance(drone, &s);
        if (dd < best) best = dd;
    }
    return best;
}
/* entry fraction of segment p0->p1 into a cylinder (or > 1 if it misses) */
static double ray_cylinder(const shape_t* s, v3 p0, v3 p1) {
    v3 a = mtv(s->R, vsub(p0, s->c)), d = mtv(s->R, vsub(p1, p0));
    double lo = -INFINITY, hi = INFINITY;
    if (fabs(d.z) < 1e-300) {
        if (fabs(a.z) > s->h.z) return 2;
    } else {
        double t1 = (-s->h.z - a.z) / d.z, t2 = (s->h.z - a.z) / d.z;
        if (t1 > t2) { double t = t1; t1 = t2; t2 = t; }
        lo = t1; hi = t2;
    }
    double qa = d.x * d.x + d.y * d.y, qb = 2 * (a.x * d.x + a.y * d.y), qc = a.x * a.x + a.y * a.y - s->r * s->r;
    if (qa < 1e-300) {
        if (qc > 0) return 2;
    } else {
        double disc = qb * qb - 4 * qa * qc;
        if (disc < 0) return 2;
        double sq = sqrt(disc), t3 = (-qb - sq) / (2 * qa), t4 = (-qb + sq) / (2 * qa);
        if (t3 > lo) lo = t3;
        if (t4 < hi) hi = t4;
    }
    if (lo > hi || hi < 0 || lo > 1) return 2;
    return lo < 0 ? 0 : lo;
}

/* ---------------------------------------------------------------------------------- */
/* race env                                                                             */
/* ---------------------------------------------------------------------------------- */
static int race_obs_dim(const adrp_config* c) {
    return 49 + (c->race_mode == ADRP_RACE_COMPETE ? 6 * (c->num_drones - 1) : 0);
}

static int race_alloc(orc_t* o) {
    o->rd = (rdrone_t*)calloc((size_t)o->E * o->N, sizeof(rdrone_t));
    o->re = (renv_t*)calloc((size_t)o->E, sizeof(renv_t));
    return ADRP_OK;
}

/* Box-Muller of one Philox pair from IEEE float operations only (+ - * /, sqrtf, fmaf, frexpf, rintf;
   C float arithmetic, no contraction), so the fp64 kernels (adrp_device.h normal_pair_f, the same
   sequence) draw bit-identical action noise: u1 = (x0 >> 8 + 1) 2^-24 in (0, 1], u2 = (x1 >> 8) 2^-24
   in [0, 1); r = sqrt(-2 log u1) with log u1 = e ln2 + 2 atanh(s), s = (m - 1) / (m + 1),
   m in [sqrt(1/2), sqrt(2)); (sin, cos)(2 pi u2) from the octant n = rint(8 u2) and the Taylor pair
   on |x| = |2 pi (u2 - n / 8)| <= pi / 8.  Accuracy ~2 float ulp: the samples are float, scaled by the
   noise std in double. */
static void normal_pair_f(uint32_t x0, uint32_t x1, float* z0, float* z1) {
    const float u1 = ((float)(x0 >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = (float)(x1 >> 8) * (1.0f / 16777216.0f);
    int e;
    float m = frexpf(u1, &e);                       /* u1 = m 2^e, m in [0.5, 1) */
    if (m < 0.70710677f) { m = m * 2.0f; e -= 1; }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float z = s * s;
    float p = 1.0f / 11;
    p = fmaf(p, z, 1.0f / 9); p = fmaf(p, z, 1.0f / 7); p = fmaf(p, z, 1.0f / 5); p = fmaf(p, z, 1.0f / 3);
    const float lm = fmaf(2.0f * s * z, p, 2.0f * s);  /* log m = 2 s (1 + z/3 + ... + z^5/11) */
    const float fe = (float)e;
    const float lg = fmaf(fe, 0.693145751953125f, fmaf(fe, 1.428606765330187e-06f, lm));
    const float r = sqrtf(-2.0f * lg);
    const float n = rintf(u2 * 8.0f);
    const float x = (u2 - n * 0.125f) * 6.28318548f;
    const float x2 = x * x;
    float ps = -1.98412698e-4f;
    ps = fmaf(ps, x2, 8.33333377e-3f); ps = fmaf(ps, x2, -0.166666672f);
    float pc = 2.48015876e-5f;
    pc = fmaf(pc, x2, -1.38888892e-3f); pc = fmaf(pc, x2, 4.16666679e-2f); pc = fmaf(pc, x2, -0.5f);
    const float sx = fmaf(x * x2, ps, x), cx = fmaf(x2, pc, 1.0f);
    const float h = 0.70710677f;
    const float a = h * (cx + sx), b = h * (cx - sx);
    float sn, cs;
    switch ((int)n & 7) {
        case 0: sn = sx; cs = cx; break;
        case 1: sn = a; cs = b; break;
        case 2: sn = cx; cs = -sx; break;
        case 3: sn = b; cs = -a; break;
        case 4: sn = -sx; cs = -cx; break;
        case 5: sn = -a; cs = -b; break;
        case 6: sn = -cx; cs = sx; break;
        default: sn = -b; cs = a; break;
    }
    *z0 = r * cs;
    *z1 = r * sn;
}

static void draw_normal4(uint64_t seed, uint64_t gid, uint32_t ep, uint32_t tag, uint32_t idx, double z[4]) {
    uint32_t cc[4] = {(uint32_t)gid, ep, tag, idx}, k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, x[4];
    orc_philox4x32_10(cc, k, x);
    float f[4];
    normal_pair_f(x[0], x[1], &f[0], &f[1]);
    normal_pair_f(x[2], x[3], &f[2], &f[3]);
    for (int j = 0; j < 4; ++j) z[j] = f[j];
}

int orc_normal_pair(uint32_t x0, uint32_t x1, float* z) {   /* (tests: accuracy, GPU bit-identity) */
    normal_pair_f(x0, x1, &z[0], &z[1]);
    return 0;
}

static v3 body_ang_v(const orc_t* o, const body_t* b) {   /* getBaseVelocity angular part */
    return o->cfg.physics == ADRP_PHYS_DYN ? b->ang_v : b->omega;
}

static void gate_pose(const renv_t* re, int g, v3* origin, m33* R) {
    *origin = V(re->gate[g][0], re->gate[g][1], re->gate[g][2]);
    *R = rot_z(re->gate[g][3]);   /* loadURDF(..., getQuaternionFromEuler([0, 0, yaw])) */
}

/* _computeObs assembly (MultiRaceAviary.py:597-661) for drone i from the drones' kinematic
   rows kin[k] = [pos, rpy, vel, ang_v], the actual gate (x,y,z,yaw) / obstacle (x,y,z) poses
   and the getClosestPoints(..., VISIBILITY_RANGE) outcomes */
static void race_obs_assemble(const adrp_config* c, int N, int i, const double (*kin)[12], const double gate_act[][4],
                              const uint8_t* gate_in, const double obst_act[][3], const uint8_t* obst_in,
                              int current_gate, double* row) {
    const adrp_track* t = &c->track;
    memset(row, 0, sizeof(double) * race_obs_dim(c));
    memcpy(row, kin[i], sizeof(double) * 12);
    for (int g = 0; g < t->num_gates; ++g) {
        if (gate_in[g]) { for (int j = 0; j < 4; ++j) row[12 + 4 * g + j] = gate_act[g][j]; }
        else { row[12 + 4 * g] = t->gates[g][0]; row[13 + 4 * g] = t->gates[g][1]; row[14 + 4 * g] = t->gates[g][2]; row[15 + 4 * g] = t->gates[g][5]; }
        row[28 + g] = gate_in[g] ? 1 : 0;
    }
    for (int k = 0; k < t->num_obstacles; ++k) {
        for (int j = 0; j < 3; ++j) row[32 + 3 * k + j] = obst_in[k] ? obst_act[k][j] : t->obstacles[k][j];
        row[44 + k] = obst_in[k] ? 1 : 0;
    }
    row[48] = current_gate;
    if (c->race_mode == ADRP_RACE_COMPETE) {
        int idx = 0;
        for (int k = 0; k < N; ++k) {
            if (k == i) continue;
            double* p = row + 49 + 6 * idx;
            for (int j = 0; j < 6; ++j) p[j] = kin[k][j];
            ++idx;
        }
    }
}

static void race_kin_row(const orc_t* o, const body_t* b, double* k12) {
    double rpy[3];
    body_rpy(b, rpy);
    v3 w = body_ang_v(o, b);
    double v[12] = {b->pos.x, b->pos.y, b->pos.z, rpy[0], rpy[1], rpy[2], b->vel.x, b->vel.y, b->vel.z, w.x, w.y, w.z};
    memcpy(k12, v, sizeof v);
}

/* _computeObs (MultiRaceAviary.py:566-661) of drone i in env e, float64 row */
static void race_obs_row(const orc_t* o, int e, int i, double* row) {
    const adrp_config* c = &o->cfg;
    const adrp_track* t = &c->track;
    const int N = o->N;
    const body_t* bs = &o->b[(size_t)e * N];
    const renv_t* re = &o->re[e];
    double kin[ADRP_MAX_DRONES][12];
    for (int k = 0; k < N; ++k) race_kin_row(o, &bs[k], kin[k]);
    shape_t ds = drone_shape(o, &bs[i]);
    part_t parts[5];
    uint8_t gin[ADRP_MAX_GATES] = {0}, oin[ADRP_MAX_OBSTACLES] = {0};
    for (int g = 0; g < t->num_gates; ++g) {
        v3 org; m33 Rg;
        gate_pose(re, g, &org, &Rg);
        int np = gate_parts(t->gates[g][6] > 0, parts);
        gin[g] = body_distance(&ds, parts, np, org, Rg) < VISIBILITY_RANGE;
    }
    for (int k = 0; k < t->num_obstacles; ++k) {
        int np = obstacle_parts(parts);
        oin[k] = body_distance(&ds, parts, np, V(re->obst[k][0], re->obst[k][1], re->obst[k][2]), m_eye()) < VISIBILITY_RANGE;
    }
    race_obs_assemble(c, N, i, (const double(*)[12])kin, (const double(*)[4])re->gate, gin,
                      (const double(*)[3])re->obst, oin, o->rd[(size_t)e * N + i].gate, row);
}

static void race_write_obs(const orc_t* o, int e, float* obs_env, double* row0) {
    double row[64 + 6 * ADRP_MAX_DRONES];
    for (int i = 0; i < o->N; ++i) {
        race_obs_row(o, e, i, row);
        for (int k = 0; k < o->D; ++k) obs_env[(size_t)i * o->D + k] = (float)row[k];
        if (i == 0 && row0) memcpy(row0, row, sizeof(double) * o->D);
    }
}

/* MultiRaceAviary.reset (127-167): BaseAviary.reset loads the drones at the nominal
   init_states (pos, rpy*DEG_TO_RAD), computes the initial obs there and resets the
   controllers with it; _drone_init then moves the drones to the randomised pose. */
static void race_reset_env(orc_t* o, int e, float* obs_env) {
    const adrp_config* c = &o->cfg;
    const adrp_track* t = &c->track;
    const int N = o->N;
    const uint64_t gid = (uint64_t)(c->env_offset + e);
    const uint32_t ep = (uint32_t)o->episode[e];
    renv_t* re = &o->re[e];
    double u[4];
    for (int g = 0; g < ADRP_MAX_GATES; ++g) {
        re->gate[g][0] = t->gates[g][0]; re->gate[g][1] = t->gates[g][1];
        re->gate[g][2] = t->gates[g][2]; re->gate[g][3] = t->gates[g][5];
        if (t->random_gates_obstacles && g < t->num_gates) {   /* _addObstacles (359-369) */
            const double lo = t->gate_offset_range[0], hi = t->gate_offset_range[1];
            draw4(c->seed, gid, ep, TAG_RACE_TRACK, (uint32_t)g, u);
            re->gate[g][0] += lo + (hi - lo) * u[0];
            re->gate[g][1] += lo + (hi - lo) * u[1];
            re->gate[g][3] += lo + (hi - lo) * u[2];
        }
    }
    for (int k = 0; k < ADRP_MAX_OBSTACLES; ++k) {
        for (int j = 0; j < 3; ++j) re->obst[k][j] = t->obstacles[k][j];
        if (t->random_gates_obstacles && k < t->num_obstacles) {   /* (371-380) */
            const double lo = t->obstacle_offset_range[0], hi = t->obstacle_offset_range[1];
            draw4(c->seed, gid, ep, TAG_RACE_TRACK, (uint32_t)(4 + k), u);
            re->obst[k][0] += lo + (hi - lo) * u[0];
            re->obst[k][1] += lo + (hi - lo) * u[1];
        }
    }
    /* nominal pose, at rest (loadURDF in _housekeeping) */
    for (int i = 0; i < N; ++i) {
        body_t* b = &o->b[(size_t)e * N + i];
        rdrone_t* d = &o->rd[(size_t)e * N + i];
        double rpy[3], q[4];
        for (int k = 0; k < 3; ++k) rpy[k] = t->init_rpy[i][k] * DEG_TO_RAD;
        orc_quat_from_euler(rpy, q);
        memset(b, 0, sizeof *b);
        b->pos = V(t->init_pos[i][0], t->init_pos[i][1], t->init_pos[i][2]);
        qt qq = {q[0], q[1], q[2], q[3]};
        b->q_wtb = qconj(qq);
        forward_kinematics(b);
        d->gate = 0; d->elim = 0; d->fin = 0;
    }
    double row0[64 + 6 * ADRP_MAX_DRONES];
    float tmp[ADRP_MAX_DRONES * (64 + 6 * ADRP_MAX_DRONES)];
    race_write_obs(o, e, obs_env ? obs_env : tmp, row0);
    /* controllers reset with the initial obs; _drone_init moves the drones */
    for (int i = 0; i < N; ++i) {
        body_t* b = &o->b[(size_t)e * N + i];
        rdrone_t* d = &o->rd[(size_t)e * N + i];
        double nom_rpy[3], zero[3] = {0, 0, 0};
        body_rpy(b, nom_rpy);
        mellinger_wrapper_reset(d, nom_rpy, zero);
        const double nom_pos[3] = {b->pos.x, b->pos.y, b->pos.z};
        hl_reset(d, nom_pos, nom_rpy);
        d->kin_pos = b->pos;                 /* self.pos still holds the nominal pose */
        d->mass = t->race_mass;
        d->inertia = V(t->race_inertia[0], t->race_inertia[1], t->race_inertia[2]);
        if (t->random_drone_inertia) {       /* _drone_init (419-424), clipped to [0, 100] */
            draw4(c->seed, gid, ep, TAG_RACE_DRONE | (uint32_t)i, 2, u);
            double v[4] = {d->mass, d->inertia.x, d->inertia.y, d->inertia.z};
            for (int k = 0; k < 4; ++k) {
                const double lo = t->inertia_offset_range[k][0], hi = t->inertia_offset_range[k][1];
                v[k] = clampd(v[k] + lo + (hi - lo) * u[k], 0, 100);
            }
            d->mass = v[0]; d->inertia = V(v[1], v[2], v[3]);
        }
        double po[3] = {0, 0, 0}, ro[3] = {0, 0, 0};
        if (t->random_drone_state) {         /* (434-450) */
            double u2[4];
            draw4(c->seed, gid, ep, TAG_RACE_DRONE | (uint32_t)i, 0, u);
            draw4(c->seed, gid, ep, TAG_RACE_DRONE | (uint32_t)i, 1, u2);
            for (int k = 0; k < 3; ++k) {
                po[k] = t->pos_offset_range[k][0] + (t->pos_offset_range[k][1] - t->pos_offset_range[k][0]) * u[k];
                ro[k] = t->rot_offset_range[k][0] + (t->rot_offset_range[k][1] - t->rot_offset_range[k][0]) * u2[k];
            }
        }
        double rpy[3], q[4];
        for (int k = 0; k < 3; ++k) rpy[k] = t->init_rpy[i][k] + ro[k];   /* raw config rpy (Q26) */
        orc_quat_from_euler(rpy, q);
        b->pos = V(t->init_pos[i][0] + po[0], t->init_pos[i][1] + po[1], t->init_pos[i][2] + po[2]);
        qt qq = {q[0], q[1], q[2], q[3]};
        b->q_wtb = qconj(qq);
        b->vel = V(t->init_vel[i][0], t->init_vel[i][1], t->init_vel[i][2]);
        b->omega = V(t->init_pqr[i][0], t->init_pqr[i][1], t->init_pqr[i][2]);
        b->ang_v = b->omega;
        b->rpy_rates = V(0, 0, 0);
        forward_kinematics(b);               /* resetBasePositionAndOrientation */
        for (int k = 0; k < 4; ++k) d->rpm[k] = d->prev_rpm[k] = 0;
        if (c->physics != ADRP_PHYS_PYB) d->kin_pos = b->pos;   /* refreshed before the first _apply_physics */
    }
    re->wr_gate = (int)row0[48];             /* RewardWrapper.reset (wrapper.py:98-101) */
    for (int k = 0; k < 3; ++k) { re->wr_target[k] = row0[12 + k]; re->wr_prev[k] = row0[k]; }
    o->step_counter[e] = 0;
    o->episode[e] += 1;
}

static int race_contact(const orc_t* o, int e, int i) {   /* _collision (552-562) */
    const adrp_config* c = &o->cfg;
    const adrp_track* t = &c->track;
    const int N = o->N;
    const body_t* bs = &o->b[(size_t)e * N];
    const renv_t* re = &o->re[e];
    const body_t* b = &bs[i];
    shape_t ds = drone_shape(o, b);
    part_t parts[5];
    for (int g = 0; g < t->num_gates; ++g) {
        v3 org; m33 Rg;
        gate_pose(re, g, &org, &Rg);
        if (body_distance(&ds, parts, gate_parts(t->gates[g][6] > 0, parts), org, Rg) < 1e-6) return 1;
    }
    for (int k = 0; k < t->num_obstacles; ++k)
        if (body_distance(&ds, parts, obstacle_parts(parts), V(re->obst[k][0], re->obst[k][1], re->obst[k][2]), m_eye()) < 1e-6)
            return 1;
    m33 R = ds.R;   /* plane z = 0: lowest point of the collision cylinder */
    double low = ds.c.z - ds.h.z * fabs(R.m[2][2]) - ds.r * sqrt(R.m[0][2] * R.m[0][2] + R.m[1][2] * R.m[1][2]);
    if (low <= 1e-6) return 1;
    if (c->race_mode == ADRP_RACE_COMPETE)
        for (int k = 0; k < N; ++k) {
            if (k == i) continue;
            shape_t dk = drone_shape(o, &bs[k]);
            if (gjk_distance(&ds, &dk) < 1e-6) return 1;
        }
    return 0;
}

/* the 7 vertical rays of _gate_progress (MultiRaceAviary.py:484-494), reference order:
   centre, then +-i * 0.05 (cos yaw, sin yaw) for i = 1, 2, 3 */
static void race_rays(const double gate_xyyaw[3], int type, double from[7][3], double to[7][3]) {
    const double x = gate_xyyaw[0], y = gate_xyyaw[1], rot = gate_xyyaw[2];
    const double h = type == 0 ? 1.0 : 0.525, half = 0.1875;   /* Z_HIGH / Z_LOW (URDF dependent) */
    const double dx = 0.05 * cos(rot), dy = 0.05 * sin(rot);
    for (int r = 0; r < 7; ++r) {
        const int m = r == 0 ? 0 : ((r + 1) / 2) * (r % 2 ? 1 : -1);
        from[r][0] = to[r][0] = x + m * dx;
        from[r][1] = to[r][1] = y + m * dy;
        from[r][2] = h - half;
        to[r][2] = h + half;
    }
}
/* decision part of _gate_progress (502-506): rays' first-hit ids and fractions */
static void race_progress_decide(int num_gates, int self_id, const int hit_id[7], const double hit_frac[7],
                                 int* gate, int* fin) {
    const int g = *gate;
    if (num_gates > 0 && g < num_gates) {
        int passed = 0;
        for (int r = 0; r < 7; ++r) passed |= (hit_frac[r] < 0.9999 && hit_id[r] == self_id);
        if (passed) *gate = g + 1;
    }
    if (g >= num_gates) *fin = 1;
}

/* _gate_progress (471-506) for drone i */
static void race_gate_progress(orc_t* o, int e, int i) {
    const adrp_track* t = &o->cfg.track;
    const int N = o->N;
    rdrone_t* d = &o->rd[(size_t)e * N + i];
    const renv_t* re = &o->re[e];
    int hit_id[7] = {-1, -1, -1, -1, -1, -1, -1};
    double hit_frac[7] = {1, 1, 1, 1, 1, 1, 1};
    if (t->num_gates > 0 && d->gate < t->num_gates) {
        double from[7][3], to[7][3], g3[3] = {re->gate[d->gate][0], re->gate[d->gate][1], re->gate[d->gate][3]};
        race_rays(g3, t->gates[d->gate][6] > 0, from, to);
        for (int r = 0; r < 7; ++r) {
            for (int k = 0; k < N; ++k) {   /* first hit among the drones (gates/obstacles lie off the rays) */
                shape_t sk = drone_shape(o, &o->b[(size_t)e * N + k]);
                double f = ray_cylinder(&sk, V(from[r][0], from[r][1], from[r][2]), V(to[r][0], to[r][1], to[r][2]));
                if (f < hit_frac[r] && f <= 1) { hit_frac[r] = f; hit_id[r] = k; }
            }
        }
    }
    race_progress_decide(t->num_gates, i, hit_id, hit_frac, &d->gate, &d->fin);
}

/* _computeTerminated (674-698): updates elim[], returns terminated */
static int race_terminated(const adrp_track* t, int N, const double (*pos)[3], const double (*angv)[3],
                           const uint8_t* contact, uint8_t* elim, const uint8_t* fin) {
    int all_done = 1;
    for (int i = 0; i < N; ++i) {
        int oob = fabs(pos[i][0]) > t->bounds_hi[0] || fabs(pos[i][1]) > t->bounds_hi[1] || fabs(pos[i][2]) > t->bounds_hi[2];
        int unstable = fabs(angv[i][0]) > 20 || fabs(angv[i][1]) > 20 || fabs(angv[i][2]) > 20;
        elim[i] = (uint8_t)(elim[i] || oob || unstable || contact[i]);
        all_done &= (elim[i] || fin[i]);
    }
    return all_done;
}
/* _computeTruncated (702-709), evaluated before step_counter += S */
static int race_truncated(const adrp_config* c, int step_counter) {
    return (double)step_counter / c->pyb_freq > c->track.episode_len_sec;
}
/* RewardWrapper._compute_reward (utils/wrapper.py:121-186) on drone 0's obs row */
static double race_reward_wrapper(int* wr_gate, double target[3], double prev[3], const double* row0, int term,
                                  int completed) {
    int gate_id = (int)row0[48];
    double r_passed = 0;
    if (gate_id > *wr_gate % 4) {
        *wr_gate = gate_id;
        if (gate_id < 4)   /* gate_positions has keys 0..3 (KeyError otherwise) */
            for (int k = 0; k < 3; ++k) target[k] = row0[12 + 4 * gate_id + k];
        r_passed = 5;
    }
    double r_col = (term && !completed) ? -1 : 0, r_lab = (term && completed) ? 10 : 0;
    double pxy = sqrt((target[0] - prev[0]) * (target[0] - prev[0]) + (target[1] - prev[1]) * (target[1] - prev[1]));
    double cxy = sqrt((target[0] - row0[0]) * (target[0] - row0[0]) + (target[1] - row0[1]) * (target[1] - row0[1]));
    double pz = fabs(target[2] - prev[2]), cz = fabs(target[2] - row0[2]);
    for (int k = 0; k < 3; ++k) prev[k] = row0[k];
    return (pxy - cxy) + (pz - cz) + r_passed + r_col + r_lab;
}

/* DroneObservationWrapper.step (wrapper.py:61-63): terminated once self.env.current_gate[0] >= 2.
   Stacked with the RewardWrapper, mode 1 = RewardWrapper(DroneObservationWrapper(env)) (the reward's
   terminal terms see the early termination), 2 = DroneObservationWrapper(RewardWrapper(env)). */
static void obs_wrapper_term(int mode, int term_env, int gate0, uint8_t* term, int* term_rw) {
    const int early = mode && gate0 >= 2;
    *term = (uint8_t)(term_env || early);
    *term_rw = mode == 1 ? (term_env || early) : term_env;
}
void orc_obs_wrapper_term(int mode, int term_env, int gate0, uint8_t* term, int* term_rw) {
    obs_wrapper_term(mode, term_env, gate0, term, term_rw);
}

static void race_step_env(orc_t* o, int e, const float* act, float* obs_env, float* rew, uint8_t* term,
                          uint8_t* trunc, float* tobs_env) {
    const adrp_config* c = &o->cfg;
    const adrp_track* t = &c->track;
    const int N = o->N;
    const uint64_t gid = (uint64_t)(c->env_offset + e);
    const uint32_t ep = (uint32_t)(o->episode[e] - 1);   /* episode index of the running episode */
    body_t* bs = &o->b[(size_t)e * N];
    rdrone_t* ds = &o->rd[(size_t)e * N];
    int touched = 0;
    for (int i = 0; i < N; ++i) {
        ds[i].mom_margin = INFINITY;
        ds[i].mom_hash = MOM_HASH_SEED;
        const size_t slot = (size_t)e * N + i;
        ds[i].rp_mom = o->rp_mom ? o->rp_mom + slot * (size_t)o->S * 3 : NULL;
        ds[i].rp_n = o->rp_mom ? o->rp_n[slot] : 0;
        ds[i].rp_call = 0;
    }
    /* the command message per drone (190-210): FULLSTATE (act[:3], 0, 0, act[3], 0, step_counter)
       from an ndarray action (act = NULL: the commands adrp_race_command / orc_race_command sent);
       eliminated drones get STOP [step_counter] */
    for (int i = 0; i < N; ++i) {
        double a[ADRP_CMD_ARGS] = {0};
        a[ADRP_CMD_TIME_SLOT] = o->step_counter[e];
        if (ds[i].elim) {
            hl_command(&ds[i], ADRP_CMD_STOP, a, 0);
        } else if (act) {
            for (int k = 0; k < 3; ++k) a[k] = act[(size_t)i * 4 + k];
            a[9] = act[(size_t)i * 4 + 3];   /* zeroed under the DroneObservationWrapper (wrapper.py:51-57) */
            hl_command(&ds[i], ADRP_CMD_FULLSTATE, a, t->obs_wrapper);
        }
    }
    for (int s = 0; s < o->S; ++s) {
        const uint32_t idx = (uint32_t)(o->step_counter[e] + s);
        if (c->physics != ADRP_PHYS_PYB)     /* KIN_PHYSICS: _updateAndStoreKinematicInformation */
            for (int i = 0; i < N; ++i) ds[i].kin_pos = bs[i].pos;
        forces_t F[ADRP_MAX_DRONES];
        if (c->physics != ADRP_PHYS_DYN)
            for (int i = 0; i < N; ++i) {
                assemble_forces(o, &F[i], bs, i, ds[i].rpm, ds[i].prev_rpm);
                if (t->disturbances) {       /* world-frame force on link 4 at posObj = self.pos (532-544) */
                    v3 f;
                    if (o->inj_force) {      /* parity mode: the caller's draws (orc_set_noise) */
                        const double* p = o->inj_force + (((size_t)e * N + i) * o->S + s) * 3;
                        f = V(p[0], p[1], p[2]);
                    } else {
                        double u[4];
                        draw4(c->seed, gid, ep, TAG_RACE_DIST | (uint32_t)i, idx, u);
                        f = V(t->dyn_dist_low[0] + (t->dyn_dist_high[0] - t->dyn_dist_low[0]) * u[0],
                              t->dyn_dist_low[1] + (t->dyn_dist_high[1] - t->dyn_dist_low[1]) * u[1],
                              t->dyn_dist_low[2] + (t->dyn_dist_high[2] - t->dyn_dist_low[2]) * u[2]);
                    }
                    v3 rel = vsub(ds[i].kin_pos, bs[i].link_pos);   /* posObj - cached link origin */
                    F[i].f_world[4] = vadd(F[i].f_world[4], f);
                    F[i].t_world[4] = vadd(F[i].t_world[4], vcross(rel, f));
                }
            }
        for (int i = 0; i < N; ++i) {
            if (c->physics == ADRP_PHYS_DYN) {
                dyn_step(o, &bs[i], ds[i].rpm);
            } else {
                F[i].base_f_world = V(0, 0, -c->gravity * ds[i].mass);
                touched |= bullet_step(o, &bs[i], &F[i], ds[i].mass, ds[i].inertia);
            }
            ds[i].kin_pos = bs[i].pos;       /* _updateAndStoreKinematicInformation (218) */
        }
        for (int i = 0; i < N; ++i) {
            rdrone_t* d = &ds[i];
            if (d->elim) {                   /* (233-235) */
                for (int k = 0; k < 4; ++k) d->prev_rpm[k] = d->rpm[k] = 0;
                continue;
            }
            double noise[4] = {0, 0, 0, 0};
            if (t->disturbances) {           /* (223-228) */
                if (o->inj_act) {            /* parity mode: the caller's draws (orc_set_noise) */
                    const double* p = o->inj_act + (((size_t)e * N + i) * o->S + s) * 4;
                    for (int k = 0; k < 4; ++k) noise[k] = p[k];
                } else {
                    draw_normal4(c->seed, gid, ep, TAG_RACE_NOISE | (uint32_t)i, idx, noise);
                    for (int k = 0; k < 4; ++k) noise[k] *= t->action_noise_std;
                }
            }
            double rpy[3], pos[3] = {bs[i].pos.x, bs[i].pos.y, bs[i].pos.z}, vel[3] = {bs[i].vel.x, bs[i].vel.y, bs[i].vel.z};
            body_rpy(&bs[i], rpy);
            memcpy(d->prev_rpm, d->rpm, sizeof d->rpm);
            mellinger_compute(d, pos, rpy, vel, noise, d->rpm);
        }
    }
    o->contact[e] = (uint8_t)touched;
    for (int i = 0; i < N; ++i) race_gate_progress(o, e, i);
    double row0[64 + 6 * ADRP_MAX_DRONES];
    race_write_obs(o, e, obs_env, row0);
    double pos[ADRP_MAX_DRONES][3], angv[ADRP_MAX_DRONES][3];
    uint8_t contact[ADRP_MAX_DRONES], elim[ADRP_MAX_DRONES], fin[ADRP_MAX_DRONES];
    for (int i = 0; i < N; ++i) {
        v3 w = body_ang_v(o, &bs[i]);
        pos[i][0] = bs[i].pos.x; pos[i][1] = bs[i].pos.y; pos[i][2] = bs[i].pos.z;
        angv[i][0] = w.x; angv[i][1] = w.y; angv[i][2] = w.z;
        contact[i] = (uint8_t)race_contact(o, e, i);
        elim[i] = (uint8_t)ds[i].elim; fin[i] = (uint8_t)ds[i].fin;
    }
    int all_fin = 1;
    *term = (uint8_t)race_terminated(t, N, (const double(*)[3])pos, (const double(*)[3])angv, contact, elim, fin);
    for (int i = 0; i < N; ++i) { ds[i].elim = elim[i]; all_fin &= fin[i]; }
    int term_rw;
    obs_wrapper_term(t->obs_wrapper, *term, ds[0].gate, term, &term_rw);
    *trunc = (uint8_t)race_truncated(c, o->step_counter[e]);
    double r = 0;
    if (t->reward_wrapper) {
        renv_t* re = &o->re[e];
        /* info["task_completed"] does not exist in the reference (KeyError, Q23):
           defined here as "every drone finished".  RewardWrapper(DroneObservationWrapper(env))
           (obs_wrapper 1) sees the wrapper's early termination, the other order (2) does not. */
        r = race_reward_wrapper(&re->wr_gate, re->wr_target, re->wr_prev, row0, term_rw, all_fin);
    }
    *rew = (float)r;
    o->step_counter[e] += o->S;                /* (268) */
    if (c->autoreset && (*term || *trunc)) {
        if (tobs_env) memcpy(tobs_env, obs_env, sizeof(float) * N * o->D);
        race_reset_env(o, e, obs_env);
    }
}

/* ---- race state snapshot (field order shared with libadrp) ---------------------------- */
static const char* race_field_name(int k) {
    static char buf[40];
    static const char* base[64] = {
        "pos_x", "pos_y", "pos_z", "quat_x", "quat_y", "quat_z", "quat_w", "vel_x", "vel_y", "vel_z",
        "omega_x", "omega_y", "omega_z", "rpm_0", "rpm_1", "rpm_2", "rpm_3", "prev_rpm_0", "prev_rpm_1",
        "prev_rpm_2", "prev_rpm_3", "angv_x", "angv_y", "angv_z", "link_quat_x", "link_quat_y", "link_quat_z",
        "link_quat_w", "link_pos_x", "link_pos_y", "link_pos_z", "kin_pos_x", "kin_pos_y", "kin_pos_z",
        "prev_rpy_0", "prev_rpy_1", "prev_rpy_2", "prev_vel_0", "prev_vel_1", "prev_vel_2",
        "lpf_d1_0", "lpf_d1_1", "lpf_d1_2", "lpf_d2_0", "lpf_d2_1", "lpf_d2_2",
        "i_err_0", "i_err_1", "i_err_2", "i_err_m_0", "i_err_m_1", "i_err_m_2",
        "prev_omega_roll", "prev_omega_pitch", "prev_sp_roll", "prev_sp_pitch",
        "ctl_roll", "ctl_pitch", "ctl_yaw", "ctl_thrust", "mass", "ixx", "iyy", "izz"};
    if (k < 0 || k >= RACE_NF) return NULL;
    if (k < 64) return base[k];
    static const char* gc[4] = {"x", "y", "z", "yaw"};
    static const char* oc[3] = {"x", "y", "z"};
    if (k < 80) { snprintf(buf, sizeof buf, "gate_%d_%s", (k - 64) / 4, gc[(k - 64) % 4]); return buf; }
    if (k < 92) { snprintf(buf, sizeof buf, "obst_%d_%s", (k - 80) / 3, oc[(k - 80) % 3]); return buf; }
    if (k < 95) { snprintf(buf, sizeof buf, "wr_target_%d", k - 92); return buf; }
    snprintf(buf, sizeof buf, "wr_prev_%d", k - 95);
    return buf;
}

static void race_get_row(const orc_t* o, size_t slot, int e, double* v, int32_t* iv) {
    const body_t* b = &o->b[slot];
    const rdrone_t* d = &o->rd[slot];
    const renv_t* re = &o->re[e];
    qt q = qconj(b->q_wtb), lq = qconj(b->link_q_wtb);
    v3 w = o->cfg.physics == ADRP_PHYS_DYN ? b->rpy_rates : b->omega;
    double base[64] = {b->pos.x, b->pos.y, b->pos.z, q.x, q.y, q.z, q.w, b->vel.x, b->vel.y, b->vel.z, w.x, w.y, w.z,
                       d->rpm[0], d->rpm[1], d->rpm[2], d->rpm[3], d->prev_rpm[0], d->prev_rpm[1], d->prev_rpm[2],
                       d->prev_rpm[3], b->ang_v.x, b->ang_v.y, b->ang_v.z, lq.x, lq.y, lq.z, lq.w,
                       b->link_pos.x, b->link_pos.y, b->link_pos.z, d->kin_pos.x, d->kin_pos.y, d->kin_pos.z,
                       d->prev_rpy[0], d->prev_rpy[1], d->prev_rpy[2], d->prev_vel[0], d->prev_vel[1], d->prev_vel[2],
                       d->lpf_d1[0], d->lpf_d1[1], d->lpf_d1[2], d->lpf_d2[0], d->lpf_d2[1], d->lpf_d2[2],
                       d->i_err[0], d->i_err[1], d->i_err[2], d->i_err_m[0], d->i_err_m[1], d->i_err_m[2],
                       d->prev_omega_roll, d->prev_omega_pitch, d->prev_sp_roll, d->prev_sp_pitch,
                       d->ctl[0], d->ctl[1], d->ctl[2], d->ctl[3], d->mass, d->inertia.x, d->inertia.y, d->inertia.z};
    memcpy(v, base, sizeof base);
    for (int g = 0; g < 4; ++g) for (int j = 0; j < 4; ++j) v[64 + 4 * g + j] = re->gate[g][j];
    for (int k = 0; k < 4; ++k) for (int j = 0; j < 3; ++j) v[80 + 3 * k + j] = re->obst[k][j];
    /* RewardWrapper state is per env and lives in drone 0's slot (0 elsewhere) */
    const int lead = (slot % (size_t)o->N) == 0;
    for (int j = 0; j < 3; ++j) { v[92 + j] = lead ? re->wr_target[j] : 0; v[95 + j] = lead ? re->wr_prev[j] : 0; }
    iv[0] = o->step_counter[e]; iv[1] = o->episode[e]; iv[2] = d->tick; iv[3] = d->last_att_tick;
    iv[4] = d->last_pos_tick; iv[5] = d->tumble; iv[6] = d->gate; iv[7] = (d->elim ? 1 : 0) | (d->fin ? 2 : 0);
    iv[8] = lead ? re->wr_gate : 0;
}

static void race_set_row(orc_t* o, size_t slot, int e, int first, const double* v, const int32_t* iv) {
    body_t* b = &o->b[slot];
    rdrone_t* d = &o->rd[slot];
    renv_t* re = &o->re[e];
    b->pos = V(v[0], v[1], v[2]);
    qt q = {v[3], v[4], v[5], v[6]};
    b->q_wtb = qconj(q);
    b->vel = V(v[7], v[8], v[9]);
    if (o->cfg.physics == ADRP_PHYS_DYN) { b->rpy_rates = V(v[10], v[11], v[12]); b->omega = V(v[21], v[22], v[23]); }
    else { b->omega = V(v[10], v[11], v[12]); b->rpy_rates = V(0, 0, 0); }
    for (int k = 0; k < 4; ++k) { d->rpm[k] = v[13 + k]; d->prev_rpm[k] = v[17 + k]; }
    b->ang_v = V(v[21], v[22], v[23]);
    qt lq = {v[24], v[25], v[26], v[27]};
    b->link_q_wtb = qconj(lq);
    b->link_pos = V(v[28], v[29], v[30]);
    d->kin_pos = V(v[31], v[32], v[33]);
    for (int k = 0; k < 3; ++k) {
        d->prev_rpy[k] = v[34 + k]; d->prev_vel[k] = v[37 + k];
        d->lpf_d1[k] = (float)v[40 + k]; d->lpf_d2[k] = (float)v[43 + k];
        d->i_err[k] = (float)v[46 + k]; d->i_err_m[k] = (float)v[49 + k];
    }
    d->prev_omega_roll = (float)v[52]; d->prev_omega_pitch = (float)v[53];
    d->prev_sp_roll = (float)v[54]; d->prev_sp_pitch = (float)v[55];
    for (int k = 0; k < 4; ++k) d->ctl[k] = (float)v[56 + k];
    d->mass = v[60]; d->inertia = V(v[61], v[62], v[63]);
    if (first) {
        for (int g = 0; g < 4; ++g) for (int j = 0; j < 4; ++j) re->gate[g][j] = v[64 + 4 * g + j];
        for (int k = 0; k < 4; ++k) for (int j = 0; j < 3; ++j) re->obst[k][j] = v[80 + 3 * k + j];
        for (int j = 0; j < 3; ++j) { re->wr_target[j] = v[92 + j]; re->wr_prev[j] = v[95 + j]; }
        o->step_counter[e] = iv[0]; o->episode[e] = iv[1]; re->wr_gate = iv[8];
    }
    d->tick = iv[2]; d->last_att_tick = iv[3]; d->last_pos_tick = iv[4]; d->tumble = iv[5]; d->gate = iv[6];
    d->elim = iv[7] & 1; d->fin = (iv[7] >> 1) & 1;
}

/* per drone slot: the smallest distance of a firmware moment to an int16 truncation point over the
   firmware calls of the last env.step (+inf: no call with positive thrust) */
int orc_race_moment_margin(const orc_t* o, float* out) {
    if (!o->rd) return ADRP_ERR_INVALID;
    for (size_t k = 0; k < (size_t)o->E * o->N; ++k) out[k] = o->rd[k].mom_margin;
    return 0;
}
int orc_race_moment_hash(const orc_t* o, uint32_t* out) {
    if (!o || !o->rd) return -1;
    for (size_t k = 0; k < (size_t)o->E * o->N; ++k) out[k] = o->rd[k].mom_hash;
    return 0;
}

/* diagnostics: the next steps take the firmware's int16 moments from `mom` ([E*N][S][3], call order,
   counts[E*N] calls per drone; the kernel's adrp_race_moment_log) instead of truncating their own;
   NULL turns it off.  The arrays are the caller's and must stay alive while it is on. */
int orc_race_set_moment_replay(orc_t* o, const int16_t* mom, const int32_t* counts) {
    if (o->cfg.task != ADRP_TASK_RACE) return fail("moment replay: MultiRaceAviary only");
    if ((mom == NULL) != (counts == NULL)) return fail("moment replay: both arrays or neither");
    o->rp_mom = mom;
    o->rp_n = counts;
    return 0;
}

int orc_set_noise(orc_t* o, const double* act_noise, const double* force) {
    if (o->cfg.task != ADRP_TASK_RACE) return fail("noise injection: MultiRaceAviary only");
    if ((act_noise == NULL) != (force == NULL)) return fail("noise injection: both arrays or neither");
    o->inj_act = act_noise;
    o->inj_force = force;
    return 0;
}

/* ---- high-level commands ---------------------------------------------------------------- */
int orc_race_command(orc_t* o, const int32_t* cmd, const double* args) {
    if (o->cfg.task != ADRP_TASK_RACE) return fail("commands: MultiRaceAviary only");
    const size_t EN = (size_t)o->E * o->N;
    for (size_t slot = 0; slot < EN; ++slot) {
        rdrone_t* d = &o->rd[slot];
        if (d->elim) {   /* MultiRaceAviary.py:198-199 */
            double a[ADRP_CMD_ARGS] = {0};
            a[ADRP_CMD_TIME_SLOT] = o->step_counter[slot / o->N];
            hl_command(d, ADRP_CMD_STOP, a, 0);
        } else {
            hl_command(d, cmd[slot], args + slot * ADRP_CMD_ARGS, o->cfg.track.obs_wrapper);
        }
    }
    return ADRP_OK;
}
/* float fields in adrp.h order: sp pos 3, vel 3, acc 3, rate 3, qz, qw, yaw; commander pos 3,
   vel 3, yaw; state pos 3, vel 3, yaw; t_begin, duration, coef 32 */
static void cmd_fields(rdrone_t* d, float* p[ADRP_CMD_NF], int* q[ADRP_CMD_NI]) {
    int n = 0;
    for (int k = 0; k < 3; ++k) p[n++] = &d->sp_pos[k];
    for (int k = 0; k < 3; ++k) p[n++] = &d->sp_vel[k];
    for (int k = 0; k < 3; ++k) p[n++] = &d->sp_acc[k];
    for (int k = 0; k < 3; ++k) p[n++] = &d->sp_rate[k];
    p[n++] = &d->sp_qz; p[n++] = &d->sp_qw; p[n++] = &d->sp_yaw;
    for (int k = 0; k < 3; ++k) p[n++] = &d->c_pos[k];
    for (int k = 0; k < 3; ++k) p[n++] = &d->c_vel[k];
    p[n++] = &d->c_yaw;
    for (int k = 0; k < 3; ++k) p[n++] = &d->st_pos[k];
    for (int k = 0; k < 3; ++k) p[n++] = &d->st_vel[k];
    p[n++] = &d->st_yaw;
    p[n++] = &d->plan_t0; p[n++] = &d->plan_dur;
    for (int a = 0; a < 4; ++a) for (int k = 0; k < 8; ++k) p[n++] = &d->coef[a][k];
    q[0] = &d->plan_state; q[1] = &d->override; q[2] = &d->sp_mode;
}
int orc_get_command_state(const orc_t* o, float* f, int32_t* ii) {
    if (o->cfg.task != ADRP_TASK_RACE) return fail("commands: MultiRaceAviary only");
    const size_t EN = (size_t)o->E * o->N;
    for (size_t slot = 0; slot < EN; ++slot) {
        float* p[ADRP_CMD_NF];
        int* q[ADRP_CMD_NI];
        cmd_fields(&o->rd[slot], p, q);
        for (int k = 0; k < ADRP_CMD_NF; ++k) f[k * EN + slot] = *p[k];
        for (int k = 0; k < ADRP_CMD_NI; ++k) ii[k * EN + slot] = *q[k];
    }
    return ADRP_OK;
}
int orc_set_command_state(orc_t* o, const float* f, const int32_t* ii) {
    if (o->cfg.task != ADRP_TASK_RACE) return fail("commands: MultiRaceAviary only");
    const size_t EN = (size_t)o->E * o->N;
    for (size_t slot = 0; slot < EN; ++slot) {
        float* p[ADRP_CMD_NF];
        int* q[ADRP_CMD_NI];
        cmd_fields(&o->rd[slot], p, q);
        for (int k = 0; k < ADRP_CMD_NF; ++k) *p[k] = f[k * EN + slot];
        for (int k = 0; k < ADRP_CMD_NI; ++k) *q[k] = ii[k * EN + slot];
    }
    return ADRP_OK;
}
void orc_poly4d_eval(const float* coef, float t, float out[13]) {
    float c[4][8];
    memcpy(c, coef, sizeof c);
    traj_eval_t ev = poly4d_eval((const float(*)[8])c, t);
    const f3 v[4] = {ev.pos, ev.vel, ev.acc, ev.omega};
    for (int k = 0; k < 4; ++k) { out[3 * k] = v[k].x; out[3 * k + 1] = v[k].y; out[3 * k + 2] = v[k].z; }
    out[12] = ev.yaw;
}
void orc_poly7_nojerk(float T, float x0, float dx0, float ddx0, float xf, float dxf, float ddxf, float out[8]) {
    poly7_nojerk(out, T, x0, dx0, ddx0, xf, dxf, ddxf);
}

/* ---- unit entry points for tests ------------------------------------------------------ */
/* distance between the drone collision cylinder at (pos, quat xyzw) and gate g / obstacle k
   (kind 0 = gate type t at pose x,y,z,yaw; kind 1 = obstacle at x,y,z) */
double orc_race_body_distance(const adrp_config* cfg, const double pos[3], const double quat[4], int kind,
                              int gate_type, const double pose[4]) {
    orc_t o;
    memset(&o, 0, sizeof o);
    o.cfg = *cfg;
    body_t b;
    memset(&b, 0, sizeof b);
    b.pos = V(pos[0], pos[1], pos[2]);
    qt q = {quat[0], quat[1], quat[2], quat[3]};
    b.q_wtb = qconj(q);
    shape_t ds = drone_shape(&o, &b);
    part_t parts[5];
    if (kind == 0) return body_distance(&ds, parts, gate_parts(gate_type > 0, parts), V(pose[0], pose[1], pose[2]), rot_z(pose[3]));
    return body_distance(&ds, parts, obstacle_parts(parts), V(pose[0], pose[1], pose[2]), m_eye());
}
/* distance between two oriented boxes/cylinders: s = {type, cx,cy,cz, 9 R row-major, hx,hy,hz, r} */
double orc_shape_distance(const double* a, const double* b) {
    shape_t s[2];
    const double* p[2] = {a, b};
    for (int k = 0; k < 2; ++k) {
        s[k].type = (int)p[k][0];
        s[k].c = V(p[k][1], p[k][2], p[k][3]);
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) s[k].R.m[i][j] = p[k][4 + 3 * i + j];
        s[k].h = V(p[k][13], p[k][14], p[k][15]);
        s[k].r = p[k][16];
    }
    return gjk_distance(&s[0], &s[1]);
}
/* lpf2p coefficients b0,b1,b2,a1,a2 (firmware filter.c) */
void orc_lpf_coeffs(double fs, double fc, double out[5]) {
    lpf_t l = lpf_coeffs((float)fs, (float)fc);
    out[0] = l.b0; out[1] = l.b1; out[2] = l.b2; out[3] = l.a1; out[4] = l.a2;
}

/* ---- decision-logic entry points (golden tests against the reference's Python) ------- */
int orc_race_obs_assemble(const adrp_config* cfg, int N, int i, const double* kin, const double* gate_act,
                          const uint8_t* gate_in, const double* obst_act, const uint8_t* obst_in, int current_gate,
                          double* row) {
    if (N < 1 || N > ADRP_MAX_DRONES || i < 0 || i >= N) return fail("drone index");
    race_obs_assemble(cfg, N, i, (const double(*)[12])kin, (const double(*)[4])gate_act, gate_in,
                      (const double(*)[3])obst_act, obst_in, current_gate, row);
    return ADRP_OK;
}
int orc_race_terminated(const adrp_config* cfg, int N, const double* pos, const double* angv, const uint8_t* contact,
                        uint8_t* elim, const uint8_t* fin) {
    return race_terminated(&cfg->track, N, (const double(*)[3])pos, (const double(*)[3])angv, contact, elim, fin);
}
int orc_race_truncated(const adrp_config* cfg, int step_counter) { return race_truncated(cfg, step_counter); }
void orc_race_rays(const double gate_xyyaw[3], int type, double* from, double* to) {
    race_rays(gate_xyyaw, type, (double(*)[3])from, (double(*)[3])to);
}
void orc_race_progress(int num_gates, int self_id, const int* hit_id, const double* hit_frac, int* gate, int* fin) {
    race_progress_decide(num_gates, self_id, hit_id, hit_frac, gate, fin);
}
double orc_race_reward(int* wr_gate, double* target, double* prev, const double* row0, int term, int completed) {
    return race_reward_wrapper(wr_gate, target, prev, row0, term, completed);
}
