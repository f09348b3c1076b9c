// commander.h — the Crazyflie high-level commander in the race step.
//
// Reference call sites: low_level_control (control/MellingerControl.py:17-61) hands each command
// message to send*Cmd and then process_command_queue(args[-1]) (292-303: HighLevelStop,
// UpdateTime(args[-1]), the queued _send*Cmd, 491-699); while full_state_cmd_override is off every
// controller call runs _update_setpoint (369-374: TellState, UpdateTime(tick / 500), GetSetpoint).
// The firmware pieces (crtp_commander_high_level.c, planner.c, pptraj.c) are not in the reference
// (pycffirmware is an un-vendored dependency): they follow the published algorithm, as the oracle's
// restatement does (oracle/race.c hl_*), in C float with FP contraction off.  Parity unpinned.
//
// State: per drone, float [ADRP_CMD_NF][E*N] + int32 [ADRP_CMD_NI][E*N] (adrp.h order).  The
// command kernel writes it once per env.step; the step kernel (CMD instantiation) keeps the scalar
// part in registers and reads the 32 polynomial coefficients from memory when it evaluates the
// trajectory (only while the commander drives the setpoint).
#pragma once

#include "../../include/adrp.h"

namespace adrp {

enum CmdField {
    CF_SP_POS = 0, CF_SP_VEL = 3, CF_SP_ACC = 6, CF_SP_RATE = 9, CF_SP_QZ = 12, CF_SP_QW = 13, CF_SP_YAW = 14,
    CF_C_POS = 15, CF_C_VEL = 18, CF_C_YAW = 21, CF_ST_POS = 22, CF_ST_VEL = 25, CF_ST_YAW = 28,
    CF_T0 = 29, CF_DUR = 30, CF_COEF = 31, CF_N = 63
};
enum CmdInt { CI_PLAN = 0, CI_OVR = 1, CI_MODE = 2, CI_N = 3 };
static_assert(CF_N == ADRP_CMD_NF && CI_N == ADRP_CMD_NI, "command state layout (adrp.h)");
enum { PLAN_IDLE = 0, PLAN_FLYING = 1, PLAN_LANDING = 2 };
enum { SP_UNSET = 0, SP_FULLSTATE = 1, SP_COMMANDER = 2 };

constexpr float kPiF = 3.14159265358979323846f;

// the register part of the command state
struct CmdState {
    float sp_pos[3], sp_vel[3], sp_acc[3], sp_rate[3], sp_qz, sp_qw, sp_yaw;
    float c_pos[3], c_vel[3], c_yaw;
    float st_pos[3], st_vel[3], st_yaw;
    float t0, dur;
    int plan, ovr, mode;
};

__device__ __forceinline__ void cmd_load(const float* cf, const int32_t* ci, size_t EN, size_t slot, CmdState& c) {
#define L_(k) cf[size_t(k) * EN + slot]
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        c.sp_pos[k] = L_(CF_SP_POS + k); c.sp_vel[k] = L_(CF_SP_VEL + k); c.sp_acc[k] = L_(CF_SP_ACC + k);
        c.sp_rate[k] = L_(CF_SP_RATE + k); c.c_pos[k] = L_(CF_C_POS + k); c.c_vel[k] = L_(CF_C_VEL + k);
        c.st_pos[k] = L_(CF_ST_POS + k); c.st_vel[k] = L_(CF_ST_VEL + k);
    }
    c.sp_qz = L_(CF_SP_QZ); c.sp_qw = L_(CF_SP_QW); c.sp_yaw = L_(CF_SP_YAW);
    c.c_yaw = L_(CF_C_YAW); c.st_yaw = L_(CF_ST_YAW); c.t0 = L_(CF_T0); c.dur = L_(CF_DUR);
#undef L_
    c.plan = ci[CI_PLAN * EN + slot]; c.ovr = ci[CI_OVR * EN + slot]; c.mode = ci[CI_MODE * EN + slot];
}

__device__ __forceinline__ void cmd_store(float* cf, int32_t* ci, size_t EN, size_t slot, const CmdState& c) {
#define S_(k, v) cf[size_t(k) * EN + slot] = (v)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        S_(CF_SP_POS + k, c.sp_pos[k]); S_(CF_SP_VEL + k, c.sp_vel[k]); S_(CF_SP_ACC + k, c.sp_acc[k]);
        S_(CF_SP_RATE + k, c.sp_rate[k]); S_(CF_C_POS + k, c.c_pos[k]); S_(CF_C_VEL + k, c.c_vel[k]);
        S_(CF_ST_POS + k, c.st_pos[k]); S_(CF_ST_VEL + k, c.st_vel[k]);
    }
    S_(CF_SP_QZ, c.sp_qz); S_(CF_SP_QW, c.sp_qw); S_(CF_SP_YAW, c.sp_yaw);
    S_(CF_C_YAW, c.c_yaw); S_(CF_ST_YAW, c.st_yaw); S_(CF_T0, c.t0); S_(CF_DUR, c.dur);
#undef S_
    ci[CI_PLAN * EN + slot] = c.plan; ci[CI_OVR * EN + slot] = c.ovr; ci[CI_MODE * EN + slot] = c.mode;
}

// math3d / pptraj helpers (firmware C float)
__device__ __forceinline__ float hl_rad(float d) { return (kPiF / 180.0f) * d; }
__device__ __forceinline__ float hl_deg(float r) { return (180.0f / kPiF) * r; }

// pptraj.c poly7_nojerk: x, x', x'' given and x''' = 0 at t = 0 and t = T
__device__ __forceinline__ void hl_poly7_nojerk(float p[8], float T, float x0, float dx0, float ddx0, float xf) {
#pragma clang fp contract(off)
    const float dxf = 0.0f, ddxf = 0.0f;
    if (T <= 0.0f) {
        p[0] = xf; p[1] = dxf; p[2] = ddxf / 2;
#pragma unroll
        for (int i = 3; i < 8; ++i) p[i] = 0.0f;
        return;
    }
    const float T2 = T * T, T3 = T2 * T, T4 = T3 * T, T5 = T4 * T, T6 = T5 * T, T7 = T6 * T;
    p[0] = x0; p[1] = dx0; p[2] = ddx0 / 2; p[3] = 0.0f;
    p[4] = -(5 * (14 * x0 - 14 * xf + 8 * T * dx0 + 6 * T * dxf + 2 * T2 * ddx0 - T2 * ddxf)) / (2 * T4);
    p[5] = (84 * x0 - 84 * xf + 45 * T * dx0 + 39 * T * dxf + 10 * T2 * ddx0 - 7 * T2 * ddxf) / T5;
    p[6] = -(140 * x0 - 140 * xf + 72 * T * dx0 + 68 * T * dxf + 15 * T2 * ddx0 - 13 * T2 * ddxf) / (2 * T6);
    p[7] = (2 * (10 * x0 - 10 * xf + 5 * T * dx0 + 5 * T * dxf + T2 * ddx0 - T2 * ddxf)) / T7;
}

// value and the first three derivatives of one axis (polyval after successive in-place polyder)
__device__ __forceinline__ void hl_polyval4(const float* coef, size_t EN, size_t slot, float t, float out[4]) {
#pragma clang fp contract(off)
    float p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = coef[size_t(i) * EN + slot];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        float x = 0.0f;
#pragma unroll
        for (int i = 7 - d; i >= 0; --i) x = x * t + p[i];
        out[d] = x;
#pragma unroll
        for (int i = 1; i <= 7 - d; ++i) p[i - 1] = float(i) * p[i];
    }
}

struct TrajEval { float pos[3], vel[3], acc[3], omega[3], yaw; };

// poly4d_eval (pptraj.c) of the coefficients at coef (CF_COEF block)
__device__ __forceinline__ TrajEval hl_poly4d_eval(const float* coef, size_t EN, size_t slot, float t) {
#pragma clang fp contract(off)
    TrajEval o;
    float v[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) hl_polyval4(coef + size_t(8 * a) * EN, EN, slot, t, v[a]);
    float jerk[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { o.pos[k] = v[k][0]; o.vel[k] = v[k][1]; o.acc[k] = v[k][2]; jerk[k] = v[k][3]; }
    o.yaw = v[3][0];
    const float dyaw = v[3][1];
    const float th[3] = {o.acc[0] + 0.0f, o.acc[1] + 0.0f, o.acc[2] + 9.81f};   // vadd(acc, (0, 0, GRAV))
    const float thn = sqrtf(th[0] * th[0] + th[1] * th[1] + th[2] * th[2]);
    const float izb = 1.0f / thn;                                              // vnormalize = vscl(1/|v|, v)
    const float zb[3] = {izb * th[0], izb * th[1], izb * th[2]};
    const float xw[3] = {cosf(o.yaw), sinf(o.yaw), 0.0f};
    float yb[3] = {zb[1] * xw[2] - zb[2] * xw[1], zb[2] * xw[0] - zb[0] * xw[2], zb[0] * xw[1] - zb[1] * xw[0]};
    const float iyb = 1.0f / sqrtf(yb[0] * yb[0] + yb[1] * yb[1] + yb[2] * yb[2]);
#pragma unroll
    for (int k = 0; k < 3; ++k) yb[k] = iyb * yb[k];
    const float xb[3] = {yb[1] * zb[2] - yb[2] * zb[1], yb[2] * zb[0] - yb[0] * zb[2], yb[0] * zb[1] - yb[1] * zb[0]};
    const float jz = jerk[0] * zb[0] + jerk[1] * zb[1] + jerk[2] * zb[2];           // vorthunit(jerk, z_body)
    const float jo[3] = {jerk[0] - jz * zb[0], jerk[1] - jz * zb[1], jerk[2] - jz * zb[2]};
    const float ith = 1.0f / sqrtf(th[0] * th[0] + th[1] * th[1] + th[2] * th[2]);
    const float hw[3] = {ith * jo[0], ith * jo[1], ith * jo[2]};
    o.omega[0] = -(hw[0] * yb[0] + hw[1] * yb[1] + hw[2] * yb[2]);
    o.omega[1] = hw[0] * xb[0] + hw[1] * xb[1] + hw[2] * xb[2];
    o.omega[2] = zb[2] * dyaw;
    return o;
}

// crtpCommanderHighLevelTellState(state)
__device__ __forceinline__ void hl_tell_state(CmdState& c) {
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < 3; ++k) { c.c_pos[k] = c.st_pos[k]; c.c_vel[k] = c.st_vel[k]; }
    c.c_yaw = c.st_yaw * kPiF / 180.0f;
}

// _update_setpoint (MellingerControl.py:369-374) at t = tick / 500: TellState, UpdateTime,
// GetSetpoint = plan_current_goal (piecewise_eval, LANDING -> IDLE once finished) and, unless the
// planner is stopped, the setpoint (x, y, z, yaw modeAbs; rates in deg/s) and the commander's pos.
// Before t_begin the polynomial is extrapolated, as the firmware's piecewise_eval does.
__device__ __forceinline__ void hl_update_setpoint(CmdState& c, const float* coef, size_t EN, size_t slot, float t) {
#pragma clang fp contract(off)
    hl_tell_state(c);
    if (c.plan == PLAN_LANDING && t - c.t0 >= c.dur * 1.0f) c.plan = PLAN_IDLE;
    if (c.plan == PLAN_IDLE) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { c.c_pos[k] = c.st_pos[k]; c.c_vel[k] = c.st_vel[k]; }
        c.c_yaw = hl_rad(c.st_yaw);
        return;
    }
    const float tr = t - c.t0;
    const bool past = !(tr <= c.dur * 1.0f);
    TrajEval ev = hl_poly4d_eval(coef, EN, slot, past ? c.dur : tr);
    if (past) {
#pragma unroll
        for (int k = 0; k < 3; ++k) ev.vel[k] = ev.acc[k] = ev.omega[k] = 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        c.sp_pos[k] = ev.pos[k]; c.sp_vel[k] = ev.vel[k]; c.sp_acc[k] = ev.acc[k];
        c.sp_rate[k] = hl_deg(ev.omega[k]);
        c.c_pos[k] = ev.pos[k]; c.c_vel[k] = ev.vel[k];
    }
    c.sp_yaw = hl_deg(ev.yaw);
    c.c_yaw = ev.yaw;
    c.mode = SP_COMMANDER;
}

// piecewise_plan_7th_order_no_jerk into the planner (end velocity, acceleration, yaw rate 0)
__device__ __forceinline__ void hl_plan(CmdState& c, float* coef, size_t EN, size_t slot, int state, float t,
                                        float dur, const float p0[3], float y0, const float v0[3], const float p1[3],
                                        float y1) {
    float p[8];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        if (a < 3) hl_poly7_nojerk(p, dur, p0[a], v0[a], 0.0f, p1[a]);
        else hl_poly7_nojerk(p, dur, y0, 0.0f, 0.0f, y1);
#pragma unroll
        for (int i = 0; i < 8; ++i) coef[size_t(8 * a + i) * EN + slot] = p[i];
    }
    c.dur = dur;
    c.plan = state;
    c.t0 = t;
}

__device__ __forceinline__ float hl_shortest_signed_angle(float start, float goal) {
#pragma clang fp contract(off)
    const float diff = goal - start;
    float sd = fmodf(diff + kPiF, 2 * kPiF) - kPiF;
    if (sd < -kPiF) sd += 2 * kPiF;
    return sd;
}

// one command message (low_level_control -> send*Cmd -> process_command_queue(args[-1])):
// crtpCommanderHighLevelStop, UpdateTime(args[ADRP_CMD_TIME_SLOT]), the queued _send*Cmd.
// The planner is stopped first, so a takeoff always starts from IDLE, a landing never does
// (plan_land refuses IDLE), and a go_to starts from the commander's last pos / vel / yaw.
__device__ __forceinline__ void hl_command(CmdState& c, float* coef, size_t EN, size_t slot, int code,
                                           const double* a, bool zero_yaw) {
#pragma clang fp contract(off)
    if (code <= ADRP_CMD_NONE || code > ADRP_CMD_NOTIFY) return;
    c.plan = PLAN_IDLE;
    const float t = float(a[ADRP_CMD_TIME_SLOT]);
    const float zero[3] = {0.0f, 0.0f, 0.0f};
    if (code == ADRP_CMD_FULLSTATE) {   // _sendFullStateCmd (510-543)
        const double yaw = zero_yaw ? 0.0 : a[9];   // DroneObservationWrapper (wrapper.py:56-57)
        double sq, cq;
        sincos(yaw * 0.5, &sq, &cq);   // get_quaternion_from_euler(0, 0, yaw): (0, 0, sin, cos)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            c.sp_pos[k] = float(a[k]); c.sp_vel[k] = float(a[3 + k]); c.sp_acc[k] = float(a[6 + k]);
            c.sp_rate[k] = float(a[10 + k] * 57.29577951308232);
        }
        c.sp_qz = float(sq);
        c.sp_qw = float(cq);
        c.mode = SP_FULLSTATE;
        c.ovr = 1;
        return;
    }
    const float h = float(a[0]);
    if (code == ADRP_CMD_TAKEOFF || code == ADRP_CMD_TAKEOFFYAW || code == ADRP_CMD_TAKEOFFVEL) {
        float hh = h, hyaw = c.c_yaw, dur = float(a[1]);
        if (code == ADRP_CMD_TAKEOFFYAW) hyaw = float(a[2]);
        if (code == ADRP_CMD_TAKEOFFVEL) {   // takeoff_with_velocity
            if (a[2] != 0.0) hh += c.c_pos[2];
            const float v = float(a[1]) > 0.0f ? float(a[1]) : 0.5f;
            dur = fabsf(hh - c.c_pos[2]) / v;
        }
        const float p1[3] = {c.c_pos[0], c.c_pos[1], hh};
        hl_plan(c, coef, EN, slot, PLAN_FLYING, t, dur, c.c_pos, c.c_yaw, zero, p1, hyaw);
    } else if (code == ADRP_CMD_GOTO) {   // go_to from a stopped planner (plan_go_to_from)
        float p1[3] = {float(a[0]), float(a[1]), float(a[2])}, hyaw = float(a[3]);
        if (a[5] != 0.0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) p1[k] = p1[k] + c.c_pos[k];
            hyaw += c.c_yaw;
        }
        const float end_yaw = c.c_yaw + hl_shortest_signed_angle(c.c_yaw, hyaw);
        hl_plan(c, coef, EN, slot, PLAN_FLYING, t, float(a[4]), c.c_pos, c.c_yaw, c.c_vel, p1, end_yaw);
    } else if (code == ADRP_CMD_NOTIFY) {
        hl_tell_state(c);
    }
    // LAND / LANDYAW / LANDVEL: plan_land refuses the stopped planner; STOP: stopped
    c.ovr = 0;
}

// reset (MellingerControl.py:119-150): zeroed setpoint_t, override on, planner IDLE,
// _update_state from the initial obs row (nominal pose, at rest), TellState
__device__ __forceinline__ void hl_reset(CmdState& c, float px, float py, float pz, float yaw_deg) {
#pragma unroll
    for (int k = 0; k < 3; ++k) { c.sp_pos[k] = c.sp_vel[k] = c.sp_acc[k] = c.sp_rate[k] = 0.0f; c.st_vel[k] = 0.0f; }
    c.st_pos[0] = px; c.st_pos[1] = py; c.st_pos[2] = pz;
    c.sp_qz = c.sp_qw = c.sp_yaw = 0.0f;
    c.st_yaw = yaw_deg;
    c.t0 = c.dur = 0.0f;
    c.plan = PLAN_IDLE; c.ovr = 1; c.mode = SP_UNSET;
    hl_tell_state(c);
}

}  // namespace adrp
