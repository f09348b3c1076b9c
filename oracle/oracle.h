/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.  CPU float64 restatement of the reference hot
 * path (HoverAviary / MultiRaceAviary env.step of FelixWaiblinger/gym-pybullet-adrp),
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product (libadrp.so) never links, loads or calls this code.
 *
 * Parity status (details in DESIGN.md §Oracle):
 *   - pinned by golden fixtures generated from the reference's own Python
 *     (tests/golden/make_golden.py): HoverAviary action preprocessing, obs assembly,
 *     reward / terminated / truncated, URDF-derived constants, the Physics.DYN
 *     integrator, the PYB force assembly (_physics/_groundEffect/_drag/_downwash,
 *     captured through a force-recording pybullet stand-in), the Mellinger wrapper
 *     arithmetic (_compute_pwms, _thr2pwm, PWM<->RPM) and its float64 tick schedule,
 *     get_quaternion_from_euler, MultiRace termination/truncation/obs assembly.
 *   - parity unpinned (no runnable pybullet / pycffirmware here): the Bullet
 *     btMultiBody integration step (restated from Bullet 3.x, pybullet ^3.2.5,
 *     pyproject.toml:20), Bullet collision/ray/proximity queries, and the Crazyflie
 *     firmware Mellinger controller + lpf2p, and the firmware's high-level commander /
 *     planner (restated from the published algorithm).
 */
#ifndef ADRP_ORACLE_H
#define ADRP_ORACLE_H

#include <stdint.h>
#include "../include/adrp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_handle orc_t;

int orc_create(const adrp_config* cfg, orc_t** out);
void orc_destroy(orc_t* o);
const char* orc_last_error(void);
int orc_obs_dim(const orc_t* o);
int orc_act_dim(const orc_t* o);
int orc_reset(orc_t* o, const uint8_t* env_mask, float* obs);
int orc_step(orc_t* o, const float* act, float* obs, float* rew, uint8_t* term,
             uint8_t* trunc, float* terminal_obs);
/* MultiRace high-level commands (adrp.h ADRP_CMD_*): one command per drone, cmd [E*N], args
   [E*N][ADRP_CMD_ARGS]; then orc_step(o, NULL, ...) keeps the setpoints.  The command state
   snapshot has the adrp_get_command_state layout (float [ADRP_CMD_NF][E*N], int [ADRP_CMD_NI][E*N]). */
int orc_race_command(orc_t* o, const int32_t* cmd, const double* args);
/* MultiRace parity mode (adrp.h adrp_set_noise): the next steps take the action noise [E*N][S][4]
   and the disturbance force [E*N][S][3] of sub-step s of drone slot e*N+n from these host arrays
   (kept by pointer) instead of the Philox draws; NULL, NULL returns to Philox */
int orc_set_noise(orc_t* o, const double* act_noise, const double* force);
/* firmware int16 moments replayed from the kernel's log ([E*N][S][3] + counts; NULL, NULL: off) */
int orc_race_set_moment_replay(orc_t* o, const int16_t* mom, const int32_t* counts);
int orc_race_moment_margin(const orc_t* o, float* out);
int orc_race_moment_hash(const orc_t* o, uint32_t* out);   /* fw_moment_hash of the last step, per drone */
int orc_normal_pair(uint32_t x0, uint32_t x1, float* z);
int orc_get_command_state(const orc_t* o, float* f, int32_t* i);
int orc_set_command_state(orc_t* o, const float* f, const int32_t* i);
/* one poly4d_eval of the commander's trajectory (tests): coef [4][8], out = pos 3, vel 3, acc 3,
   omega 3, yaw; poly7_nojerk coefficients */
void orc_poly4d_eval(const float* coef, float t, float out[13]);
void orc_poly7_nojerk(float T, float x0, float dx0, float ddx0, float xf, float dxf, float ddxf, float out[8]);
int orc_state_layout(const orc_t* o, int* nf, int* ni);
const char* orc_state_field(const orc_t* o, int is_int, int index);
int orc_get_state(const orc_t* o, double* f, int32_t* i);
int orc_set_state(orc_t* o, const double* f, const int32_t* i);
/* number of (env, drone) sub-steps that touched the ground model in the last orc_step */
int64_t orc_contact_count(const orc_t* o);
uint8_t orc_env_contact(const orc_t* o, int env);

/* unit entry points (golden / known-answer tests) */
void orc_default_config(int task, adrp_config* cfg);
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void orc_euler_from_quat(const double q[4], double rpy[3]);
void orc_quat_from_euler(const double rpy[3], double q[4]);
void orc_derived_constants(const adrp_config* cfg, double out[6]);
/* Force assembly of one sub-step for drone n among N drones of one env at the given
 * states (rows of pos3, quat4 xyzw, vel3, omega3), as the reference's
 * _physics/_groundEffect/_drag/_downwash would apply it: link_force[5][3] and
 * link_torque[5][3] in the LINK frame (sum of all applyExternalForce/Torque calls per
 * link index 0..4).  rpm = clipped_action, prev_rpm = last_clipped_action. */
int orc_force_assembly(const adrp_config* cfg, int N, const double* states, int n, const double rpm[4],
                       const double prev_rpm[4], double link_force[5][3], double link_torque[5][3]);
void orc_hover_rpm(const adrp_config* cfg, const float* act, double rpm[4]);
/* DSLPIDControl.computeControl (control/DSLPIDControl.py:82-259): in = pos 3, quat 4, vel 3,
 * target_pos 3, target_rpy 3, target_vel 3; st = last_rpy 3, integral_pos_e 3,
 * integral_rpy_e 3 (in/out) */
void orc_dslpid(const adrp_config* cfg, double dt, const double in[19], double st[9], double rpm[4]);
/* HoverAviary obs / reward / terminated / truncated at the current state (no physics,
 * step_counter unchanged): _computeObs/_computeReward/_computeTerminated/_computeTruncated */
int orc_hover_eval(const orc_t* o, float* obs, float* rew, uint8_t* term, uint8_t* trunc);
/* Mellinger wrapper pieces (control/MellingerControl.py:423-442, 307-343, 246-262) */
void orc_compute_pwms(const double control[4], double pwm[4]);
void orc_pwms_to_rpms(const double pwm[4], const double noise[4], double rpm[4]);
int orc_tick_schedule(int n, uint8_t* ticks);
uint32_t orc_config_size(void);
/* 1: integrate the base without the spatial -> classical "+ w x v" term (probe of an unpinned
 * Bullet reading, tests/test_closed_form.py); 0 (default): the restatement */
void orc_set_bullet_variant(int omit_wxv);
/* DroneObservationWrapper termination (oracle/race.c obs_wrapper_term) */
void orc_obs_wrapper_term(int mode, int term_env, int gate0, uint8_t* term, int* term_rw);

#ifdef __cplusplus
}
#endif

#endif
