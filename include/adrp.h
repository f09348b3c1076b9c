/*
 * adrp.h — C-ABI of the MI355X-native batched quadrotor step (libadrp.so).
 *
 * One handle = one batch of E independent envs x N drones resident in the HBM of one
 * GPU.  Every pointer argument named *_dev is a DEVICE pointer (e.g. a torch tensor's
 * data_ptr() on the same GPU); `stream` is a hipStream_t (NULL = default stream).
 * All calls are stream-ordered and asynchronous; none of them synchronises the host
 * except adrp_create / adrp_destroy.  Return codes: ADRP_OK (0) or a negative
 * ADRP_ERR_*; nothing throws across the ABI.  adrp_last_error() gives the text.
 *
 * Reference interfaces replaced (file:line into FelixWaiblinger/gym-pybullet-adrp
 * snapshot 2024-10-08):
 *   adrp_create  <- BaseAviary.__init__            envs/BaseAviary.py:25-219
 *                   HoverAviary.__init__           envs/HoverAviary.py:11-64
 *                   MultiRaceAviary.__init__       envs/MultiRaceAviary.py:31-123
 *                   (+ the controller processes    envs/MultiRaceAviary.py:107-115)
 *   adrp_reset   <- BaseAviary.reset               envs/BaseAviary.py:223-258
 *                   MultiRaceAviary.reset          envs/MultiRaceAviary.py:127-167
 *   adrp_step    <- BaseAviary.step                envs/BaseAviary.py:262-387
 *                   MultiRaceAviary.step           envs/MultiRaceAviary.py:171-270
 *                   (+ MellingerControl.computeControl control/MellingerControl.py:154-262
 *                    + RewardWrapper._compute_reward utils/wrapper.py:121-186)
 *   adrp_get_state / adrp_set_state
 *                <- p.getBasePositionAndOrientation / p.resetBasePositionAndOrientation /
 *                   p.getBaseVelocity / p.resetBaseVelocity (BaseAviary.py:520-523,
 *                   MultiRaceAviary.py:456-467): state snapshot / teacher forcing
 *   adrp_destroy <- BaseAviary.close / MultiRaceAviary.close
 *                   envs/BaseAviary.py:420-425, envs/MultiRaceAviary.py:274-280
 */
#ifndef ADRP_H
#define ADRP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADRP_ABI_VERSION 2

#define ADRP_MAX_DRONES 8
#define ADRP_MAX_GATES 4      /* MultiRaceAviary._computeObs hard-codes 4 (MultiRaceAviary.py:591-651) */
#define ADRP_MAX_OBSTACLES 4

/* status codes */
#define ADRP_OK 0
#define ADRP_ERR_INVALID (-1)   /* bad argument / config (cf. ValueError, BaseAviary.py:79-80) */
#define ADRP_ERR_DEVICE (-2)    /* HIP runtime error */
#define ADRP_ERR_OOM (-3)       /* device allocation failed */

/* adrp_config.task */
#define ADRP_TASK_HOVER 0       /* HoverAviary (envs/HoverAviary.py) */
#define ADRP_TASK_RACE 1        /* MultiRaceAviary (envs/MultiRaceAviary.py) */

/* adrp_config.physics — utils/enums.py:18-26 (Physics) */
#define ADRP_PHYS_PYB 0
#define ADRP_PHYS_DYN 1
#define ADRP_PHYS_PYB_GND 2
#define ADRP_PHYS_PYB_DRAG 3
#define ADRP_PHYS_PYB_DW 4
#define ADRP_PHYS_PYB_GND_DRAG_DW 5

/* adrp_config.act_type — utils/enums.py:40-47 (ActionType) */
#define ADRP_ACT_RPM 0          /* HoverAviary: a in [-1,1]^4 -> HOVER_RPM*(1+0.05a) (BaseRLAviary.py:192) */
#define ADRP_ACT_ONE_D_RPM 1    /* HoverAviary: a in [-1,1]   -> 4 x HOVER_RPM*(1+0.05a) (BaseRLAviary.py:225) */
#define ADRP_ACT_FULLSTATE 2    /* MultiRace: [x,y,z,yaw] absolute FULLSTATE setpoint (MultiRaceAviary.py:190-194) */
/* HoverAviary with the fused DSLPIDControl (control/DSLPIDControl.py:82-259), once per env.step */
#define ADRP_ACT_PID 3          /* a in R^3: waypoint, capped 1 m away (BaseRLAviary.py:193-207, BaseAviary.py:1112-1160) */
#define ADRP_ACT_VEL 4          /* a in R^4: direction + |a3| x SPEED_LIMIT target velocity (BaseRLAviary.py:208-223) */
#define ADRP_ACT_ONE_D_PID 5    /* a in R:   target z = z + 0.1a (BaseRLAviary.py:226-235) */

/* adrp_config.race_mode — utils/enums.py:84-87 (RaceMode) */
#define ADRP_RACE_COMPARE 0
#define ADRP_RACE_COMPETE 1

/* High-level commands: utils/enums.py:58-70 (Command), as MultiRaceAviary.step sends them to
 * each drone's MellingerControl (envs/MultiRaceAviary.py:190-210, control/MellingerControl.py:17-61).
 * adrp_race_command args: ADRP_CMD_ARGS float64 per drone.  Slots 0..12 hold the command's own
 * arguments, flattened in the reference's order; slot 13 holds the reference's args[-1], which
 * low_level_control hands to process_command_queue as the commander clock (MellingerControl.py:57,
 * 292-303) — for FULLSTATE that is its timestep, for TAKEOFF [h, d] it is d. */
#define ADRP_CMD_NONE 0         /* ignored (low_level_control: else -> continue) */
#define ADRP_CMD_FULLSTATE 1    /* pos[3], vel[3], acc[3], yaw, rpy_rate[3]            (491-543) */
#define ADRP_CMD_TAKEOFF 2      /* height, duration                                    (547-561) */
#define ADRP_CMD_TAKEOFFYAW 3   /* height, duration, yaw                               (565-580) */
#define ADRP_CMD_TAKEOFFVEL 4   /* height, velocity, relative                          (584-599) */
#define ADRP_CMD_LAND 5         /* height, duration                                    (603-617) */
#define ADRP_CMD_LANDYAW 6      /* height, duration, yaw                               (621-636) */
#define ADRP_CMD_LANDVEL 7      /* height, velocity, relative                          (640-655) */
#define ADRP_CMD_STOP 8         /* -                                                   (659-668) */
#define ADRP_CMD_GOTO 9         /* x, y, z, yaw, duration, relative                    (672-689) */
#define ADRP_CMD_NOTIFY 10      /* - (notifySetpointStop)                              (691-699) */
#define ADRP_CMD_ARGS 14
#define ADRP_CMD_TIME_SLOT 13
/* Per-drone command state (adrp_get_command_state), float fields then int32 fields, each a
 * contiguous [E*N] vector like adrp_get_state's.  Floats: setpoint_t position 3, velocity 3,
 * acceleration 3, attitudeRate 3 [deg/s], attitudeQuaternion z, w (FULLSTATE), attitude.yaw [deg]
 * (commander); the commander's pos 3, vel 3, yaw [rad]; state_t position 3, velocity 3,
 * attitude.yaw [deg] of the last _update_state; planner t_begin, duration, 4 x 8 polynomial
 * coefficients (x, y, z, yaw).  Ints: planner state (0 idle, 1 flying, 2 landing),
 * full_state_cmd_override, setpoint mode (0 never set, 1 FULLSTATE, 2 commander). */
#define ADRP_CMD_NF 63
#define ADRP_CMD_NI 3

/* Drone constants, as BaseAviary._parseURDFParameters reads them (BaseAviary.py:989-1021). */
typedef struct adrp_drone_params {
    double m;                  /* base mass [kg] */
    double l;                  /* arm [m] */
    double thrust2weight;
    double ixx, iyy, izz;      /* diagonal inertia [kg m^2] */
    double kf, km;             /* thrust / torque coefficients */
    double collision_h, collision_r, collision_z_offset;
    double max_speed_kmh;
    double gnd_eff_coeff, prop_radius;
    double drag_coeff[3];      /* xy, xy, z */
    double dw_coeff[3];
    double prop_pos[4][3];     /* prop link COM in the body frame (URDF inertial origins) */
} adrp_drone_params;

/* MultiRace track / randomisation description: the YAML schema of config/level*.yaml. */
typedef struct adrp_track {
    int32_t num_gates;                               /* <= ADRP_MAX_GATES */
    int32_t num_obstacles;                           /* <= ADRP_MAX_OBSTACLES */
    double gates[ADRP_MAX_GATES][7];                 /* nominal x,y,z,r,p,y,type(0 tall,1 low) */
    double obstacles[ADRP_MAX_OBSTACLES][6];         /* nominal x,y,z,r,p,y */
    double bounds_hi[3];                             /* |pos| > bounds[1] eliminates (MultiRaceAviary.py:684) */
    double episode_len_sec;
    int32_t random_gates_obstacles;
    double gate_offset_range[2];                     /* U(lo,hi) on x,y,yaw */
    double obstacle_offset_range[2];                 /* U(lo,hi) on x,y */
    int32_t random_drone_state;
    double pos_offset_range[3][2];                   /* U ranges x,y,z */
    double rot_offset_range[3][2];                   /* U ranges r,p,y */
    int32_t random_drone_inertia;
    double inertia_offset_range[4][2];               /* U ranges on M, Ixx, Iyy, Izz */
    int32_t disturbances;
    double action_noise_std;                         /* N(0,std) thrust noise per motor per sub-step */
    double dyn_dist_low[3], dyn_dist_high[3];        /* U(low,high) world force per drone per sub-step */
    double init_pos[ADRP_MAX_DRONES][3];             /* config init_states.droneK.pos */
    double init_vel[ADRP_MAX_DRONES][3];
    double init_rpy[ADRP_MAX_DRONES][3];             /* raw config value */
    double init_pqr[ADRP_MAX_DRONES][3];
    double race_mass;                                /* cf2x.urdf base mass used by changeDynamics (0.027) */
    double race_inertia[3];
    int32_t reward_wrapper;                          /* 0: env reward (0, MultiRaceAviary.py:665-670);
                                                        1: RewardWrapper (utils/wrapper.py:121-186) */
    int32_t obs_wrapper;                             /* DroneObservationWrapper (utils/wrapper.py:38-65):
                                                        yaw actions forced to 0, terminated once drone 0's
                                                        current gate >= 2.  0: off; 1: inside the
                                                        RewardWrapper (its terminal terms see the early
                                                        termination); 2: outside it */
} adrp_track;

typedef struct adrp_config {
    uint32_t struct_size;      /* = sizeof(adrp_config); checked by adrp_create */
    int32_t task;              /* ADRP_TASK_* */
    int32_t physics;           /* ADRP_PHYS_* */
    int32_t act_type;          /* ADRP_ACT_* */
    int32_t race_mode;         /* ADRP_RACE_* */
    int32_t num_envs;          /* E (envs on THIS device) */
    int32_t num_drones;        /* N drones per env */
    int32_t pyb_freq;          /* physics Hz (must be a multiple of ctrl_freq) */
    int32_t ctrl_freq;         /* env.step Hz */
    int32_t action_buffer_size;/* HoverAviary obs action ring (ctrl_freq//2, BaseRLAviary.py:66) */
    int32_t autoreset;         /* 1: done envs are reset inside adrp_step (VecEnv semantics) */
    int32_t precision;         /* 0 = fp32 kernel, 1 = fp64 kernel */
    int32_t link_frame_lag;    /* 1 (pybullet): LINK_FRAME forces/torques on links are rotated by the
                                  link transform cached at the last forwardKinematics, i.e. the pose
                                  at the start of the previous stepSimulation */
    int64_t env_offset;        /* global id of local env 0 (RNG key; multi-GPU sharding) */
    uint64_t seed;
    double gravity;            /* G = 9.8 (BaseAviary.py:74) */
    adrp_drone_params drone;
    /* HoverAviary */
    double init_xyz[ADRP_MAX_DRONES][3];   /* INIT_XYZS (BaseAviary.py:194-199) */
    double init_rpy[ADRP_MAX_DRONES][3];   /* INIT_RPYS [rad] */
    double init_xyz_noise[3];              /* extension: U(-n,n) added per reset (0 = reference) */
    double init_rpy_noise[3];
    double init_vel_noise[3];
    double init_omega_noise[3];
    double target_pos[3];                  /* HoverAviary.TARGET_POS (HoverAviary.py:51) */
    double episode_len_sec;                /* HoverAviary.EPISODE_LEN_SEC (HoverAviary.py:52) */
    /* MultiRaceAviary */
    adrp_track track;
} adrp_config;

typedef struct adrp_handle adrp_t;

/* ABI version of the loaded library (must equal ADRP_ABI_VERSION). */
int adrp_abi_version(void);

/* Fill *cfg with the reference defaults for `task` (HoverAviary or MultiRaceAviary,
 * CF2X = cf2x_IROS.urdf constants, level0 track for RACE). */
int adrp_default_config(int task, adrp_config* cfg);

/* Create a handle on GPU `device`; allocates all state in HBM. */
int adrp_create(const adrp_config* cfg, int device, adrp_t** out);
void adrp_destroy(adrp_t* h);

/* Error text of the last failing call on h (h may be NULL for adrp_create failures). */
const char* adrp_last_error(const adrp_t* h);

/* Per-drone observation width D (12 + B*A for Hover: 72 RPM/VEL, 57 PID, 27 ONE_D_*;
 * 49 / 49+6(N-1) Race) and action width A (4, 3 or 1). */
int adrp_obs_dim(const adrp_t* h);
int adrp_act_dim(const adrp_t* h);

/* Re-key the handle's random streams (reset randomisation, level1-3 disturbances) as a fresh
 * handle created with `seed` has them: sets the seed and zeroes every env's episode counter
 * (stream-ordered).  Follow it with a full adrp_reset, as BaseAviary.reset(seed=...) reseeds and
 * resets (envs/BaseAviary.py:223-258).  A captured graph keeps the seed it was captured with. */
int adrp_reseed(adrp_t* h, uint64_t seed, void* stream);

/* MultiRaceAviary only: switch the RewardWrapper / DroneObservationWrapper fused into the step
 * (adrp_track.reward_wrapper / .obs_wrapper) on an existing handle, as wrapping the reference env
 * with RewardWrapper(env) / DroneObservationWrapper(env) does (utils/wrapper.py).  Synchronises. */
int adrp_set_wrappers(adrp_t* h, int reward_wrapper, int obs_wrapper);

/* Reset the envs selected by env_mask_dev (uint8 [E], NULL = all) and write their
 * observations into obs_dev (float [E,N,D]); rows of unselected envs are left as is. */
int adrp_reset(adrp_t* h, const uint8_t* env_mask_dev, float* obs_dev, void* stream);

/* One env.step() of every env: act_dev float [E,N,A] -> obs_dev [E,N,D],
 * rew_dev float [E], term_dev / trunc_dev uint8 [E].  With autoreset, envs whose
 * episode ended are reset in the same launch; their final observation is written to
 * terminal_obs_dev [E,N,D] (only those rows) when it is non-NULL, and obs_dev holds
 * the reset observation (SB3 VecEnv semantics). */
int adrp_step(adrp_t* h, const float* act_dev, float* obs_dev, float* rew_dev,
              uint8_t* term_dev, uint8_t* trunc_dev, float* terminal_obs_dev, void* stream);

/* MultiRaceAviary only: high-level command mode.  adrp_enable_commands
 * allocates the per-drone setpoint / commander / planner state; call it before the adrp_reset that
 * starts the episodes (envs already running start from an idle planner and an unset setpoint).
 * From then on adrp_step runs the step kernel that evaluates the commander's trajectory at every
 * controller call (MellingerControl._update_setpoint, MellingerControl.py:369-374).
 * adrp_race_command applies one command per drone (cmd_dev int32 [E,N] ADRP_CMD_*, args_dev float64
 * [E,N,ADRP_CMD_ARGS]) as the controller processes MultiRaceAviary.step's command message before the
 * sub-steps; eliminated drones get STOP (MultiRaceAviary.py:198-199).  Follow it with
 * adrp_step(h, NULL, ...), which keeps the setpoints the commands left.  adrp_step with a non-NULL
 * act_dev sends FULLSTATE (act[:3], 0, 0, act[3], 0, step_counter) first, as the ndarray path does
 * (MultiRaceAviary.py:190-194).  Parity of the commander is unpinned. */
int adrp_enable_commands(adrp_t* h);
int adrp_race_command(adrp_t* h, const int32_t* cmd_dev, const double* args_dev, void* stream);
/* float [ADRP_CMD_NF][E*N] (float32 at every precision), int32 [ADRP_CMD_NI][E*N] */
int adrp_get_command_state(adrp_t* h, float* f_dev, int32_t* i_dev, void* stream);
int adrp_set_command_state(adrp_t* h, const float* f_dev, const int32_t* i_dev, void* stream);

/* Snapshot layout: nf float fields and ni int32 fields, each field a contiguous
 * [E*N] vector (drone-major within env: index e*N+n).  Field names: adrp_state_field. */
int adrp_state_layout(const adrp_t* h, int* nf, int* ni);
const char* adrp_state_field(const adrp_t* h, int is_int, int index);
/* f_dev elements are float32 for precision 0 and float64 for precision 1. */
int adrp_get_state(adrp_t* h, void* f_dev, int32_t* i_dev, void* stream);
int adrp_set_state(adrp_t* h, const void* f_dev, const int32_t* i_dev, void* stream);

/* Name of the step-kernel instantiation a config selects (no device needed), e.g.
 * "hover_step<f32,PYB,A4,B15,cf2x>": "cf2x" = per-config constants compiled in (the
 * reference default drone at 240/30 Hz, chosen only when the config's derived constants
 * are bit-identical), "generic" = read from the handle's device-resident block. */
const char* adrp_kernel_name(const adrp_config* cfg);
/* the instantiation this handle launches now (after adrp_enable_commands a race handle runs the
   command-mode kernel, "...,CMD>"; ADRP_RACE_QUAD as read at create) */
const char* adrp_handle_kernel_name(const adrp_t* h);

/* Algorithmic HBM bytes one adrp_step moves (roofline accounting). */
int64_t adrp_step_bytes(const adrp_t* h);

/* Kernel timing with HIP events attached to the step kernel's own dispatch
 * (hipExtLaunchKernelGGL start/stop events): after adrp_profile_begin(h, n) the next n
 * adrp_step launches are timed; adrp_profile_end synchronises and writes up to `cap`
 * kernel durations [ms] to kernel_ms (host memory), returning how many were written. */
int adrp_profile_begin(adrp_t* h, int max_launches);
int adrp_profile_end(adrp_t* h, float* kernel_ms, int cap);

/* ---------------------------------------------------------------------------------------
 * Persistent step (HoverAviary, RPM / ONE_D_RPM actions, E <= 1024): BASELINE config 1, the
 * reference's one-env loop (examples/pid.py:101-147 calling BaseAviary.step, envs/BaseAviary.py:
 * 262-387) with no kernel launch per step.  begin launches one resident kernel (a workgroup per 64
 * envs) on its own stream and returns HOST pointers into a host-mapped mailbox: act [E][A] float,
 * obs [E][D] float, reward [E] float, terminated / truncated [E] uint8, terminal obs [E][D] float
 * (auto-reset envs).  step: the caller writes act, calls adrp_persistent_step, which returns when
 * the env.step is done and the outputs are in the mailbox (same results as adrp_step on the same
 * state).  While active, adrp_step / adrp_reset / adrp_get_state / adrp_set_state are refused.
 * end stops the kernel (destroy ends it too); the kernel also ends by itself after 10 s without a
 * request, after which step fails and end + begin restart it. */
int adrp_persistent_begin(adrp_t* h, void** act, void** obs, void** reward, void** terminated, void** truncated,
                          void** terminal_obs);
int adrp_persistent_step(adrp_t* h);
int adrp_persistent_end(adrp_t* h);

/* Diagnostics (off by default, costs a same-address atomic per touching wave):
 * count env-steps whose sub-steps touched the plane contact model. */
int adrp_set_diagnostics(adrp_t* h, int enable);
int adrp_diagnostic_contact_count(adrp_t* h, int reset);
/* Race handles: with diagnostics on, each env.step also records per drone a hash of the int16
 * (roll, pitch, yaw) moments of every firmware controllerMellinger call of the step, in call order
 * (FNV-1a over the int32 values, seed 2166136261, prime 16777619; oracle/race.c computes the same).
 * Parity tests use it as the causal witness of an int16 truncation difference.  Copies E * N values
 * of the last step to `out` (host memory); n must be E * N.  Replaces nothing in the reference. */
int adrp_race_moment_hash(adrp_t* h, uint32_t* out, size_t n);
/* Race handles, diagnostics level 2 (adrp_set_diagnostics(h, 2); the step then runs the one-lane
 * kernel): each env.step also records per drone the int16 (roll, pitch, yaw) of every firmware
 * controllerMellinger call, in call order (MellingerControl.py:413-415: control_t's moments).
 * Copies them to `out` [E*N][max_calls][3] and the number of calls to `counts` [E*N] (host memory);
 * n must be E * N and max_calls the sub-steps per env.step.  The oracle replays them
 * (oracle/race.c orc_race_set_moment_replay) to show that a drone whose truncation differs agrees
 * once the same integers are used.  Replaces nothing in the reference. */
int adrp_race_moment_log(adrp_t* h, int16_t* out, int32_t* counts, size_t n, int max_calls);
/* Race handles, diagnostics on: auto-resets of the four-lane kernel since the last read, out[0]
 * copied from a next-reset image (computed ahead by the refill launch every ADRP_RESET_IMAGES
 * steps, default 32, 0 = off), out[1] computed inline.  Replaces nothing in the reference. */
int adrp_race_reset_counts(adrp_t* h, int32_t* out, int reset);

/* ---------------------------------------------------------------------------------------
 * On-device policy forward: the actor of an SB3 PPO MlpPolicy
 * (in_dim -> hidden1 -> hidden2 -> 4, Tanh or ReLU) + the RLController action transform,
 * on f32 MFMA.  Replaces, batched, RLController.predict / _action_transform
 * (user_controller/RLController.py:39-73, RLControllerTwoGates.py:38-69) over
 * PPO.predict(obs, deterministic=True) (stable_baselines3 2.3.2: mlp_extractor.policy_net,
 * action_net, clip to the [-1, 1] Box).  Weights are host float32 arrays in torch Linear
 * layout ([out][in] row-major): the policy.pth tensors mlp_extractor.policy_net.{0,2}.* and
 * action_net.*.  obs rows are the first in_dim floats of each obs_stride-wide row (e.g.
 * adrp_step's obs_dev with rows = E*N); act_dev receives float [rows][4].
 * --------------------------------------------------------------------------------------- */
#define ADRP_POLICY_TANH 0          /* SB3 MlpPolicy default activation_fn (nn.Tanh) */
#define ADRP_POLICY_RELU 1          /* policy_kwargs activation_fn=nn.ReLU (twogates.zip) */
#define ADRP_POLICY_RAW 0           /* act = clip(mean, -1, 1) */
#define ADRP_POLICY_RELATIVE 1      /* RLController: a[3]=0; obs[[0,1,2,5]] + a*[1,1,1,pi], yaw map2pi */
#define ADRP_POLICY_ABSOLUTE 2      /* RLControllerTwoGates: a[3]=0; a*[1,1,1,pi], yaw map2pi */

typedef struct adrp_policy adrp_policy_t;

/* hidden1, hidden2 in {16, 32, 64, 128}; in_dim 1..64 */
int adrp_policy_create(int device, int in_dim, int hidden1, int hidden2, int activation,
                       const float* w1, const float* b1, const float* w2, const float* b2,
                       const float* w3, const float* b3, adrp_policy_t** out);
int adrp_policy_act(adrp_policy_t* p, const float* obs_dev, int rows, int obs_stride, int mode,
                    float* act_dev, void* stream);
void adrp_policy_destroy(adrp_policy_t* p);
/* act_dim 1..4 (HoverAviary ONE_D_RPM policies: 1); adrp_policy_act needs 4, adrp_policy_sample any */
int adrp_policy_create2(int device, int in_dim, int hidden1, int hidden2, int act_dim, int activation,
                        const float* w1, const float* b1, const float* w2, const float* b2,
                        const float* w3, const float* b3, adrp_policy_t** out);

/* ---------------------------------------------------------------------------------------
 * On-device PPO rollout step (examples/learn.py:72-94 trains PPO): what SB3's
 * OnPolicyAlgorithm.collect_rollouts does per step, `actions, values, log_probs = policy(obs)`
 * with ActorCriticPolicy.forward(obs, deterministic=False) (stable_baselines3 2.3.2): the actor
 * mean (as adrp_policy_act), the critic mlp_extractor.value_net (in_dim -> hidden1 -> hidden2, the
 * same activation) + value_net (-> 1), a DiagGaussianDistribution sample a = mean +
 * exp(log_std) eps and log_prob = sum_i Normal(mean_i, std_i).log_prob(a_i).  eps ~ N(0, 1): one
 * Philox4x32-10 block per row, counter {row, counter, 0x504f4c00, 0} keyed by seed, Box-Muller of
 * its word pairs (the race action noise's IEEE float form).  Replaces, batched on the device,
 * policy(obs_tensor) inside collect_rollouts plus the np.clip of the actions it sends the env.
 * adrp_policy_set_critic: value_net.{0,2}.* / value_net.* in torch layout and log_std [act_dim].
 * adrp_policy_sample: action_dev [rows][act_dim] (the sample, what the rollout buffer stores),
 * env_act_dev (clip to [-1, 1], then the mode transform; [rows][act_dim], RELATIVE / ABSOLUTE
 * [rows][4]), value_dev [rows], logprob_dev [rows], eps_dev [rows][act_dim] or NULL.
 * --------------------------------------------------------------------------------------- */
int adrp_policy_set_critic(adrp_policy_t* p, const float* vw1, const float* vb1, const float* vw2,
                           const float* vb2, const float* vw3, const float* vb3, const float* log_std);
int adrp_policy_sample(adrp_policy_t* p, const float* obs_dev, int rows, int obs_stride, int mode,
                       uint64_t seed, uint32_t counter, float* env_act_dev, float* action_dev,
                       float* value_dev, float* logprob_dev, float* eps_dev, void* stream);

/* GAE over a rollout (SB3 RolloutBuffer.compute_returns_and_advantage, stable_baselines3 2.3.2):
 * rewards / values / episode_starts [n_steps][n_envs] float32 on the device, last_values /
 * dones [n_envs]; writes advantages and returns [n_steps][n_envs] (returns = advantages + values).
 * One lane per env runs the backward recursion. */
int adrp_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
             const float* dones, int n_steps, int n_envs, double gamma, double gae_lambda, float* advantages,
             float* returns, void* stream);

/* SB3 VecEnv host path: the terminal observations of the finished envs, compacted on the device
 * behind the step's packed outputs so ONE device -> host copy returns them (replaces the per-env
 * infos[e]["terminal_observation"] = obs that stable_baselines3 DummyVecEnv.step_wait fills from
 * its sub-envs, vec_env/dummy_vec_env.py, 2.3.2).  term / trunc [n] uint8, rows [n][row_floats]
 * (the env's terminal-obs buffer); writes count[0] = number of envs with term | trunc, idx[j] = the
 * j-th such env (ascending, j < count, so idx holds up to n entries) and out_rows[j] = rows[idx[j]]
 * for j < min(count, cap).  One workgroup; stream-ordered after the step. */
int adrp_compact_rows(const uint8_t* term, const uint8_t* trunc, const float* rows, int n, int row_floats,
                      int cap, int32_t* count, int32_t* idx, float* out_rows, void* stream);
/* The same host path's copies (kind 1: host -> device, 2: device -> host; pinned host memory makes
 * them asynchronous on the stream) and its one wait, without a framework dispatch in between. */
int adrp_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream);
int adrp_stream_synchronize(void* stream);

/* SB3 VecEnv host path in ONE call per step (vec_env.py AviaryVecEnv; replaces what
 * stable_baselines3 DummyVecEnv.step_async / step_wait do around the reference's env.step,
 * examples/learn.py:53-57, 72): the step kernel reads the actions from, and writes obs / reward
 * straight into, pinned host memory (device-mapped: no copy engine on the path), a compaction
 * writes the terminated / truncated / done flags, the finished envs' count and ids and their
 * terminal rows into the same host block, and the host waits once.  A handle holds
 * ADRP_VEC_SLOTS such host blocks (a ring: the caller's views of slot k stay valid until slot k is
 * stepped again); adrp_vec_bind records one (host pointers of hipHostMalloc'd / pinned memory,
 * translated to device addresses here), adrp_vec_step(h, k, stream) steps into it.  term_dev /
 * trunc_dev / tobs_dev / idx_dev are the caller's device buffers ([E] u8, [E] u8, [E][N][D] f32,
 * [E] i32): the step's own flags and terminal obs, the compaction's scratch.  Rows beyond cap are
 * left in tobs_dev (count says how many envs finished).  Stream-ordered; returns after the wait. */
#define ADRP_VEC_SLOTS 4
typedef struct adrp_vec_io {
    const float* act;            /* host [E][N][A] float32 (read by the step kernel) */
    float* obs;                  /* host [E][N][D] */
    float* rew;                  /* host [E] */
    uint8_t* term;               /* host [E] terminated */
    uint8_t* trunc;              /* host [E] truncated */
    uint8_t* done;               /* host [E] terminated | truncated */
    int32_t* count;              /* host [1] finished envs */
    int32_t* idx;                /* host [E] their ids, ascending */
    float* rows;                 /* host [cap][N*D] their terminal rows */
    int cap;
    uint8_t* term_dev;
    uint8_t* trunc_dev;
    float* tobs_dev;
    int32_t* idx_dev;
} adrp_vec_io;
int adrp_vec_bind(adrp_t* h, int slot, const adrp_vec_io* io);
int adrp_vec_step(adrp_t* h, int slot, void* stream);

/* ---------------------------------------------------------------------------------------
 * Parity mode noise (MultiRaceAviary).  The reference draws, per sub-step, the disturbance force
 * of every drone (np_random.<distrib>(low, high), MultiRaceAviary.py:532-537) and then the (N, 4)
 * action noise (np_random.<distrib>(0, std, (N, 4)), :223-228).  After adrp_set_noise the race
 * step takes them from these caller-owned DEVICE arrays instead of its Philox streams:
 *   act_noise_dev [E*N][S][4], force_dev [E*N][S][3] float64, drone slot e*N + n, sub-step s of
 *   the NEXT adrp_step (S = pyb_freq / ctrl_freq); the caller refills them (stream-ordered)
 *   before every step.  The pointers are kept until adrp_set_noise(h, NULL, NULL).  Only used when
 *   the track has disturbances on.  Replaces: nothing in the reference's API (its RNG is internal);
 *   lets a noisy reference step be replayed with the reference's own draws.
 * --------------------------------------------------------------------------------------- */
int adrp_set_noise(adrp_t* h, const double* act_noise_dev, const double* force_dev);

/* ---------------------------------------------------------------------------------------
 * Numerics probe (no reference counterpart: test support).  Evaluates one of the fp64
 * fast transcendentals the fp64 step kernels inline (csrc/adrp_device.h namespace f64:
 * refined v_rcp_f64 / v_rsq_f64, range-reduced polynomials) on n device doubles:
 * out[i] = f(in[i]); ATAN2 reads y = in[i], x = in[n + i], DIVC x = in[i], c = in[n + i].
 * Stream-ordered.
 * --------------------------------------------------------------------------------------- */
#define ADRP_MATH_RCP 0
#define ADRP_MATH_RSQ 1
#define ADRP_MATH_SQRT 2
#define ADRP_MATH_SIN_SMALL 3      /* |x| <= pi/8 */
#define ADRP_MATH_COS_SMALL 4      /* |x| <= pi/8 */
#define ADRP_MATH_ATAN2 5
#define ADRP_MATH_ASIN 6           /* |x| < 1 */
#define ADRP_MATH_EXP 7            /* x <= 0 in the kernels */
#define ADRP_MATH_SQRT_NN 8        /* sums of squares: x >= 0 or NaN (Bullet step norms) */
#define ADRP_MATH_RCP_NC 9         /* finite, non-zero x (no non-finite fix-up) */
#define ADRP_MATH_RSQ_NC 10        /* finite, positive x (quaternion norm) */
#define ADRP_MATH_SIN_TINY 11      /* |x| <= 0.03 (exp-map half angle) */
#define ADRP_MATH_COS_TINY 12      /* |x| <= 0.03 */
#define ADRP_MATH_EXPMAP_SINC 13   /* sin(x)/x of the hover exp map (per-lane series choice) */
#define ADRP_MATH_EXPMAP_COS 14    /* cos(x) of the hover exp map */
#define ADRP_MATH_QUAT_INV_NORM 15 /* 1/sqrt(n2) of the hover exp-map quaternion (per-lane form) */
#define ADRP_MATH_NORMAL_Z0 16     /* race action-noise Box-Muller of a Philox word pair: in[i]'s bits */
#define ADRP_MATH_NORMAL_Z1 17     /*   = x1 << 32 | x0; out = z0 / z1 (float samples, as doubles) */
#define ADRP_MATH_DIVC 18          /* in[i] / in[n + i] by the fp64 kernels' constant-divisor form */
#define ADRP_MATH_SIN_FAST 19      /* octant-reduced sin / cos (gate yaws, reset attitudes) */
#define ADRP_MATH_COS_FAST 20
#define ADRP_MATH_EXP_TAB 21       /* exp(x), x <= 0, table form of the fp64 race downwash */
#define ADRP_MATH_ATAN2_NC 22      /* atan2(in[i], in[n + i]) for finite operands (race Euler angles) */
#define ADRP_MATH_FDIV_RCP 23      /* float(in[i]) / float(in[n + i]) as the fp64 race firmware divides (f64::fdiv_rcp) */
int adrp_math_probe(int fn, const double* in_dev, double* out_dev, int n, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADRP_H */
