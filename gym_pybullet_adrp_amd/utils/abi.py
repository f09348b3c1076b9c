"""ctypes mirror of include/adrp.h (struct layouts and constants).

Must stay byte-identical with the header: tests/test_abi.py checks sizeof() against the
value adrp_default_config() writes into ``struct_size``.
"""
import ctypes

ABI_VERSION = 2
MAX_DRONES = 8
MAX_GATES = 4
MAX_OBSTACLES = 4

OK, ERR_INVALID, ERR_DEVICE, ERR_OOM = 0, -1, -2, -3

TASK_HOVER, TASK_RACE = 0, 1
PHYS_PYB, PHYS_DYN, PHYS_PYB_GND, PHYS_PYB_DRAG, PHYS_PYB_DW, PHYS_PYB_GND_DRAG_DW = range(6)
ACT_RPM, ACT_ONE_D_RPM, ACT_FULLSTATE, ACT_PID, ACT_VEL, ACT_ONE_D_PID = 0, 1, 2, 3, 4, 5
MATH_RCP, MATH_RSQ, MATH_SQRT, MATH_SIN_SMALL, MATH_COS_SMALL, MATH_ATAN2, MATH_ASIN, MATH_EXP = range(8)   # adrp_math_probe
MATH_SQRT_NN, MATH_RCP_NC, MATH_RSQ_NC, MATH_SIN_TINY, MATH_COS_TINY = 8, 9, 10, 11, 12
MATH_EXPMAP_SINC, MATH_EXPMAP_COS, MATH_QUAT_INV_NORM, MATH_NORMAL_Z0, MATH_NORMAL_Z1 = 13, 14, 15, 16, 17
MATH_DIVC, MATH_SIN_FAST, MATH_COS_FAST = 18, 19, 20
MATH_EXP_TAB, MATH_ATAN2_NC, MATH_FDIV_RCP = 21, 22, 23
RACE_COMPARE, RACE_COMPETE = 0, 1
POLICY_TANH, POLICY_RELU = 0, 1
POLICY_RAW, POLICY_RELATIVE, POLICY_ABSOLUTE = 0, 1, 2
VEC_SLOTS = 4   # ADRP_VEC_SLOTS

_d = ctypes.c_double
_i32 = ctypes.c_int32


def _arr(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class AdrpDroneParams(ctypes.Structure):
    _fields_ = [
        ("m", _d), ("l", _d), ("thrust2weight", _d),
        ("ixx", _d), ("iyy", _d), ("izz", _d),
        ("kf", _d), ("km", _d),
        ("collision_h", _d), ("collision_r", _d), ("collision_z_offset", _d),
        ("max_speed_kmh", _d),
        ("gnd_eff_coeff", _d), ("prop_radius", _d),
        ("drag_coeff", _arr(_d, 3)),
        ("dw_coeff", _arr(_d, 3)),
        ("prop_pos", _arr(_d, 4, 3)),
    ]


class AdrpTrack(ctypes.Structure):
    _fields_ = [
        ("num_gates", _i32), ("num_obstacles", _i32),
        ("gates", _arr(_d, MAX_GATES, 7)),
        ("obstacles", _arr(_d, MAX_OBSTACLES, 6)),
        ("bounds_hi", _arr(_d, 3)),
        ("episode_len_sec", _d),
        ("random_gates_obstacles", _i32),
        ("gate_offset_range", _arr(_d, 2)),
        ("obstacle_offset_range", _arr(_d, 2)),
        ("random_drone_state", _i32),
        ("pos_offset_range", _arr(_d, 3, 2)),
        ("rot_offset_range", _arr(_d, 3, 2)),
        ("random_drone_inertia", _i32),
        ("inertia_offset_range", _arr(_d, 4, 2)),
        ("disturbances", _i32),
        ("action_noise_std", _d),
        ("dyn_dist_low", _arr(_d, 3)), ("dyn_dist_high", _arr(_d, 3)),
        ("init_pos", _arr(_d, MAX_DRONES, 3)),
        ("init_vel", _arr(_d, MAX_DRONES, 3)),
        ("init_rpy", _arr(_d, MAX_DRONES, 3)),
        ("init_pqr", _arr(_d, MAX_DRONES, 3)),
        ("race_mass", _d),
        ("race_inertia", _arr(_d, 3)),
        ("reward_wrapper", _i32),
        ("obs_wrapper", _i32),
    ]


class AdrpConfig(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("task", _i32), ("physics", _i32), ("act_type", _i32), ("race_mode", _i32),
        ("num_envs", _i32), ("num_drones", _i32),
        ("pyb_freq", _i32), ("ctrl_freq", _i32),
        ("action_buffer_size", _i32),
        ("autoreset", _i32),
        ("precision", _i32),
        ("link_frame_lag", _i32),
        ("env_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("gravity", _d),
        ("drone", AdrpDroneParams),
        ("init_xyz", _arr(_d, MAX_DRONES, 3)),
        ("init_rpy", _arr(_d, MAX_DRONES, 3)),
        ("init_xyz_noise", _arr(_d, 3)),
        ("init_rpy_noise", _arr(_d, 3)),
        ("init_vel_noise", _arr(_d, 3)),
        ("init_omega_noise", _arr(_d, 3)),
        ("target_pos", _arr(_d, 3)),
        ("episode_len_sec", _d),
        ("track", AdrpTrack),
    ]

    def copy(self):
        c = AdrpConfig()
        ctypes.memmove(ctypes.byref(c), ctypes.byref(self), ctypes.sizeof(self))
        return c


def set_vec(arr, values):
    """Assign a (nested) python sequence into a ctypes array in place."""
    for k, v in enumerate(values):
        if hasattr(arr[k], "__len__") and not isinstance(arr[k], (int, float)):
            set_vec(arr[k], v)
        else:
            arr[k] = v


def to_list(arr):
    out = []
    for x in arr:
        out.append(to_list(x) if hasattr(x, "__len__") else x)
    return out


class AdrpVecIO(ctypes.Structure):
    """adrp_vec_io (include/adrp.h): one host block of the SB3 host path (adrp_vec_bind)"""
    _p = ctypes.c_void_p
    _fields_ = [("act", _p), ("obs", _p), ("rew", _p), ("term", _p), ("trunc", _p), ("done", _p),
                ("count", _p), ("idx", _p), ("rows", _p), ("cap", ctypes.c_int),
                ("term_dev", _p), ("trunc_dev", _p), ("tobs_dev", _p), ("idx_dev", _p)]
