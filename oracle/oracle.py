"""ctypes binding of the CPU oracle (oracle/oracle.c) — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
product package (gym_pybullet_adrp_amd) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build(force=False):
    src = os.path.join(HERE, "oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(HERE, "race.c")),
            os.path.getmtime(os.path.join(HERE, "oracle.h")),
            os.path.getmtime(os.path.join(HERE, "..", "include", "adrp.h"))):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


def _load():
    build()
    lib = ctypes.CDLL(LIB)
    P, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.orc_create.argtypes = [P, ctypes.POINTER(P)]
    lib.orc_create.restype = I
    lib.orc_destroy.argtypes = [P]
    lib.orc_last_error.restype = ctypes.c_char_p
    for f in ("orc_obs_dim", "orc_act_dim"):
        getattr(lib, f).argtypes = [P]
        getattr(lib, f).restype = I
    lib.orc_reset.argtypes = [P, P, P]
    lib.orc_step.argtypes = [P, P, P, P, P, P, P]
    lib.orc_state_layout.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I)]
    lib.orc_state_field.argtypes = [P, I, I]
    lib.orc_state_field.restype = ctypes.c_char_p
    lib.orc_get_state.argtypes = [P, P, P]
    lib.orc_set_state.argtypes = [P, P, P]
    lib.orc_contact_count.argtypes = [P]
    lib.orc_contact_count.restype = ctypes.c_int64
    lib.orc_env_contact.argtypes = [P, I]
    lib.orc_env_contact.restype = ctypes.c_uint8
    lib.orc_default_config.argtypes = [I, P]
    lib.orc_set_bullet_variant.argtypes = [I]
    lib.orc_obs_wrapper_term.argtypes = [I, I, I, P, P]
    lib.orc_set_threads.argtypes = [I]
    lib.orc_get_threads.restype = I
    lib.orc_philox4x32_10.argtypes = [P, P, P]
    lib.orc_euler_from_quat.argtypes = [P, P]
    lib.orc_quat_from_euler.argtypes = [P, P]
    lib.orc_derived_constants.argtypes = [P, P]
    lib.orc_force_assembly.argtypes = [P, I, P, I, P, P, P, P]
    lib.orc_hover_rpm.argtypes = [P, P, P]
    lib.orc_dslpid.argtypes = [P, D, P, P, P]
    lib.orc_hover_eval.argtypes = [P, P, P, P, P]
    lib.orc_config_size.restype = ctypes.c_uint32
    lib.orc_compute_pwms.argtypes = [P, P]
    lib.orc_pwms_to_rpms.argtypes = [P, P, P]
    lib.orc_tick_schedule.argtypes = [I, P]
    lib.orc_race_body_distance.argtypes = [P, P, P, I, I, P]
    lib.orc_race_body_distance.restype = D
    lib.orc_shape_distance.argtypes = [P, P]
    lib.orc_shape_distance.restype = D
    lib.orc_lpf_coeffs.argtypes = [D, D, P]
    lib.orc_race_obs_assemble.argtypes = [P, I, I, P, P, P, P, P, I, P]
    lib.orc_race_terminated.argtypes = [P, I, P, P, P, P, P]
    lib.orc_race_truncated.argtypes = [P, I]
    lib.orc_race_rays.argtypes = [P, I, P, P]
    lib.orc_race_progress.argtypes = [I, I, P, P, P, P]
    lib.orc_race_reward.argtypes = [P, P, P, P, I, I]
    lib.orc_race_reward.restype = D
    lib.orc_race_command.argtypes = [P, P, P]
    lib.orc_set_noise.argtypes = [P, P, P]
    lib.orc_race_set_moment_replay.argtypes = [P, P, P]
    lib.orc_race_moment_margin.argtypes = [P, P]
    lib.orc_race_moment_hash.argtypes = [P, P]
    lib.orc_normal_pair.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P]
    lib.orc_get_command_state.argtypes = [P, P, P]
    lib.orc_set_command_state.argtypes = [P, P, P]
    lib.orc_poly4d_eval.argtypes = [P, ctypes.c_float, P]
    lib.orc_poly7_nojerk.argtypes = [ctypes.c_float] * 7 + [P]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    """Batched CPU restatement behind the same config struct as libadrp."""

    def __init__(self, cfg):
        from gym_pybullet_adrp_amd.utils.abi import AdrpConfig  # struct layout only
        assert isinstance(cfg, AdrpConfig)
        self.cfg = cfg
        h = ctypes.c_void_p()
        rc = lib().orc_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise ValueError(lib().orc_last_error().decode())
        self.h = h
        self.E, self.N = cfg.num_envs, cfg.num_drones
        self.S = cfg.pyb_freq // cfg.ctrl_freq     # sub-steps per env.step
        self.D = lib().orc_obs_dim(h)
        self.A = lib().orc_act_dim(h)
        nf, ni = ctypes.c_int(), ctypes.c_int()
        lib().orc_state_layout(h, ctypes.byref(nf), ctypes.byref(ni))
        self.nf, self.ni = nf.value, ni.value

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().orc_destroy(self.h)
                self.h = None
        except Exception:   # interpreter shutdown
            pass

    def field_names(self):
        return ([lib().orc_state_field(self.h, 0, k).decode() for k in range(self.nf)],
                [lib().orc_state_field(self.h, 1, k).decode() for k in range(self.ni)])

    def reset(self, mask=None):
        obs = np.zeros((self.E, self.N, self.D), np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        lib().orc_reset(self.h, _ptr(m), _ptr(obs))
        return obs

    def step(self, act):
        """act None: MultiRace command mode, the setpoints the last command() left."""
        if act is not None:
            act = np.ascontiguousarray(act, np.float32).reshape(self.E, self.N, self.A)
        obs = np.zeros((self.E, self.N, self.D), np.float32)
        tobs = np.zeros_like(obs)
        rew = np.zeros(self.E, np.float32)
        term = np.zeros(self.E, np.uint8)
        trunc = np.zeros(self.E, np.uint8)
        lib().orc_step(self.h, _ptr(act), _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc), _ptr(tobs))
        return obs, rew, term.astype(bool), trunc.astype(bool), tobs

    CMD_NF, CMD_NI, CMD_ARGS = 63, 3, 14

    def set_noise(self, act_noise=None, force=None):
        """parity mode (orc_set_noise): action noise [E, N, S, 4] and disturbance force [E, N, S, 3]
        of the next step's sub-steps, or None, None for the Philox draws"""
        if act_noise is None:
            self._noise = None
            assert lib().orc_set_noise(self.h, None, None) == 0
            return
        self._noise = (np.ascontiguousarray(act_noise, np.float64), np.ascontiguousarray(force, np.float64))
        assert lib().orc_set_noise(self.h, _ptr(self._noise[0]), _ptr(self._noise[1])) == 0

    def set_moment_replay(self, moments=None, counts=None):
        """diagnostics (orc_race_set_moment_replay): the next steps use these int16 firmware moments
        ([E*N][S][3], call order, counts [E*N]; the kernel's Handle.moment_log()) instead of their own
        truncation; None, None turns it off"""
        if moments is None:
            self._replay = None
            assert lib().orc_race_set_moment_replay(self.h, None, None) == 0
            return
        self._replay = (np.ascontiguousarray(moments, np.int16), np.ascontiguousarray(counts, np.int32))
        assert self._replay[0].shape == (self.E * self.N, self.S, 3)
        assert lib().orc_race_set_moment_replay(self.h, _ptr(self._replay[0]), _ptr(self._replay[1])) == 0

    def command(self, cmd, args):
        """One high-level command per drone: cmd int32 [E, N], args float64 [E, N, 14]."""
        c = np.ascontiguousarray(cmd, np.int32).reshape(self.E * self.N)
        a = np.ascontiguousarray(args, np.float64).reshape(self.E * self.N, self.CMD_ARGS)
        rc = lib().orc_race_command(self.h, _ptr(c), _ptr(a))
        assert rc == 0, lib().orc_last_error()

    def get_command_state(self):
        f = np.zeros((self.CMD_NF, self.E * self.N), np.float32)
        i = np.zeros((self.CMD_NI, self.E * self.N), np.int32)
        assert lib().orc_get_command_state(self.h, _ptr(f), _ptr(i)) == 0
        return f, i

    def set_command_state(self, f, i):
        f = np.ascontiguousarray(f, np.float32)
        i = np.ascontiguousarray(i, np.int32)
        assert f.shape == (self.CMD_NF, self.E * self.N) and i.shape == (self.CMD_NI, self.E * self.N)
        assert lib().orc_set_command_state(self.h, _ptr(f), _ptr(i)) == 0

    def get_state(self):
        f = np.zeros((self.nf, self.E * self.N), np.float64)
        i = np.zeros((self.ni, self.E * self.N), np.int32)
        lib().orc_get_state(self.h, _ptr(f), _ptr(i))
        return f, i

    def set_state(self, f, i):
        f = np.ascontiguousarray(f, np.float64)
        i = np.ascontiguousarray(i, np.int32)
        assert f.shape == (self.nf, self.E * self.N) and i.shape == (self.ni, self.E * self.N)
        lib().orc_set_state(self.h, _ptr(f), _ptr(i))

    def moment_margin(self):
        """[E*N] per drone slot: the smallest distance of a firmware moment (control_t roll / pitch / yaw
        before the int16 cast) to a truncation point (a nonzero integer) over the last env.step's
        firmware calls; inf if no call produced moments"""
        out = np.zeros(self.E * self.N, np.float32)
        assert lib().orc_race_moment_margin(self.h, _ptr(out)) == 0
        return out

    def moment_hash(self):
        """[E*N] uint32 per drone slot: the hash of the int16 (roll, pitch, yaw) moments of every
        firmware call of the last env.step, in call order (the kernel's adrp_race_moment_hash)"""
        out = np.zeros(self.E * self.N, np.uint32)
        assert lib().orc_race_moment_hash(self.h, _ptr(out)) == 0
        return out

    def contact_count(self):
        return lib().orc_contact_count(self.h)

    def env_contact(self):
        return np.array([lib().orc_env_contact(self.h, e) for e in range(self.E)], bool)

    def hover_eval(self):
        obs = np.zeros((self.E, self.N, self.D), np.float32)
        rew = np.zeros(self.E, np.float32)
        term = np.zeros(self.E, np.uint8)
        trunc = np.zeros(self.E, np.uint8)
        lib().orc_hover_eval(self.h, _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc))
        return obs, rew, term.astype(bool), trunc.astype(bool)


def poly4d_eval(coef, t):
    """firmware poly4d_eval of a [4, 8] float32 coefficient block -> (pos, vel, acc, omega, yaw)."""
    c = np.ascontiguousarray(coef, np.float32).reshape(4, 8)
    o = np.zeros(13, np.float32)
    lib().orc_poly4d_eval(_ptr(c), float(t), _ptr(o))
    return o[0:3], o[3:6], o[6:9], o[9:12], o[12]


def poly7_nojerk(T, x0, dx0, ddx0, xf, dxf, ddxf):
    o = np.zeros(8, np.float32)
    lib().orc_poly7_nojerk(T, x0, dx0, ddx0, xf, dxf, ddxf, _ptr(o))
    return o


def force_assembly(cfg, states, n, rpm, prev):
    """states: [N, 13] rows pos3, quat4 (xyzw), vel3, omega3 -> (link_force, link_torque) [5,3]."""
    st = np.ascontiguousarray(states, float)
    lf = np.zeros((5, 3)); lt = np.zeros((5, 3))
    rc = lib().orc_force_assembly(ctypes.byref(cfg), st.shape[0], _ptr(st), n,
                                  _ptr(np.ascontiguousarray(rpm, float)),
                                  _ptr(np.ascontiguousarray(prev, float)), _ptr(lf), _ptr(lt))
    assert rc == 0, lib().orc_last_error()
    return lf, lt


def hover_rpm(cfg, act):
    a = np.ascontiguousarray(act, np.float32); o = np.zeros(4)
    lib().orc_hover_rpm(ctypes.byref(cfg), _ptr(a), _ptr(o))
    return o


def dslpid(cfg, dt, inp, st):
    """DSLPIDControl.computeControl: inp = pos3 quat4 vel3 target_pos3 target_rpy3 target_vel3;
    st (9, float64) = last_rpy, integral_pos_e, integral_rpy_e, updated in place."""
    i = np.ascontiguousarray(inp, float)
    assert i.shape == (19,) and st.dtype == np.float64 and st.shape == (9,) and st.flags.c_contiguous
    o = np.zeros(4)
    lib().orc_dslpid(ctypes.byref(cfg), dt, _ptr(i), _ptr(st), _ptr(o))
    return o


def normal_pair(x0, x1):
    """the race action-noise Box-Muller of one Philox word pair (oracle/race.c normal_pair)"""
    z = np.zeros(2, np.float32)
    lib().orc_normal_pair(int(x0) & 0xFFFFFFFF, int(x1) & 0xFFFFFFFF, _ptr(z))
    return z


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32); k = np.ascontiguousarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(_ptr(c), _ptr(k), _ptr(o))
    return o


def euler_from_quat(q):
    q = np.ascontiguousarray(q, float); r = np.zeros(3)
    lib().orc_euler_from_quat(_ptr(q), _ptr(r))
    return r


def quat_from_euler(e):
    e = np.ascontiguousarray(e, float); q = np.zeros(4)
    lib().orc_quat_from_euler(_ptr(e), _ptr(q))
    return q


def derived_constants(cfg):
    out = np.zeros(6)
    lib().orc_derived_constants(ctypes.byref(cfg), _ptr(out))
    return out


def set_threads(n):
    """OpenMP threads for the env loop of Oracle.step (1 = the scalar restatement)."""
    lib().orc_set_threads(int(n))


def obs_wrapper_term(mode, term_env, gate0):
    """DroneObservationWrapper termination -> (terminated, terminated as the RewardWrapper sees it)"""
    t = ctypes.c_uint8(0); r = ctypes.c_int(0)
    lib().orc_obs_wrapper_term(int(mode), int(term_env), int(gate0), ctypes.byref(t), ctypes.byref(r))
    return bool(t.value), bool(r.value)


def set_bullet_variant(omit_wxv):
    """1: the base integrates without the spatial -> classical "+ w x v" conversion (probe of an
    unpinned reading of btMultiBody); 0: the restatement (default)"""
    lib().orc_set_bullet_variant(int(omit_wxv))


def default_config(task):
    from gym_pybullet_adrp_amd.utils.abi import AdrpConfig
    cfg = AdrpConfig()
    lib().orc_default_config(task, ctypes.byref(cfg))
    return cfg


def compute_pwms(control):
    c = np.ascontiguousarray(control, float); o = np.zeros(4)
    lib().orc_compute_pwms(_ptr(c), _ptr(o))
    return o


def pwms_to_rpms(pwm, noise):
    p = np.ascontiguousarray(pwm, float); n = np.ascontiguousarray(noise, float); o = np.zeros(4)
    lib().orc_pwms_to_rpms(_ptr(p), _ptr(n), _ptr(o))
    return o


def tick_schedule(n):
    o = np.zeros(n, np.uint8)
    lib().orc_tick_schedule(n, _ptr(o))
    return o


def race_body_distance(cfg, pos, quat, kind, gate_type, pose):
    """drone collision cylinder at (pos, quat) vs gate (kind 0, type 0 tall / 1 low) or obstacle (kind 1)"""
    return lib().orc_race_body_distance(ctypes.byref(cfg), _ptr(np.ascontiguousarray(pos, float)),
                                        _ptr(np.ascontiguousarray(quat, float)), kind, gate_type,
                                        _ptr(np.ascontiguousarray(pose, float)))


def shape_distance(a, b):
    """GJK distance; shape = [type(0 box, 1 cyl), c(3), R(9 row-major), h(3), r]"""
    return lib().orc_shape_distance(_ptr(np.ascontiguousarray(a, float)), _ptr(np.ascontiguousarray(b, float)))


def lpf_coeffs(fs, fc):
    o = np.zeros(5)
    lib().orc_lpf_coeffs(fs, fc, _ptr(o))
    return o


def race_obs_assemble(cfg, i, kin, gate_act, gate_in, obst_act, obst_in, current_gate):
    """MultiRaceAviary._computeObs assembly for drone i given the range-test outcomes"""
    N = kin.shape[0]
    D = 49 + (6 * (N - 1) if cfg.race_mode == 1 else 0)
    row = np.zeros(D)
    rc = lib().orc_race_obs_assemble(ctypes.byref(cfg), N, i, _ptr(np.ascontiguousarray(kin, float)),
                                     _ptr(np.ascontiguousarray(gate_act, float)), _ptr(np.ascontiguousarray(gate_in, np.uint8)),
                                     _ptr(np.ascontiguousarray(obst_act, float)), _ptr(np.ascontiguousarray(obst_in, np.uint8)),
                                     int(current_gate), _ptr(row))
    assert rc == 0
    return row


def race_terminated(cfg, pos, angv, contact, elim, fin):
    """-> (terminated, updated eliminated flags)"""
    e = np.ascontiguousarray(elim, np.uint8).copy()
    t = lib().orc_race_terminated(ctypes.byref(cfg), len(e), _ptr(np.ascontiguousarray(pos, float)),
                                  _ptr(np.ascontiguousarray(angv, float)), _ptr(np.ascontiguousarray(contact, np.uint8)),
                                  _ptr(e), _ptr(np.ascontiguousarray(fin, np.uint8)))
    return bool(t), e.astype(bool)


def race_truncated(cfg, step_counter):
    return bool(lib().orc_race_truncated(ctypes.byref(cfg), int(step_counter)))


def race_rays(gate_xyyaw, gate_type):
    fr = np.zeros((7, 3)); to = np.zeros((7, 3))
    lib().orc_race_rays(_ptr(np.ascontiguousarray(gate_xyyaw, float)), int(gate_type), _ptr(fr), _ptr(to))
    return fr, to


def race_progress(num_gates, self_id, hit_id, hit_frac, gate):
    g = ctypes.c_int(int(gate)); f = ctypes.c_int(0)
    lib().orc_race_progress(int(num_gates), int(self_id), _ptr(np.ascontiguousarray(hit_id, np.int32)),
                            _ptr(np.ascontiguousarray(hit_frac, float)), ctypes.byref(g), ctypes.byref(f))
    return g.value, bool(f.value)


class RewardWrapperState:
    """RewardWrapper internal state (current_gate_id, current_target, previous_pos)"""

    def __init__(self, obs0_row):
        self.gate = ctypes.c_int(int(obs0_row[48]))
        self.target = np.ascontiguousarray(obs0_row[12:15], float).copy()
        self.prev = np.ascontiguousarray(obs0_row[:3], float).copy()

    def step(self, row0, term, completed):
        return lib().orc_race_reward(ctypes.byref(self.gate), _ptr(self.target), _ptr(self.prev),
                                     _ptr(np.ascontiguousarray(row0, float)), int(term), int(completed))
