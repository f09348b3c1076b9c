"""HoverAviary on the GPU: E independent envs stepped by one fused HIP launch.

Mirrors the reference surface (envs/HoverAviary.py:11-117, envs/BaseRLAviary.py,
envs/BaseAviary.py): same constructor arguments and attributes, same per-env
observation/action spaces, same obs layout [pos, rpy, vel, ang_v, 15 past actions],
reward max(0, 2-|p-(0,0,1)|^4), terminated |p-target|<1e-4, truncated by bounds / tilt /
8 s.  Batched extras: ``num_envs``, ``device``, ``precision``, ``seed``, ``autoreset``
and ``init_noise`` (per-reset uniform perturbation of the initial state, 0 = reference).
``precision`` defaults to ``"fp64"`` (the reference integrates in float64; held to 1e-9 of the
float64 CPU restatement per env.step); ``"fp32"`` is the faster float32 kernel, held to the north
star's 1e-4.

``step``/``reset`` take and return torch tensors that live on the GPU (no host copy):
obs [E, 1, D] float32, reward [E] float32, terminated / truncated [E] bool.
"""
import numpy as np
import torch

from .. import _lib
from ..utils import abi
from ..utils.enums import ActionType, DroneModel, ObservationType, Physics, PHYSICS_CODE
from ..utils.spaces import Box
from .base import AviaryEnv


# ActionType -> C-ABI code, and the per-drone action width (BaseRLAviary.py:141-147).  PID /
# VEL / ONE_D_PID run DSLPIDControl (control/DSLPIDControl.py) fused into the step kernel; its
# state persists across resets, as the reference builds the controllers once (:73-78).
_ACT_CODE = {ActionType.RPM: abi.ACT_RPM, ActionType.ONE_D_RPM: abi.ACT_ONE_D_RPM, ActionType.PID: abi.ACT_PID,
             ActionType.VEL: abi.ACT_VEL, ActionType.ONE_D_PID: abi.ACT_ONE_D_PID}
_ACT_SIZE = {ActionType.RPM: 4, ActionType.VEL: 4, ActionType.PID: 3, ActionType.ONE_D_RPM: 1,
             ActionType.ONE_D_PID: 1}


class HoverAviary(AviaryEnv):
    """Batched counterpart of gym_pybullet_adrp.envs.HoverAviary."""

    def __init__(self, drone_model: DroneModel = DroneModel.CF2X, initial_xyzs=None, initial_rpys=None,
                 physics: Physics = Physics.PYB, pyb_freq: int = 240, ctrl_freq: int = 30, gui=False,
                 record=False, obs: ObservationType = ObservationType.KIN, act: ActionType = ActionType.RPM,
                 *, num_envs: int = 1, device: int = 0, precision: str = "fp64", seed: int = 0,
                 autoreset: bool = True, init_noise=None, env_offset: int = 0, link_frame_lag: bool = True):
        if drone_model != DroneModel.CF2X:
            raise ValueError("only DroneModel.CF2X (cf2x_IROS.urdf) is supported")
        if gui or record:
            raise ValueError("GUI / video recording are out of scope (DESIGN.md)")
        if obs != ObservationType.KIN:
            raise ValueError("only ObservationType.KIN is supported")
        if act not in _ACT_CODE:
            raise ValueError("supported action types: RPM, ONE_D_RPM, PID, VEL, ONE_D_PID")
        if pyb_freq % ctrl_freq != 0:
            raise ValueError("[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.")
        cfg = _lib.default_config(abi.TASK_HOVER)
        cfg.physics = PHYSICS_CODE[physics]
        cfg.act_type = _ACT_CODE[act]
        cfg.num_envs = int(num_envs)
        cfg.pyb_freq, cfg.ctrl_freq = int(pyb_freq), int(ctrl_freq)
        cfg.action_buffer_size = int(ctrl_freq // 2)
        cfg.autoreset = 1 if autoreset else 0
        cfg.precision = {"fp32": 0, "fp64": 1}[precision]
        cfg.link_frame_lag = 1 if link_frame_lag else 0
        cfg.seed = int(seed) & (2 ** 64 - 1)
        cfg.env_offset = int(env_offset)
        if initial_xyzs is not None:
            abi.set_vec(cfg.init_xyz[0], np.asarray(initial_xyzs, float).reshape(3))
        if initial_rpys is not None:
            abi.set_vec(cfg.init_rpy[0], np.asarray(initial_rpys, float).reshape(3))
        for key, dst in (("xyz", cfg.init_xyz_noise), ("rpy", cfg.init_rpy_noise), ("vel", cfg.init_vel_noise),
                         ("omega", cfg.init_omega_noise)):
            if init_noise and key in init_noise:
                abi.set_vec(dst, np.broadcast_to(np.asarray(init_noise[key], float), 3))
        self.cfg = cfg
        self.h = _lib.Handle(cfg, device)
        self.device = self.h.device
        # reference attributes
        self.DRONE_MODEL, self.PHYSICS, self.OBS_TYPE, self.ACT_TYPE = drone_model, physics, obs, act
        self.NUM_DRONES = 1
        self.PYB_FREQ, self.CTRL_FREQ = int(pyb_freq), int(ctrl_freq)
        self.PYB_STEPS_PER_CTRL = self.PYB_FREQ // self.CTRL_FREQ
        self.PYB_TIMESTEP, self.CTRL_TIMESTEP = 1.0 / self.PYB_FREQ, 1.0 / self.CTRL_FREQ
        self.ACTION_BUFFER_SIZE = int(ctrl_freq // 2)
        self.TARGET_POS = np.array([0, 0, 1])
        self.EPISODE_LEN_SEC = 8
        d = cfg.drone
        self.M, self.L, self.KF, self.KM = d.m, d.l, d.kf, d.km
        self.J = np.diag([d.ixx, d.iyy, d.izz])
        self.G = cfg.gravity
        self.GRAVITY = self.G * self.M
        self.HOVER_RPM = np.sqrt(self.GRAVITY / (4 * self.KF))
        self.MAX_RPM = np.sqrt((d.thrust2weight * self.GRAVITY) / (4 * self.KF))
        if act == ActionType.VEL:
            self.SPEED_LIMIT = 0.03 * d.max_speed_kmh * (1000 / 3600)   # BaseRLAviary.py:94-95
        self.num_envs = cfg.num_envs
        self.action_space = self._actionSpace()
        self.observation_space = self._observationSpace()
        E, D = self.num_envs, self.h.D
        self._obs = torch.zeros((E, 1, D), dtype=torch.float32, device=self.device)
        self._tobs = torch.zeros_like(self._obs)
        self._rew = torch.zeros(E, dtype=torch.float32, device=self.device)
        # the kernel writes 0/1 bytes: valid torch.bool storage, returned without a cast
        self._term = torch.zeros(E, dtype=torch.bool, device=self.device)
        self._trunc = torch.zeros(E, dtype=torch.bool, device=self.device)
        self._act_shape = (E, 1, self.h.A)
        self._info = {"answer": 42, "terminal_observation": self._tobs}
        self.h.bind(self._obs, self._rew, self._term, self._trunc, self._tobs)
        self._act_ok = (None, 0)        # (tensor, address) of the last validated action

    # ---- spaces (BaseRLAviary.py:132-156, 243-277) ----
    def _actionSpace(self):
        size = _ACT_SIZE[self.ACT_TYPE]
        return Box(low=-np.ones((1, size)), high=np.ones((1, size)), dtype=np.float32)

    def _observationSpace(self):
        lo, hi = -np.inf, np.inf
        low = [lo, lo, 0] + [lo] * 9
        high = [hi] * 12
        size = _ACT_SIZE[self.ACT_TYPE]
        low += [-1] * size * self.ACTION_BUFFER_SIZE
        high += [+1] * size * self.ACTION_BUFFER_SIZE
        return Box(low=np.array([low]), high=np.array([high]), dtype=np.float32)

    # ---- gymnasium-style API, batched ----
    def reset(self, seed: int = None, options: dict = None, mask=None):
        """Reset all envs (or those with mask[e] != 0); `seed` re-keys the random streams first.
        Returns (obs [E,1,D], info)."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        if seed is not None:
            # BaseAviary.reset(seed) reseeds np_random, then resets: here the Philox key of every env
            # (a fresh env built with this seed gives the same episodes from here on)
            if m is not None:
                raise ValueError("reset(seed=...) re-keys every env: call it without a mask")
            self.h.reseed(seed)
        self.h.reset(self._obs, m)
        return self._obs, {"answer": 42}

    def step(self, action):
        """One env.step of every env: action [E,1,A] (torch or numpy, in [-1,1]).

        Returns views of persistent device buffers (obs [E,1,D], reward [E],
        terminated [E], truncated [E]) that the next step overwrites."""
        ok, ptr = self._act_ok
        if action is ok and action.data_ptr() == ptr:      # the tensor validated last time, unchanged
            self.h.step_ptr(ptr)
            return self._obs, self._rew, self._term, self._trunc, self._info
        act = action
        if not (isinstance(act, torch.Tensor) and act.dtype == torch.float32 and act.device == self.device
                and act.is_contiguous() and act.shape == self._act_shape):
            act = torch.as_tensor(action, device=self.device, dtype=torch.float32).reshape(self._act_shape)
            act = act.contiguous()
        else:
            self._act_ok = (action, action.data_ptr())
        self.h.step_ptr(act.data_ptr())
        return self._obs, self._rew, self._term, self._trunc, self._info

    def close(self):
        self.h.close()

    def bind_outputs(self, obs, rew, term, trunc, tobs=None):
        """Write step / reset outputs into caller-owned device tensors from now on (e.g. views of a
        collective's send buffer, sharding.ShardedAviary(packed=True), or the SB3 adapter's packed
        host-copy buffer): obs [E,N,D] float32, reward [E] float32, terminated / truncated [E] bool,
        optionally the terminal observations [E,N,D] float32, all contiguous on this env's device."""
        want = ((self._obs, obs), (self._rew, rew), (self._term, term), (self._trunc, trunc))
        if tobs is not None:
            want += ((self._tobs, tobs),)
        for old, new in want:
            if new.shape != old.shape or new.dtype != old.dtype or new.device != old.device or not new.is_contiguous():
                raise ValueError(f"bind_outputs: need a contiguous {old.dtype} {tuple(old.shape)} tensor on {old.device}")
        self._obs, self._rew, self._term, self._trunc = obs, rew, term, trunc
        if tobs is not None:
            self._tobs = tobs
            self._info["terminal_observation"] = tobs
        self.h.bind(self._obs, self._rew, self._term, self._trunc, self._tobs)

    # ---- persistent stepping (BASELINE config 1: a Python loop stepping a few envs synchronously) ----
    def persistent(self):
        """A resident step kernel for this env (include/adrp.h adrp_persistent_*): ``step(action)``
        takes a numpy action, returns numpy views of host-mapped outputs, with no kernel launch per
        step.  Use as a context manager; ``step`` / ``reset`` / ``get_state`` of the env itself are
        refused until it is closed."""
        return PersistentStepper(self)

    # ---- introspection (tests / teacher forcing) ----
    def get_state(self):
        return self.h.get_state()

    def set_state(self, f, i):
        self.h.set_state(f, i)

    def state_field_names(self):
        return self.h.field_names()

    def step_bytes(self):
        return self.h.step_bytes()

    @property
    def kernel_name(self):
        """the step-kernel instantiation this env launches now (include/adrp.h adrp_handle_kernel_name)"""
        return self.h.kernel_name()


class PersistentStepper:
    """HoverAviary.persistent(): the env.step of a resident kernel polling a host-mapped mailbox.

    ``step(action)`` writes the action (numpy, [E,1,A]) into mapped memory and returns when the
    step is done: (obs [E,1,D], reward [E], terminated [E], truncated [E], info) as numpy views of
    mapped memory that the next step overwrites (``info["terminal_observation"]`` likewise, for the
    auto-reset envs).  Results are those of ``HoverAviary.step`` on the same state and action."""

    def __init__(self, env):
        import ctypes
        self.env = env
        h = env.h
        ptrs = [ctypes.c_void_p() for _ in range(6)]
        rc = h.lib.adrp_persistent_begin(h.h, *[ctypes.byref(p) for p in ptrs])
        if rc != 0:
            raise _lib.AdrpError(f"adrp_persistent_begin: {h.lib.adrp_last_error(h.h).decode()}")
        E, D, A = env.num_envs, h.D, h.A

        def view(p, ctype, shape):
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctype)), shape=shape)
        self.act = view(ptrs[0], ctypes.c_float, (E, 1, A))
        self.obs = view(ptrs[1], ctypes.c_float, (E, 1, D))
        self.rew = view(ptrs[2], ctypes.c_float, (E,))
        self.term = view(ptrs[3], ctypes.c_uint8, (E,)).view(np.bool_)
        self.trunc = view(ptrs[4], ctypes.c_uint8, (E,)).view(np.bool_)
        self.tobs = view(ptrs[5], ctypes.c_float, (E, 1, D))
        self.info = {"answer": 42, "terminal_observation": self.tobs}
        self._step, self._h, self._lib = h.lib.adrp_persistent_step, h.h, h.lib
        self.active = True

    def step(self, action):
        self.act[...] = action
        if self._step(self._h) != 0:
            raise _lib.AdrpError(f"adrp_persistent_step: {self._lib.adrp_last_error(self._h).decode()}")
        return self.obs, self.rew, self.term, self.trunc, self.info

    def close(self):
        if self.active:
            self.active = False
            if getattr(self.env.h, "h", None) is None:   # the env was closed first: adrp_destroy ended it
                return
            if self._lib.adrp_persistent_end(self._h) != 0:
                raise _lib.AdrpError(f"adrp_persistent_end: {self._lib.adrp_last_error(self._h).decode()}")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
