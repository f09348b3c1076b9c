"""MultiRaceAviary on the GPU: E envs x N drones, one fused HIP launch per env.step.

Mirrors envs/MultiRaceAviary.py:26-725 of the reference: the same constructor
arguments (race_config, drone_model, num_drones, physics, pyb_freq, ctrl_freq, gui,
record, racemode, obs, act), per-env spaces (action Box [-1,1]^(N,4); obs Box
(N, 49 [+ 6(N-1) COMPETE]) with the reference bounds), FULLSTATE actions (absolute target
x, y, z, yaw per drone), obs layout [pos, rpy, vel, ang_v | 4 x gate x,y,z,yaw | 4 gate
in-range flags | 4 x obstacle x,y,z | 4 flags | current gate (| others' pos+rpy)],
terminated = every drone eliminated or finished, truncated after episode_len_sec.
The reference returns reward 0; ``reward="wrapper"`` computes utils/wrapper.py's
RewardWrapper instead.  The Mellinger controllers that the reference runs in one OS
process per drone are fused into the kernel (500 Hz).

Batched extras: ``num_envs``, ``device``, ``precision``, ``seed``, ``autoreset``,
``env_offset``, ``link_frame_lag``.  step/reset return persistent device tensors.

``precision`` defaults to ``"fp64"``, the reference's precision: float64 physics and
MellingerControl wrapper, float32 firmware (as pycffirmware).  ``"fp32"`` selects the float32
kernel (about 1.6x the env-steps/s at config 4): its one-sub-step physics error is held to the
north star's 1e-4, its closed-loop env.step to 2e-3 (tests/test_race_gpu.py).
"""
import numpy as np
import torch

from .. import _lib
from ..utils import abi
from ..utils.enums import ActionType, DroneModel, ObservationType, Physics, PHYSICS_CODE, RaceMode
from ..utils.spaces import Box
from .base import AviaryEnv
from .tracks import fill_track


def race_config(race_config="level0", num_drones=2, physics="PYB", racemode="COMPARE", num_envs=1, seed=2024):
    """The adrp_config a MultiRaceAviary(race_config, num_drones, physics, racemode) builds, without a
    device handle (host-side: bench.py's CPU baseline, tests)."""
    cfg = _lib.default_config(abi.TASK_RACE)
    cfg.num_drones = int(num_drones)
    fill_track(cfg, race_config, int(num_drones))
    ph = Physics[physics] if isinstance(physics, str) else Physics(physics)
    rm = RaceMode[racemode] if isinstance(racemode, str) else RaceMode(racemode)
    cfg.physics = PHYSICS_CODE[ph]
    cfg.race_mode = abi.RACE_COMPETE if rm == RaceMode.COMPETE else abi.RACE_COMPARE
    cfg.num_envs = int(num_envs)
    cfg.seed = int(seed)
    return cfg


class MultiRaceAviary(AviaryEnv):
    """Batched counterpart of gym_pybullet_adrp.envs.MultiRaceAviary."""

    def __init__(self, race_config="level0", drone_model: DroneModel = DroneModel.CF2X, num_drones: int = 2,
                 physics: Physics = Physics.PYB, pyb_freq: int = 500, ctrl_freq: int = 25, gui=False, record=False,
                 racemode: RaceMode = RaceMode.COMPARE, obs: ObservationType = ObservationType.KIN,
                 act: ActionType = ActionType.PID, *, num_envs: int = 1, device: int = 0, precision: str = "fp64",
                 seed: int = 0, autoreset: bool = True, env_offset: int = 0, link_frame_lag: bool = True,
                 reward: str = "env", commands: bool = False):
        if drone_model not in (DroneModel.CF2X,):
            raise ValueError(f"DroneModel {drone_model} not supported (cf2x_IROS.urdf constants only)")
        if gui or record:
            raise ValueError("GUI / video recording are out of scope (DESIGN.md)")
        if obs != ObservationType.KIN:
            raise ValueError("only ObservationType.KIN is supported")
        if pyb_freq % ctrl_freq != 0:
            raise ValueError("[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.")
        if reward not in ("env", "wrapper"):
            raise ValueError("reward must be 'env' (MultiRaceAviary._computeReward) or 'wrapper' (RewardWrapper)")
        cfg = _lib.default_config(abi.TASK_RACE)
        cfg.num_drones = int(num_drones)
        self.config = fill_track(cfg, race_config, int(num_drones))
        cfg.physics = PHYSICS_CODE[Physics(physics)]
        cfg.race_mode = abi.RACE_COMPETE if RaceMode(racemode) == RaceMode.COMPETE else abi.RACE_COMPARE
        cfg.num_envs = int(num_envs)
        cfg.pyb_freq, cfg.ctrl_freq = int(pyb_freq), int(ctrl_freq)
        cfg.autoreset = 1 if autoreset else 0
        cfg.precision = {"fp32": 0, "fp64": 1}[precision]
        cfg.link_frame_lag = 1 if link_frame_lag else 0
        cfg.seed = int(seed) & (2 ** 64 - 1)
        cfg.env_offset = int(env_offset)
        cfg.track.reward_wrapper = 1 if reward == "wrapper" else 0
        self.cfg = cfg
        self.h = _lib.Handle(cfg, device)
        self.device = self.h.device
        # reference attributes
        self.DRONE_MODEL, self.PHYSICS, self.racemode = drone_model, physics, racemode
        self.observation_type, self.action_type = obs, act
        self.NUM_DRONES = int(num_drones)
        self.PYB_FREQ, self.CTRL_FREQ = int(pyb_freq), int(ctrl_freq)
        self.PYB_STEPS_PER_CTRL = self.PYB_FREQ // self.CTRL_FREQ
        self.PYB_TIMESTEP, self.CTRL_TIMESTEP = 1.0 / self.PYB_FREQ, 1.0 / self.CTRL_FREQ
        self.num_gates = cfg.track.num_gates
        self.env_bounds = np.array([[-cfg.track.bounds_hi[0], -cfg.track.bounds_hi[1], 0.0],
                                    list(cfg.track.bounds_hi)])
        self.action_scale = np.array([1, 1, 1, np.pi])
        self.num_envs = cfg.num_envs
        self.action_space = self._actionSpace()
        self.observation_space = self._observationSpace()
        E, N, D = self.num_envs, self.NUM_DRONES, self.h.D
        self._obs = torch.zeros((E, N, D), dtype=torch.float32, device=self.device)
        self._tobs = torch.zeros_like(self._obs)
        self._rew = torch.zeros(E, dtype=torch.float32, device=self.device)
        self._term = torch.zeros(E, dtype=torch.bool, device=self.device)
        self._trunc = torch.zeros(E, dtype=torch.bool, device=self.device)
        self._act_shape = (E, N, 4)
        self._info = {"answer": 42, "terminal_observation": self._tobs}
        self._last_act = None      # the last ndarray (FULLSTATE) action tensor, by reference
        self.commands = False
        if commands:
            self.enable_commands()

    # ---- spaces (MultiRaceAviary.py:284-343) ----
    def _actionSpace(self):
        lim = np.ones((self.NUM_DRONES, 4))
        return Box(low=-1 * lim, high=lim, dtype=float)

    def _observationSpace(self):
        lo = np.concatenate([[-5] * 3, [-np.pi] * 3, [-10] * 3, [-10] * 3, [-5, -5, -5, -np.pi] * 4, [-1] * 4,
                             [-5] * 12, [-1] * 4, [-1]])
        hi = np.concatenate([[5] * 3, [np.pi] * 3, [10] * 3, [10] * 3, [5, 5, 5, np.pi] * 4, [1] * 4,
                             [5] * 12, [1] * 4, [4]])
        if self.racemode == RaceMode.COMPETE:
            lo = np.concatenate([lo, ([-5] * 3 + [-np.pi] * 3) * (self.NUM_DRONES - 1)])
            hi = np.concatenate([hi, ([5] * 3 + [np.pi] * 3) * (self.NUM_DRONES - 1)])
        return Box(low=np.vstack([lo] * self.NUM_DRONES), high=np.vstack([hi] * self.NUM_DRONES), dtype=np.float64)

    # ---- gymnasium-style API, batched ----
    def reset(self, seed: int = None, options: dict = None, mask=None):
        """Reset all envs (or those with mask[e] != 0); `seed` re-keys the random streams first.
        Returns (obs [E,N,D], info)."""
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
        if m is None:
            self._last_act = None
        return self._obs, {"answer": 42}

    def enable_commands(self):
        """High-level command mode (include/adrp.h adrp_enable_commands): step() then also takes
        (Command, args) tuples, run through the firmware's high-level commander (commands.py).
        Enabled implicitly by the first tuple action.  The command state starts as a reset leaves
        it; drones that have stepped since their reset then get the FULLSTATE command their last
        ndarray step sent (MultiRaceAviary.py:190-202: (act[:3], 0, 0, act[3], 0, step_counter);
        eliminated drones STOP), so a drone given Command.NONE keeps flying to that target as in
        the reference.  The last action tensor is read again here (kept by reference, as
        BaseRLAviary keeps the caller's array): do not overwrite it between that step and this
        call.  From here on the steps run the command-mode kernel (one lane per drone)."""
        if not self.commands:
            self.h.enable_commands()
            self.commands = True
            if self._last_act is not None:
                self._resend_fullstate(self._last_act)

    def _resend_fullstate(self, act):
        from ..commands import CMD_ARGS, COMMAND_CODE, TIME_SLOT
        from ..utils.enums import Command
        E, N = self.num_envs, self.NUM_DRONES
        _, i = self.h.get_state()
        sc = i[self.h.field_names()[1].index("step_counter")].reshape(E, N)
        stepped = sc > 0                     # envs reset since (auto-reset) keep the reset state
        codes = torch.where(stepped, COMMAND_CODE[Command.FULLSTATE], COMMAND_CODE[Command.NONE]).to(torch.int32)
        args = torch.zeros((E, N, CMD_ARGS), dtype=torch.float64, device=self.device)
        a = act.reshape(E, N, 4).to(torch.float64)
        args[..., 0:3] = a[..., 0:3]
        args[..., 9] = a[..., 3]            # the kernel zeroes it under the DroneObservationWrapper
        args[..., TIME_SLOT] = (sc - self.PYB_STEPS_PER_CTRL).to(torch.float64)   # the step_counter it was sent at
        self.h.command(codes, args)

    def command(self, actions):
        """Send one (Command, args) per drone without stepping: a list per env of N tuples (the
        reference's list for E = 1), or (codes [E,N], args [E,N,14]) already encoded."""
        from ..commands import encode_commands
        self.enable_commands()
        if isinstance(actions, tuple) and len(actions) == 2 and hasattr(actions[0], "shape"):
            codes, args = actions
        else:
            codes, args = encode_commands(actions, self.num_envs, self.NUM_DRONES)
        self.h.command(torch.as_tensor(codes), torch.as_tensor(args))

    def step(self, action):
        """action [E,N,4]: absolute FULLSTATE target (x, y, z, yaw) per drone; or per drone a
        (Command, args) tuple (MultiRaceAviary.py:190-210; lists per env, commands.py); or the
        encoded pair (codes int32 [E,N], args float64 [E,N,14]) as tensors, e.g. from
        hardcoded.HardCodedCommander.predict: no per-drone Python on that path."""
        if isinstance(action, tuple) and len(action) == 2 and isinstance(action[0], torch.Tensor) \
                and isinstance(action[1], torch.Tensor) and action[1].dim() == 3:
            self.enable_commands()
            self.h.command(*action)
            self.h.step(None, self._obs, self._rew, self._term, self._trunc, self._tobs)
            return self._obs, self._rew, self._term, self._trunc, self._info
        if isinstance(action, (list, tuple)) and not _numeric(action):
            self.command(action)
            self.h.step(None, self._obs, self._rew, self._term, self._trunc, self._tobs)
            return self._obs, self._rew, self._term, self._trunc, self._info
        act = action
        if not (isinstance(act, torch.Tensor) and act.dtype == torch.float32 and act.device == self.device
                and act.is_contiguous() and act.shape == self._act_shape):
            act = torch.as_tensor(action, device=self.device, dtype=torch.float32).reshape(self._act_shape)
            act = act.contiguous()
        self.h.step(act, self._obs, self._rew, self._term, self._trunc, self._tobs)
        self._last_act = act
        return self._obs, self._rew, self._term, self._trunc, self._info

    def set_noise(self, act_noise=None, force=None):
        """Parity mode: the next steps take the action noise [E, N, S, 4] and the disturbance force
        [E, N, S, 3] of every drone and sub-step from these arrays instead of the device Philox
        streams (include/adrp.h adrp_set_noise): e.g. the values the reference draws from its
        np_random (MultiRaceAviary.py:223-228, 532-537).  The arrays are copied into persistent
        device buffers here, so call it before every step; set_noise() returns to Philox."""
        if act_noise is None and force is None:
            self._noise_bufs = None
            self.h.set_noise(None, None)
            return
        E, N, S = self.num_envs, self.NUM_DRONES, self.PYB_STEPS_PER_CTRL
        a = torch.as_tensor(act_noise, dtype=torch.float64).reshape(E * N, S, 4)
        f = torch.as_tensor(force, dtype=torch.float64).reshape(E * N, S, 3)
        if getattr(self, "_noise_bufs", None) is None:
            self._noise_bufs = (torch.empty((E * N, S, 4), dtype=torch.float64, device=self.device),
                                torch.empty((E * N, S, 3), dtype=torch.float64, device=self.device))
            self.h.set_noise(*self._noise_bufs)
        self._noise_bufs[0].copy_(a)
        self._noise_bufs[1].copy_(f)

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

    # ---- fused wrappers (utils/wrapper.py; gym_pybullet_adrp_amd.utils.wrapper) ----
    @property
    def reward_wrapper(self):
        return bool(self.cfg.track.reward_wrapper)

    @property
    def obs_wrapper(self):
        return int(self.cfg.track.obs_wrapper)

    def set_wrappers(self, reward_wrapper: bool, obs_wrapper: int):
        """RewardWrapper on/off; DroneObservationWrapper 0 off, 1 inside the RewardWrapper, 2 outside
        (include/adrp.h adrp_set_wrappers).  Takes effect from the next step."""
        self.h.set_wrappers(reward_wrapper, obs_wrapper)

    # ---- state ----
    @property
    def current_gate(self):
        """[E, N] gate index of every drone (MultiRaceAviary.current_gate)"""
        _, i = self.h.get_state()
        return i[6].reshape(self.num_envs, self.NUM_DRONES)

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

    def get_command_state(self):
        return self.h.get_command_state()

    def set_command_state(self, f, i):
        self.h.set_command_state(f, i)


def _numeric(x):
    """a nested list / tuple of numbers (an ndarray-like action), not (Command, args) tuples"""
    try:
        np.asarray(x, dtype=np.float64)
        return True
    except (TypeError, ValueError):
        return False
