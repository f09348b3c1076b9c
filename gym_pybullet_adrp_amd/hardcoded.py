"""Batched HardCodedController: the reference's example scripted racer for every drone of every env,
emitting the command arrays of commands.py as device tensors (no per-drone Python on the step path).

Reference: user_controller/HardCodedController.py:14-190 as scripts/sim.py:68-106 drives it (one
controller per drone, built from the reset observation with info["delay"] = drone_id, then
predict(obs[i], ep_time=episode_step / ctrl_freq) once per env.step).  Per drone:
  * construction: 16 waypoints from the drone's start xy and the nominal gates (obs[12:28]), a
    smoothing spline through them (scipy splprep, s = 0.1) sampled at 12 s x CTRL_FREQ points;
  * predict: TAKEOFF [0.3, 2] on the first call; then FULLSTATE (ref[step], 0, 0.5, 0, 0, ep_time)
    with step = int(ep_time * CTRL_FREQ) - (2 + delay) * CTRL_FREQ clipped to [0, len]; past the
    end one NOTIFY [ep_time], one LAND [0, 2], then NONE.
CTRL_FREQ is the controller's own 25 Hz (utils/constants.py:31), not the env's ctrl_freq.

The spline is planned on the host at construction / re-plan (scipy, once per distinct start);
predict() is a handful of tensor ops on the env's device and returns (codes int32 [E, N],
args float64 [E, N, 14]) for MultiRaceAviary.step((codes, args)) / adrp_race_command.
"""
import numpy as np
import torch

from .commands import CMD_ARGS, COMMAND_CODE, TIME_SLOT
from .utils.enums import Command

CTRL_FREQ = 25          # utils/constants.py:31-32 (the controller's clock)
Z_LOW, Z_HIGH = 0.3, 0.775
DURATION = 12           # s of spline (HardCodedController.py:112)
TAKEOFF = (0.3, 2.0)    # height, duration (HardCodedController.py:160)
LAND = (0.0, 2.0)       # HardCodedController.py:184


def waypoints(start_xy, gates):
    """the 16 waypoints of HardCodedController.py:63-107; gates [4, 4] (x, y, z, yaw)"""
    g = np.asarray(gates, np.float64)
    x0, y0 = float(start_xy[0]), float(start_xy[1])
    zm = (Z_LOW + Z_HIGH) / 2
    mx, my = (g[0, 0] + g[1, 0]) / 2, (g[0, 1] + g[1, 1]) / 2
    return np.array([
        [x0, y0, 0.3], [1, 0, Z_LOW],
        [g[0, 0] + 0.2, g[0, 1] + 0.1, Z_LOW], [g[0, 0] + 0.1, g[0, 1], Z_LOW], [g[0, 0] - 0.1, g[0, 1], Z_LOW],
        [mx - 0.7, my - 0.3, zm], [mx - 0.5, my - 0.6, zm],
        [g[1, 0] - 0.3, g[1, 1] - 0.2, Z_HIGH], [g[1, 0] + 0.2, g[1, 1] + 0.2, Z_HIGH],
        [g[2, 0], g[2, 1] - 0.4, Z_LOW], [g[2, 0], g[2, 1] + 0.2, Z_LOW], [g[2, 0], g[2, 1] + 0.2, Z_HIGH + 0.2],
        [g[3, 0], g[3, 1] + 0.1, Z_HIGH], [g[3, 0], g[3, 1] - 0.1, Z_HIGH + 0.1],
        [-0.5, -1.2, Z_HIGH], [-0.5, -1.4, Z_HIGH]], np.float64)


def plan(start_xy, gates):
    """[DURATION * CTRL_FREQ, 3] reference trajectory (HardCodedController.py:109-115)"""
    from scipy import interpolate
    w = waypoints(start_xy, gates)
    tck, _ = interpolate.splprep([w[:, 0], w[:, 1], w[:, 2]], s=0.1)
    ref = np.stack(interpolate.splev(np.linspace(0, 1, int(DURATION * CTRL_FREQ)), tck), -1)
    if not ref[:, 2].max() < 2.5:
        raise ValueError("Drone must stay below the ceiling")
    return ref


class HardCodedCommander:
    """One HardCodedController per drone of an [E, N] batch.

    obs0: the reset observation [E, N, D] (MultiRaceAviary.reset); delay: [N] or [E, N] seconds of
    extra take-off wait (scripts/sim.py:75 uses the drone index, the default)."""

    def __init__(self, obs0, delay=None, device=None):
        o = obs0.detach().cpu().numpy() if isinstance(obs0, torch.Tensor) else np.asarray(obs0)
        if o.ndim == 2:
            o = o[None]
        self.E, self.N = o.shape[:2]
        self.device = torch.device(device) if device is not None else (
            obs0.device if isinstance(obs0, torch.Tensor) else torch.device("cpu"))
        if delay is None:
            delay = np.arange(self.N)
        d = np.broadcast_to(np.asarray(delay, np.int64), (self.E, self.N))
        self.L = int(DURATION * CTRL_FREQ)
        self._offset = torch.as_tensor((2 + d) * CTRL_FREQ, device=self.device)
        self._ref = torch.empty((self.E, self.N, self.L, 3), dtype=torch.float64, device=self.device)
        self._flags = torch.zeros((3, self.E, self.N), dtype=torch.bool, device=self.device)  # take_off, notify, land
        self._cache = {}
        self.replan(o)
        dev = self.device
        self._codes = {c: torch.tensor(COMMAND_CODE[c], dtype=torch.int32, device=dev)
                       for c in (Command.NONE, Command.FULLSTATE, Command.TAKEOFF, Command.NOTIFY, Command.LAND)}

    def replan(self, obs0, mask=None):
        """Rebuild the controllers of the envs with mask[e] (all if None) from their reset observation
        (scripts/sim.py:72-76 builds new agents every episode)."""
        o = obs0.detach().cpu().numpy() if isinstance(obs0, torch.Tensor) else np.asarray(obs0)
        if o.ndim == 2:
            o = o[None]
        envs = range(self.E) if mask is None else np.flatnonzero(
            mask.detach().cpu().numpy() if isinstance(mask, torch.Tensor) else np.asarray(mask))
        ref = np.empty((len(envs), self.N, self.L, 3))
        for j, e in enumerate(envs):
            for n in range(self.N):
                start = o[e, n, 0:2].astype(np.float64)
                gates = o[e, n, 12:28].astype(np.float64).reshape(4, 4)   # HardCodedController.py:53
                key = start.tobytes() + gates.tobytes()
                r = self._cache.get(key)
                if r is None:
                    r = self._cache[key] = plan(start, gates)
                ref[j, n] = r
        idx = torch.as_tensor(np.asarray(list(envs), np.int64), device=self.device)
        self._ref[idx] = torch.as_tensor(ref, device=self.device)
        self._flags[:, idx] = False

    @property
    def reference_trajectory(self):
        """[E, N, L, 3] spline samples (HardCodedController.ref_x / ref_y / ref_z)"""
        return self._ref

    def predict(self, ep_time):
        """ep_time: seconds since each env's episode start, a float or [E] tensor.
        Returns (codes int32 [E, N], args float64 [E, N, 14]) (commands.py layout)."""
        E, N, L = self.E, self.N, self.L
        t = torch.as_tensor(ep_time, dtype=torch.float64, device=self.device)
        t = t.reshape(-1, 1).expand(E, N) if t.dim() else t.expand(E, N)
        it = torch.trunc(t * CTRL_FREQ).to(torch.int64)                    # int(ep_time * CTRL_FREQ)
        step = (it - self._offset).clamp(0, L)
        took, notified, landed = self._flags
        fst = took & (step < L)
        ntf = took & ~fst & ~notified
        lnd = took & ~fst & notified & ~landed
        tko = ~took
        C = self._codes
        codes = torch.where(tko, C[Command.TAKEOFF], torch.where(fst, C[Command.FULLSTATE], torch.where(
            ntf, C[Command.NOTIFY], torch.where(lnd, C[Command.LAND], C[Command.NONE]))))
        args = torch.zeros((E, N, CMD_ARGS), dtype=torch.float64, device=self.device)
        pos = torch.gather(self._ref, 2, step.clamp(max=L - 1)[..., None, None].expand(E, N, 1, 3))[:, :, 0]
        args[..., 0:3] = torch.where(fst[..., None], pos, 0.0)
        args[..., 6:9] = torch.where(fst[..., None], 0.5, 0.0)             # target_acc = ones(3) * 0.5
        args[..., 0] = torch.where(tko, TAKEOFF[0], torch.where(ntf, t, torch.where(lnd, LAND[0], args[..., 0])))
        args[..., 1] = torch.where(tko, TAKEOFF[1], torch.where(lnd, LAND[1], args[..., 1]))
        # args[-1]: the commander clock process_command_queue reads (MellingerControl.py:57)
        args[..., TIME_SLOT] = torch.where(tko, TAKEOFF[1], torch.where(fst | ntf, t, torch.where(lnd, LAND[1], 0.0)))
        self._flags[0] |= tko
        self._flags[1] |= ntf
        self._flags[2] |= lnd
        return codes, args
