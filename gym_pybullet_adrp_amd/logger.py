"""Trajectory logging in the reference ``Logger`` format.

``utils/logger.py:9-127`` stores, per drone and per logged step, the 16 kinematic values of the
20-d state vector (``BaseAviary._getDroneStateVector``, BaseAviary.py:545-565: pos 3, quat 4,
rpy 3, vel 3, ang_v 3, last_clipped_action 4) reordered as pos, vel, rpy, ang_v, rpm, plus 12
control targets and a timestamp, and ``save()`` writes ``timestamps [n, T]``, ``states
[n, 16, T]``, ``controls [n, 12, T]`` with ``np.savez``.

``DeviceLogger`` does the same for chosen drone slots of a batched env without synchronising
the host per step: ``log()`` gathers the slots' state from the handle's SoA snapshot into a
preallocated device buffer (a few small torch ops, stream-ordered); ``save()`` copies once and
writes the reference's npz, so the reference's plotting / analysis code reads GPU runs.
"""
import os
from datetime import datetime

import numpy as np
import torch


def logger_arrays(timestamps, states20, controls):
    """[T, n] times, [T, n, 20] state vectors, [T, n, 12] controls -> the arrays Logger.log
    accumulates (timestamps [n, T], states [n, 16, T], controls [n, 12, T])."""
    s = np.asarray(states20, np.float64)
    reord = np.concatenate([s[..., 0:3], s[..., 10:13], s[..., 7:10], s[..., 13:20]], -1)   # logger.py:117
    return (np.asarray(timestamps, np.float64).T.copy(), np.transpose(reord, (1, 2, 0)).copy(),
            np.transpose(np.asarray(controls, np.float64), (1, 2, 0)).copy())


def _euler_xyz(q):
    """pybullet getEulerFromQuaternion (extrinsic x-y-z) on [..., 4] (x, y, z, w), float64"""
    x, y, z, w = q.unbind(-1)
    sarg = (-2.0 * (x * z - w * y)).clamp(-1.0, 1.0)
    roll = torch.atan2(2.0 * (y * z + w * x), w * w - x * x - y * y + z * z)
    pitch = torch.asin(sarg)
    yaw = torch.atan2(2.0 * (x * y + w * z), w * w + x * x - y * y - z * z)
    return torch.stack([roll, pitch, yaw], -1)


class DeviceLogger:
    """Logger(logging_freq_hz, output_folder, num_drones, duration_sec) for a batched env.

    ``slots``: flat drone indices ``env * NUM_DRONES + drone`` to record (default: every drone
    of env 0, i.e. what the reference's single env logs).  ``duration_steps`` preallocates the
    device buffer (the reference's duration_sec * logging_freq_hz)."""

    def __init__(self, env, logging_freq_hz, output_folder="results", slots=None, duration_steps=1000):
        self.env = env
        self.LOGGING_FREQ_HZ = logging_freq_hz
        self.OUTPUT_FOLDER = output_folder
        n_drones = env.NUM_DRONES
        self.slots = torch.as_tensor(list(range(n_drones)) if slots is None else slots, dtype=torch.long,
                                     device=env.device)
        self.n = int(self.slots.numel())
        names, inames = env.state_field_names()
        idx = {k: j for j, k in enumerate(names)}
        race = "rpm_0" in idx
        dyn = getattr(env, "PHYSICS", None) is not None and env.PHYSICS.name == "DYN"
        ang = "angv" if dyn else "omega"
        self._pos = [idx[f"pos_{a}"] for a in "xyz"]
        self._quat = [idx[f"quat_{a}"] for a in "xyzw"]
        self._vel = [idx[f"vel_{a}"] for a in "xyz"]
        self._ang = [idx[f"{ang}_{a}"] for a in "xyz"]
        self._rpm, self._ring = None, None
        if race:
            self._rpm = [idx[f"rpm_{k}"] for k in range(4)]
        elif env.PHYSICS.name in ("PYB_DRAG", "PYB_GND_DRAG_DW"):
            self._rpm = [idx[f"last_rpm_{k}"] for k in range(4)]      # maintained by the drag model
        elif env.ACT_TYPE.name in ("RPM", "ONE_D_RPM"):
            # last_clipped_action = HOVER_RPM * (1 + 0.05 a) of the newest ring entry
            A = env.h.A
            self._ring = (idx["ring_0_0"], env.ACTION_BUFFER_SIZE, A, inames.index("ring_head"), float(env.HOVER_RPM))
        self.T = int(duration_steps)
        dev = env.device
        self.states = torch.zeros((self.T, self.n, 20), dtype=torch.float64, device=dev)
        self.controls = torch.zeros((self.T, self.n, 12), dtype=torch.float64, device=dev)
        self.timestamps = torch.zeros((self.T, self.n), dtype=torch.float64, device=dev)
        self.k = 0

    def log(self, timestamp, controls=None):
        """Record the current state of every slot (call after env.step / env.reset)."""
        if self.k >= self.T:
            raise IndexError("DeviceLogger buffer full (raise duration_steps)")
        f, i = self.env.get_state()
        f = f[:, self.slots].double()
        st = self.states[self.k]
        st[:, 0:3] = f[self._pos].T
        q = f[self._quat].T
        st[:, 3:7] = q
        st[:, 7:10] = _euler_xyz(q)
        st[:, 10:13] = f[self._vel].T
        st[:, 13:16] = f[self._ang].T
        if self._rpm is not None:
            st[:, 16:20] = f[self._rpm].T
        elif self._ring is not None:
            r0, B, A, hrow, hover = self._ring
            head = i[hrow][self.slots // self.env.NUM_DRONES].long()
            newest = (head - 1) % B
            cols = [r0 + newest * A + (j if A == 4 else 0) for j in range(4)]
            a = torch.stack([f[c, torch.arange(self.n, device=f.device)] for c in cols], -1).float()
            st[:, 16:20] = hover * (1.0 + 0.05 * a).double()
        else:
            st[:, 16:20] = float("nan")      # DSLPIDControl output of a non-drag config is not kept
        if controls is not None:
            self.controls[self.k] = torch.as_tensor(controls, dtype=torch.float64, device=st.device).reshape(self.n, 12)
        self.timestamps[self.k] = float(timestamp)
        self.k += 1

    def arrays(self):
        return logger_arrays(self.timestamps[:self.k].cpu().numpy(), self.states[:self.k].cpu().numpy(),
                             self.controls[:self.k].cpu().numpy())

    def save(self):
        """Logger.save (logger.py:123-127): save-flight-<date>.npy holding an npz archive."""
        os.makedirs(self.OUTPUT_FOLDER, exist_ok=True)
        ts, states, controls = self.arrays()
        path = os.path.join(self.OUTPUT_FOLDER, "save-flight-" + datetime.now().strftime("%m.%d.%Y_%H.%M.%S") + ".npy")
        with open(path, "wb") as out_file:
            np.savez(out_file, timestamps=ts, states=states, controls=controls)
        return path
