"""On-device policy forward for closed-loop rollouts.

The reference drives each MultiRaceAviary drone with an ``RLController``
(user_controller/RLController.py:39-73) that calls ``PPO.predict(obs, deterministic=True)``
(stable_baselines3 2.3.2) on one observation at a time on the host and turns the action into a
FULLSTATE setpoint.  ``DevicePolicy`` runs that actor (mlp_extractor.policy_net + action_net,
clipped to the [-1, 1] action Box) for every drone of every env in one f32-MFMA launch
(csrc/policy_kernel.h) straight from ``adrp_step``'s observation buffer into the next step's
action buffer: no host round-trip, capturable in a HIP graph.

``load_sb3_zip`` reads an SB3 zip the way ``PPO.load`` would for the actor, without SB3 and
without unpickling: ``policy.pth`` through ``torch.load(weights_only=True)`` and the
``policy_kwargs`` (net_arch / activation_fn) from the JSON ``data`` member.
"""
import ctypes
import io
import json
import zipfile

import numpy as np
import torch

from . import _lib
from .utils import abi

MODES = {"raw": abi.POLICY_RAW, "relative": abi.POLICY_RELATIVE, "absolute": abi.POLICY_ABSOLUTE}
ACTOR_KEYS = ("mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
              "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
              "action_net.weight", "action_net.bias")


def load_sb3_zip(path):
    """-> (actor weights {name: float32 ndarray}, activation "tanh" | "relu")"""
    with zipfile.ZipFile(path) as zf:
        sd = torch.load(io.BytesIO(zf.read("policy.pth")), map_location="cpu", weights_only=True)
        data = json.loads(zf.read("data"))
    kw = data.get("policy_kwargs") or {}
    act = str(kw.get("activation_fn", "Tanh"))
    activation = "relu" if "ReLU" in act else "tanh"       # SB3 MlpPolicy default: nn.Tanh
    return {k: sd[k].float().numpy() for k in ACTOR_KEYS}, activation


class DevicePolicy:
    """Actor of an SB3 MlpPolicy with two hidden layers, on one GPU.

    ``mode``: "raw" (the clipped action), "relative" (RLController: a[3] = 0, setpoint =
    obs[[0,1,2,5]] + a*[1,1,1,pi], yaw map2pi) or "absolute" (RLControllerTwoGates:
    a[3] = 0, setpoint = a*[1,1,1,pi])."""

    def __init__(self, weights, activation="tanh", device=0, mode="relative"):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.AdrpError("no HIP device visible: libadrp has no CPU fallback")
        w = [np.ascontiguousarray(weights[k], np.float32) for k in ACTOR_KEYS]
        (w1, b1, w2, b2, w3, b3) = w
        if w3.shape[0] != 4:
            raise ValueError("the action_net must have 4 outputs (x, y, z, yaw)")
        self.in_dim, self.h1, self.h2 = w1.shape[1], w1.shape[0], w2.shape[0]
        self.mode = MODES[mode]
        self.device = torch.device("cuda", device)
        self._w = w                                  # keep the host arrays alive during create
        h = ctypes.c_void_p()
        act = abi.POLICY_RELU if activation == "relu" else abi.POLICY_TANH
        ptr = [a.ctypes.data_as(ctypes.c_void_p) for a in w]
        rc = self.lib.adrp_policy_create(device, self.in_dim, self.h1, self.h2, act, *ptr, ctypes.byref(h))
        if rc != 0:
            msg = self.lib.adrp_last_error(None).decode()
            raise (ValueError if rc == abi.ERR_INVALID else _lib.AdrpError)(f"adrp_policy_create: {msg}")
        self.h = h

    @classmethod
    def from_zip(cls, path, device=0, mode="relative"):
        w, activation = load_sb3_zip(path)
        return cls(w, activation, device, mode)

    def act(self, obs, out=None):
        """obs [..., D] float32 on the device (D >= in_dim; the first in_dim columns are the
        policy input) -> setpoints [..., 4] (written into ``out`` if given)"""
        rows = obs.numel() // obs.shape[-1]
        if not (obs.is_cuda and obs.dtype == torch.float32 and obs.is_contiguous()):
            raise ValueError("obs must be a contiguous float32 device tensor")
        if out is None:
            out = torch.empty(obs.shape[:-1] + (4,), dtype=torch.float32, device=obs.device)
        assert out.is_contiguous() and out.numel() == rows * 4
        rc = self.lib.adrp_policy_act(self.h, obs.data_ptr(), rows, obs.shape[-1], self.mode, out.data_ptr(),
                                      torch.cuda.current_stream(obs.device).cuda_stream)
        if rc != 0:
            raise _lib.AdrpError(f"adrp_policy_act: {self.lib.adrp_last_error(None).decode()}")
        return out

    def close(self):
        if getattr(self, "h", None):
            self.lib.adrp_policy_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rollout(env, policy, steps, act=None):
    """Closed-loop MultiRaceAviary rollout entirely on the device: obs -> policy -> setpoints
    -> env.step, ``steps`` times (env auto-resets done envs).  Returns the last step's outputs."""
    obs = env._obs if hasattr(env, "_obs") else env.reset()[0]
    if act is None:
        act = torch.empty(obs.shape[:-1] + (4,), dtype=torch.float32, device=obs.device)
    out = None
    for _ in range(steps):
        policy.act(obs, out=act)
        out = env.step(act)
        obs = out[0]
    return out
