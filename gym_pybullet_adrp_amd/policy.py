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
CRITIC_KEYS = ("mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
               "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
               "value_net.weight", "value_net.bias", "log_std")


def load_sb3_zip(path, critic=False):
    """-> (actor weights {name: float32 ndarray}, activation "tanh" | "relu"); critic=True: the
    weights dict also holds CRITIC_KEYS (value MLP, value_net, log_std) for rollout collection"""
    with zipfile.ZipFile(path) as zf:
        sd = torch.load(io.BytesIO(zf.read("policy.pth")), map_location="cpu", weights_only=True)
        data = json.loads(zf.read("data"))
    kw = data.get("policy_kwargs") or {}
    act = str(kw.get("activation_fn", "Tanh"))
    activation = "relu" if "ReLU" in act else "tanh"       # SB3 MlpPolicy default: nn.Tanh
    keys = ACTOR_KEYS + (CRITIC_KEYS if critic else ())
    return {k: sd[k].float().numpy() for k in keys}, activation


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
        if not 1 <= w3.shape[0] <= 4:
            raise ValueError("the action_net must have 1..4 outputs")
        self.act_dim = w3.shape[0]
        if self.act_dim != 4 and mode != "raw":
            raise ValueError("RLController transforms need the 4 outputs (x, y, z, yaw)")
        self.in_dim, self.h1, self.h2 = w1.shape[1], w1.shape[0], w2.shape[0]
        self.mode = MODES[mode]
        self.device = torch.device("cuda", device)
        self._w = w                                  # keep the host arrays alive during create
        h = ctypes.c_void_p()
        act = abi.POLICY_RELU if activation == "relu" else abi.POLICY_TANH
        ptr = [a.ctypes.data_as(ctypes.c_void_p) for a in w]
        rc = self.lib.adrp_policy_create2(device, self.in_dim, self.h1, self.h2, self.act_dim, act, *ptr, ctypes.byref(h))
        if rc != 0:
            msg = self.lib.adrp_last_error(None).decode()
            raise (ValueError if rc == abi.ERR_INVALID else _lib.AdrpError)(f"adrp_policy_create: {msg}")
        self.h = h
        self.has_critic = False
        if all(k in weights for k in CRITIC_KEYS):
            self.set_critic(weights)

    @classmethod
    def from_zip(cls, path, device=0, mode="relative", critic=False):
        w, activation = load_sb3_zip(path, critic=critic)
        return cls(w, activation, device, mode)

    def set_critic(self, weights):
        """attach the critic (CRITIC_KEYS: value MLP of the same shape, value_net, log_std) for
        ``sample`` (PPO rollout collection)"""
        v = [np.ascontiguousarray(weights[k], np.float32) for k in CRITIC_KEYS]
        if v[0].shape != (self.h1, self.in_dim) or v[2].shape != (self.h2, self.h1) or v[4].shape != (1, self.h2) \
                or v[6].shape != (self.act_dim,):
            raise ValueError("critic shapes must mirror the actor (value MLP in -> h1 -> h2 -> 1, log_std [act_dim])")
        ptr = [a.ctypes.data_as(ctypes.c_void_p) for a in v]
        rc = self.lib.adrp_policy_set_critic(self.h, *ptr)
        if rc != 0:
            raise _lib.AdrpError(f"adrp_policy_set_critic: {self.lib.adrp_last_error(None).decode()}")
        self.has_critic = True

    def sample(self, obs, seed, counter, env_act=None, action=None, value=None, log_prob=None, eps=None):
        """PPO rollout step (include/adrp.h adrp_policy_sample; SB3 ActorCriticPolicy.forward with
        deterministic=False) on the rows of obs [..., D]: returns (env_act, action, value, log_prob),
        device tensors, written into the given ones if passed.  ``counter`` (e.g. the rollout step)
        and ``seed`` key the Philox draws of the Gaussian sample."""
        rows = obs.numel() // obs.shape[-1]
        if not (obs.is_cuda and obs.dtype == torch.float32 and obs.is_contiguous()):
            raise ValueError("obs must be a contiguous float32 device tensor")
        dev = obs.device
        ea = 4 if self.mode != MODES["raw"] else self.act_dim
        env_act = torch.empty((rows, ea), dtype=torch.float32, device=dev) if env_act is None else env_act
        action = torch.empty((rows, self.act_dim), dtype=torch.float32, device=dev) if action is None else action
        value = torch.empty(rows, dtype=torch.float32, device=dev) if value is None else value
        log_prob = torch.empty(rows, dtype=torch.float32, device=dev) if log_prob is None else log_prob
        for t, n in ((env_act, rows * ea), (action, rows * self.act_dim), (value, rows), (log_prob, rows)):
            assert t.is_contiguous() and t.dtype == torch.float32 and t.numel() == n
        rc = self.lib.adrp_policy_sample(self.h, obs.data_ptr(), rows, obs.shape[-1], self.mode,
                                         int(seed) & (2 ** 64 - 1), int(counter) & 0xFFFFFFFF, env_act.data_ptr(),
                                         action.data_ptr(), value.data_ptr(), log_prob.data_ptr(),
                                         None if eps is None else eps.data_ptr(), _lib._raw_stream(dev.index))
        if rc != 0:
            raise _lib.AdrpError(f"adrp_policy_sample: {self.lib.adrp_last_error(None).decode()}")
        return env_act, action, value, log_prob

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
                                      _lib._raw_stream(obs.device.index))
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
