"""Stable-Baselines3 VecEnv view of the batched aviaries (drop-in boundary).

The reference trains with ``make_vec_env(HoverAviary, env_kwargs, n_envs)`` +
``PPO('MlpPolicy', vec_env)`` (examples/learn.py:53-57, 72-94): SB3 then drives one Python
env object per env through DummyVecEnv.  Here one device handle already steps all envs,
so the adapter implements SB3's VecEnv protocol directly:

* ``reset() -> obs``; ``step_async(actions)`` / ``step_wait() -> (obs, rewards, dones, infos)``
  with ``dones = terminated | truncated``, auto-reset inside the kernel, and per-env infos
  carrying ``terminal_observation`` and ``TimeLimit.truncated`` as SB3's wrappers would;
* per-env ``observation_space`` / ``action_space`` with the reference's shapes and bounds;
* ``close``, ``seed``, ``get_attr``, ``set_attr``, ``env_method``, ``env_is_wrapped``.

Outputs are numpy (what SB3's rollout buffer consumes) unless ``as_torch=True``, which
returns the device tensors untouched (for torch-native learners).  When
stable_baselines3 is importable the class derives from its ``VecEnv`` so
``isinstance`` checks in SB3 pass; otherwise it is a plain class with the same methods.
"""
import numpy as np
import torch

try:  # pragma: no cover - SB3 is not part of this image
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except ImportError:  # pragma: no cover
    _VecEnvBase = object


class AviaryVecEnv(_VecEnvBase):
    """SB3 VecEnv over one batched aviary (HoverAviary / MultiRaceAviary of this package)."""

    def __init__(self, env, as_torch=False):
        self.env = env
        self.num_envs = env.num_envs
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self.render_mode = None
        self.as_torch = as_torch
        self._actions = None
        self._seed = None
        if _VecEnvBase is not object:  # pragma: no cover
            _VecEnvBase.__init__(self, self.num_envs, self.observation_space, self.action_space)

    # ---- conversion ----
    def _out(self, x):
        return x if self.as_torch else x.detach().cpu().numpy()

    # ---- VecEnv API ----
    def reset(self):
        seed, self._seed = self._seed, None
        obs, _ = self.env.reset(seed=seed)
        return self._out(obs).copy() if not self.as_torch else obs.clone()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        obs, rew, term, trunc, info = self.env.step(self._actions)
        done = term | trunc
        if self.as_torch:
            return obs.clone(), rew.clone(), done, {"terminated": term.clone(), "truncated": trunc.clone(),
                                                   "terminal_observation": info["terminal_observation"].clone()}
        obs_np, rew_np = obs.cpu().numpy().copy(), rew.cpu().numpy().copy()
        term_np, trunc_np = term.cpu().numpy(), trunc.cpu().numpy()
        done_np = term_np | trunc_np
        infos = [{} for _ in range(self.num_envs)]
        idx = np.flatnonzero(done_np)
        if len(idx):
            tobs = info["terminal_observation"][torch.as_tensor(idx, device=obs.device)].cpu().numpy()
            for j, e in enumerate(idx):
                infos[e]["terminal_observation"] = tobs[j]
                infos[e]["TimeLimit.truncated"] = bool(trunc_np[e] and not term_np[e])
        return obs_np, rew_np, done_np, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.env.close()

    def seed(self, seed=None):
        """SB3 VecEnv.seed: applied at the next reset (one Philox key for the batch; envs differ by
        their global env id)"""
        self._seed = seed
        return [seed] * self.num_envs

    def get_images(self):
        raise NotImplementedError("rendering is out of scope (DESIGN.md)")

    def render(self, mode=None):
        raise NotImplementedError("rendering is out of scope (DESIGN.md)")

    def get_attr(self, attr_name, indices=None):
        return [getattr(self.env, attr_name)] * len(self._indices(indices))

    def set_attr(self, attr_name, value, indices=None):
        setattr(self.env, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        out = getattr(self.env, method_name)(*method_args, **method_kwargs)
        return [out] * len(self._indices(indices))

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return list(indices)


def HoverAviaryVec(n_envs=1, as_torch=False, **env_kwargs):
    """``make_vec_env(HoverAviary, env_kwargs=..., n_envs=...)`` counterpart"""
    from .envs.hover import HoverAviary
    return AviaryVecEnv(HoverAviary(num_envs=n_envs, **env_kwargs), as_torch=as_torch)


def MultiRaceAviaryVec(n_envs=1, as_torch=False, **env_kwargs):
    from .envs.race import MultiRaceAviary
    return AviaryVecEnv(MultiRaceAviary(num_envs=n_envs, **env_kwargs), as_torch=as_torch)
