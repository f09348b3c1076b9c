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

Host path (SURVEY.md §7 hard part 7).  Default (``direct``): ONE C call per step
(include/adrp.h ``adrp_vec_step``): the step kernel reads the actions from and writes obs / reward
straight into a pinned host block (mapped into the device: no copy engine, no separate copy call), a
compaction kernel writes the flags, the finished envs' ids and their terminal rows into the same
block, and the host waits once.  The blocks form a ring of ``ring`` (default 3, at most 4): the
returned obs / rewards / dones and the infos' terminal observations are views of the block the step
wrote, valid until ``ring`` more steps have been taken (SB3's OnPolicyAlgorithm.collect_rollouts
copies obs into its rollout buffer one step later and reads the infos at once, so the default ring
is safe for it; ``zero_copy=False`` returns fresh copies, DummyVecEnv's semantics, at ~15 us more
per step for 4,096 envs).  Fallback (``direct=False``, or a library without adrp_vec_step): the env writes obs / reward / terminated / truncated into
ONE packed device buffer (``bind_outputs``) and its terminal observations into a device buffer of
their own; ``adrp_compact_rows`` then gathers the finished envs' ids and terminal rows behind the
flags in the packed buffer, so ``step_wait`` issues one asynchronous copy of about the obs size into
pinned host memory and waits once (the whole terminal-obs batch no longer crosses PCIe); the
actions go the other way through a pinned staging buffer (one asynchronous copy).
``infos`` is a lazy sequence: a finished env's dict is made when the caller first reads it; every
other entry is one shared read-only empty mapping (SB3 reads infos and copies the dicts it
annotates; writing into a shared entry raises).  Returned
arrays are fresh copies (DummyVecEnv semantics) unless ``zero_copy=True``: then they are views
of a ring of ``ring`` pinned buffers, valid until ``ring`` more steps have been taken.
"""
import contextlib
import ctypes
import types
from collections.abc import Sequence

import numpy as np
import torch

from . import _lib
from .utils import abi

_NO_INFO = types.MappingProxyType({})


class _StepInfos(Sequence):
    """infos of one step, as SB3's VecEnv returns them (one mapping per env), built lazily: the envs
    that finished get their own dict ({"terminal_observation", "TimeLimit.truncated"}) when first
    read, then the same (mutable) dict on every read; every other entry is the shared read-only
    empty mapping.  A step with hundreds of finished envs no longer builds hundreds of dicts that
    the caller may never look at; iteration walks the (ascending) finished ids alongside."""
    __slots__ = ("_n", "_idx", "_row", "_tobs", "_tl", "_made")

    def __init__(self, n, idx, tobs, tl):
        self._n, self._idx, self._row = n, idx, None
        self._tobs, self._tl, self._made = tobs, tl, {}

    def __len__(self):
        return self._n

    def _info(self, e, j):
        d = self._made.get(e)
        if d is None:
            d = self._made[e] = {"terminal_observation": self._tobs[j], "TimeLimit.truncated": bool(self._tl[j])}
        return d

    def __getitem__(self, e):
        if isinstance(e, slice):
            return [self[i] for i in range(*e.indices(self._n))]
        if e < 0:
            e += self._n
        if not 0 <= e < self._n:
            raise IndexError(e)
        if self._row is None:
            self._row = dict(zip(self._idx.tolist(), range(len(self._idx))))
        j = self._row.get(e)
        return _NO_INFO if j is None else self._info(e, j)

    def __iter__(self):
        ids = self._idx.tolist()
        j, nxt = 0, (ids[0] if ids else -1)
        for e in range(self._n):
            if e == nxt:
                yield self._info(e, j)
                j += 1
                nxt = ids[j] if j < len(ids) else -1
            else:
                yield _NO_INFO

try:  # pragma: no cover - SB3 is not part of this image
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except ImportError:  # pragma: no cover
    _VecEnvBase = object


class AviaryVecEnv(_VecEnvBase):
    """SB3 VecEnv over one batched aviary (HoverAviary / MultiRaceAviary of this package)."""

    def __init__(self, env, as_torch=False, zero_copy=None, ring=3, packed=None, terminal_rows=None, direct=None):
        self.env = env
        self.num_envs = env.num_envs
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self.render_mode = None
        self.as_torch = as_torch
        self._actions = None
        self._seed = None
        # packed host path: numpy outputs of an env that can write into caller buffers (None: auto)
        self._packed = (not as_torch) and hasattr(env, "bind_outputs") and packed is not False
        # direct: the step kernel reads / writes the pinned host blocks itself (adrp_vec_step)
        lib = _lib.load() if self._packed and env._obs.is_cuda else None
        self._direct = self._packed and direct is not False and getattr(lib, "adrp_vec_step", None) is not None
        # zero_copy (None: auto) - views of the ring blocks on the direct path, copies otherwise
        self.zero_copy = self._direct if zero_copy is None else bool(zero_copy)
        if terminal_rows is not None:   # initial terminal-row capacity of the packed copy (it grows)
            self._cap_req = max(1, min(self.num_envs, int(terminal_rows)))
        if self._direct:
            self._bind_direct(max(1, min(int(ring), abi.VEC_SLOTS)))
        elif self._packed:
            self._bind_packed(max(1, int(ring)))
        if _VecEnvBase is not object:  # pragma: no cover
            _VecEnvBase.__init__(self, self.num_envs, self.observation_space, self.action_space)

    def _bind_packed(self, ring):
        """[obs | reward | terminated | truncated | done count | done env ids | terminal rows] in one
        device buffer: the env writes the first four into it (bind_outputs) and its terminal
        observations into a separate device buffer; after the step, adrp_compact_rows gathers the
        finished envs' ids and terminal rows behind the flags, so a step's outputs reach the host in
        ONE asynchronous copy of about the obs size and one wait (not the whole terminal-obs batch)"""
        env, E = self.env, self.num_envs
        obs_shape = tuple(env._obs.shape)
        dev = env._obs.device
        rf = int(np.prod(obs_shape[1:]))
        nobs = E * rf * 4
        self._rf = rf
        # terminal rows the copy carries (more: a second copy that step, and the region grows)
        self._cap = getattr(self, "_cap_req", min(E, max(64, E // 16)))
        a16 = lambda x: (x + 15) // 16 * 16   # noqa: E731
        o_rew, o_term, o_trunc = nobs, nobs + 4 * E, nobs + 5 * E
        o_cnt = a16(nobs + 6 * E)
        o_idx = o_cnt + 16
        o_rows = a16(o_idx + 4 * E)
        self._nbytes = a16(o_rows + 4 * rf * self._cap)
        old = getattr(self, "_dev", None), getattr(self, "_tobs_dev", None)
        self._dev = torch.zeros(self._nbytes, dtype=torch.uint8, device=dev)
        self._tobs_dev = torch.zeros(obs_shape, dtype=torch.float32, device=dev)
        if old[0] is not None:   # a re-bind (larger terminal-row region): the current outputs move over
            self._dev[:o_cnt].copy_(old[0][:o_cnt])
            self._tobs_dev.copy_(old[1])
        d = self._dev
        env.bind_outputs(d[:nobs].view(torch.float32).view(obs_shape), d[o_rew:o_term].view(torch.float32),
                         d[o_term:o_trunc].view(torch.bool), d[o_trunc:o_trunc + E].view(torch.bool),
                         tobs=self._tobs_dev)
        base = d.data_ptr()
        self._offs = (o_term, o_trunc, o_cnt, o_idx, o_rows)
        lib = _lib.load() if dev.type == "cuda" else None
        self._compact = getattr(lib, "adrp_compact_rows", None)
        # raw stream-ordered copies + one stream wait (no framework dispatch per copy) when the library has them
        self._raw = lib if getattr(lib, "adrp_memcpy_async", None) is not None else None
        self._compact_args = (base + o_term, base + o_trunc, self._tobs_dev.data_ptr(), E, rf, self._cap,
                              base + o_cnt, base + o_idx, base + o_rows)
        pin = dev.type == "cuda"
        self._host = [torch.zeros(self._nbytes, dtype=torch.uint8, pin_memory=pin) for _ in range(ring)]
        self._slot = 0
        self._views = []
        for h in self._host:
            hn = h.numpy()
            self._views.append((hn[:nobs].view(np.float32).reshape(obs_shape), hn[o_rew:o_term].view(np.float32),
                                hn[o_term:o_trunc].view(np.bool_), hn[o_trunc:o_trunc + E].view(np.bool_),
                                hn[o_cnt:o_cnt + 4].view(np.int32), hn[o_idx:o_idx + 4 * E].view(np.int32),
                                hn[o_rows:o_rows + 4 * rf * self._cap].view(np.float32).reshape((self._cap,) + obs_shape[1:])))
        act_shape = tuple(getattr(env, "_act_shape", (E,) + tuple(self.action_space.shape)))
        self._act_host = torch.zeros(act_shape, dtype=torch.float32, pin_memory=pin)
        self._act_np = self._act_host.numpy()
        self._act_dev = torch.zeros(act_shape, dtype=torch.float32, device=dev)
        # the copies and the step run on the env device's current stream, which need not be the current
        # device's: the event is created on and recorded into that stream
        if pin:
            with torch.cuda.device(dev):
                self._event = torch.cuda.Event()
        else:
            self._event = None

    def _bind_direct(self, ring):
        """adrp_vec_bind of `ring` pinned host blocks [obs | reward | terminated | truncated | done |
        count | done env ids | terminal rows] and the pinned action block; the step's own flags,
        terminal obs and the compaction's id scratch stay on the device"""
        env, E = self.env, self.num_envs
        obs_shape = tuple(env._obs.shape)
        dev = env._obs.device
        rf = int(np.prod(obs_shape[1:]))
        self._rf = rf
        self._cap = getattr(self, "_cap_req", min(E, max(64, E // 16)))
        a16 = lambda x: (x + 15) // 16 * 16   # noqa: E731
        nobs = E * rf * 4
        o_rew = nobs
        o_term = a16(o_rew + 4 * E)
        o_trunc = o_term + E
        o_done = o_trunc + E
        o_cnt = a16(o_done + E)
        o_idx = o_cnt + 16
        o_rows = a16(o_idx + 4 * E)
        self._nbytes = a16(o_rows + 4 * rf * self._cap)
        self._term_dev = torch.zeros(E, dtype=torch.uint8, device=dev)
        self._trunc_dev = torch.zeros(E, dtype=torch.uint8, device=dev)
        self._tobs_dev = torch.zeros(obs_shape, dtype=torch.float32, device=dev)
        self._idx_dev = torch.zeros(E, dtype=torch.int32, device=dev)
        act_shape = tuple(env._act_shape)
        if getattr(self, "_act_host", None) is None or tuple(self._act_host.shape) != act_shape:
            self._act_host = torch.zeros(act_shape, dtype=torch.float32, pin_memory=True)
            self._act_np = self._act_host.numpy()
        self._host = [torch.zeros(self._nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(ring)]
        self._views = []
        lib = _lib.load()
        h = env.h.h
        for k, hb in enumerate(self._host):
            hn = hb.numpy()
            base = hb.data_ptr()
            io = abi.AdrpVecIO(act=self._act_host.data_ptr(), obs=base, rew=base + o_rew, term=base + o_term,
                               trunc=base + o_trunc, done=base + o_done, count=base + o_cnt, idx=base + o_idx,
                               rows=base + o_rows, cap=self._cap, term_dev=self._term_dev.data_ptr(),
                               trunc_dev=self._trunc_dev.data_ptr(), tobs_dev=self._tobs_dev.data_ptr(),
                               idx_dev=self._idx_dev.data_ptr())
            if lib.adrp_vec_bind(h, k, ctypes.byref(io)) != 0:
                raise _lib.AdrpError(f"adrp_vec_bind: {lib.adrp_last_error(h).decode()}")
            self._views.append((hn[:nobs].view(np.float32).reshape(obs_shape), hn[o_rew:o_rew + 4 * E].view(np.float32),
                                hn[o_term:o_trunc].view(np.bool_), hn[o_trunc:o_done].view(np.bool_),
                                hn[o_done:o_done + E].view(np.bool_), hn[o_cnt:o_cnt + 4].view(np.int32),
                                hn[o_idx:o_idx + 4 * E].view(np.int32),
                                hn[o_rows:o_rows + 4 * rf * self._cap].view(np.float32).reshape((self._cap,) + obs_shape[1:])))
        self._slot = 0
        self._vec_step = lib.adrp_vec_step
        self._h = h
        self._dev_index = dev.index

    def _step_wait_direct(self):
        a = self._actions
        if isinstance(a, torch.Tensor):
            self._act_host.copy_(a.reshape(self._act_host.shape))
        else:
            self._act_np[...] = np.asarray(a, np.float32).reshape(self._act_np.shape)
        self._slot = (self._slot + 1) % len(self._host)
        if self._vec_step(self._h, self._slot, _lib._raw_stream(self._dev_index)) != 0:
            raise _lib.AdrpError(f"adrp_vec_step: {_lib.load().adrp_last_error(self._h).decode()}")
        obs, rew, term, trunc, done, cnt, idx_all, rows = self._views[self._slot]
        n = int(cnt[0])
        idx = idx_all[:n]
        if n <= self._cap:
            tobs = rows[:n]
        else:   # more finished envs than the block carries: the rest from the device, and a larger
            # terminal-row region from the next step on (the blocks are re-bound; the env state stays)
            rest = torch.as_tensor(idx[self._cap:], dtype=torch.long, device=self._tobs_dev.device)
            tobs = np.concatenate([rows.copy(), self._tobs_dev[rest].cpu().numpy()])
            self._cap_req = min(self.num_envs, max(2 * self._cap, n + n // 4))
            idx = idx.copy()
            self._bind_direct(len(self._host))
        infos = _StepInfos(self.num_envs, idx, tobs, trunc[idx] & ~term[idx])
        if not self.zero_copy:
            obs, rew, done = obs.copy(), rew.copy(), done.copy()
            infos = _StepInfos(self.num_envs, idx.copy(), tobs.copy(), trunc[idx] & ~term[idx])
        return obs, rew, done, infos

    # ---- conversion ----
    def _out(self, x):
        return x if self.as_torch else x.detach().cpu().numpy()

    # ---- VecEnv API ----
    def reset(self):
        seed, self._seed = self._seed, None
        obs, _ = self.env.reset(seed=seed)
        if self._direct:
            return obs.cpu().numpy()
        if self._packed:
            with self._on_device():
                o = self._copy_out()[0]
            return o if self.zero_copy else o.copy()
        return self._out(obs).copy() if not self.as_torch else obs.clone()

    def step_async(self, actions):
        self._actions = actions

    def _copy_out(self):
        """one async device -> pinned copy of the packed outputs, one wait (on the env device's stream)"""
        self._slot = (self._slot + 1) % len(self._host)
        h = self._host[self._slot]
        if self._raw is not None:
            st = _lib._raw_stream(self._dev.device.index)
            if self._raw.adrp_memcpy_async(h.data_ptr(), self._dev.data_ptr(), self._nbytes, 2, st) != 0 or \
                    self._raw.adrp_stream_synchronize(st) != 0:
                raise _lib.AdrpError(f"packed copy: {self._raw.adrp_last_error(None).decode()}")
            return self._views[self._slot]
        h.copy_(self._dev, non_blocking=True)
        if self._event is not None:
            self._event.record(torch.cuda.current_stream(self._dev.device))
            self._event.synchronize()
        return self._views[self._slot]

    def _act_in(self, actions):
        """numpy / host actions -> the persistent device action buffer through pinned staging"""
        if isinstance(actions, torch.Tensor) and actions.device == self._act_dev.device:
            return actions
        self._act_np[...] = np.asarray(actions, np.float32).reshape(self._act_np.shape)
        if self._raw is not None:
            if self._raw.adrp_memcpy_async(self._act_dev.data_ptr(), self._act_host.data_ptr(), self._act_host.nbytes, 1,
                                           _lib._raw_stream(self._act_dev.device.index)) != 0:
                raise _lib.AdrpError(f"action copy: {self._raw.adrp_last_error(None).decode()}")
            return self._act_dev
        self._act_dev.copy_(self._act_host, non_blocking=True)
        return self._act_dev

    def _gather_terminal(self):
        """the finished envs' ids and terminal rows into the packed buffer (stream-ordered after the
        step); a build without adrp_compact_rows (CPU stand-ins, old libraries) gathers with torch"""
        if self._compact is not None and self._dev.is_cuda:
            rc = self._compact(*self._compact_args, _lib._raw_stream(self._dev.device.index))
            if rc != 0:
                raise _lib.AdrpError(f"adrp_compact_rows: {_lib.load().adrp_last_error(None).decode()}")
            return
        E, rf, cap, d = self.num_envs, self._rf, self._cap, self._dev
        o_term, o_trunc, o_cnt, o_idx, o_rows = self._offs
        ids = torch.nonzero(d[o_term:o_term + E].bool() | d[o_trunc:o_trunc + E].bool()).flatten().to(torch.int32)
        n = int(ids.numel())
        d[o_cnt:o_cnt + 4].view(torch.int32)[0] = n
        d[o_idx:o_idx + 4 * E].view(torch.int32)[:n] = ids
        m = min(n, cap)
        rows = d[o_rows:o_rows + 4 * rf * cap].view(torch.float32).view(cap, rf)
        rows[:m] = self._tobs_dev.reshape(E, rf)[ids[:m].long()]

    def _step_wait_packed(self):
        self.env.step(self._act_in(self._actions))
        self._gather_terminal()
        obs, rew, term, trunc, cnt, idx_all, rows = self._copy_out()
        n = int(cnt[0])
        idx = idx_all[:n].copy()
        if n <= self._cap:
            tobs = rows[:n].copy()
        else:   # more finished envs than the copy carries: the rest by a second copy, and a larger
            # terminal-row region from the next step on (the outputs are re-bound; the env state stays)
            rest = torch.as_tensor(idx[self._cap:], dtype=torch.long, device=self._tobs_dev.device)
            tobs = np.concatenate([rows.copy(), self._tobs_dev[rest].cpu().numpy()])
            self._cap_req = min(self.num_envs, max(2 * self._cap, n + n // 4))
            self._bind_packed(len(self._host))
        done = term | trunc
        # the dicts are built on demand from the copied terminal rows
        infos = _StepInfos(self.num_envs, idx, tobs, (trunc & ~term)[idx])
        if not self.zero_copy:
            obs, rew = obs.copy(), rew.copy()
        return obs, rew, done, infos

    def _on_device(self):
        """the env's device current while the raw C-ABI copies / compaction run: a null (default)
        stream names the current device's, so the work then lands on the env's"""
        dev = self.env._obs.device
        return torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()

    def step_wait(self):
        if self._direct:   # (adrp_vec_step makes the handle's device current itself)
            return self._step_wait_direct()
        if self._packed:
            with self._on_device():
                return self._step_wait_packed()
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


def HoverAviaryVec(n_envs=1, as_torch=False, zero_copy=None, **env_kwargs):
    """``make_vec_env(HoverAviary, env_kwargs=..., n_envs=...)`` counterpart"""
    from .envs.hover import HoverAviary
    return AviaryVecEnv(HoverAviary(num_envs=n_envs, **env_kwargs), as_torch=as_torch, zero_copy=zero_copy)


def MultiRaceAviaryVec(n_envs=1, as_torch=False, zero_copy=None, **env_kwargs):
    from .envs.race import MultiRaceAviary
    return AviaryVecEnv(MultiRaceAviary(num_envs=n_envs, **env_kwargs), as_torch=as_torch, zero_copy=zero_copy)
