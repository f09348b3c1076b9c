"""Env sharding over the GPUs of one node (one process per GPU, torch.distributed).

Envs never interact, so the shard unit is the env: rank r owns the
contiguous global env range [offset, offset + count) and steps it with its own handle.
Reset draws are keyed by the *global* env id (Philox counter {env_offset + e, episode,
tag, idx}), so a sharded run produces bit-identical trajectories to one big run.

The step itself has no collective.  ``gather`` reassembles the observation batch
(obs, reward, terminated, truncated) for a learner: an all-gather over RCCL/xGMI
(backend "nccl") on the GPU, or gloo on the CPU (tests).  Ragged shards are padded
to the largest shard for the collective and trimmed afterwards.

``packed=True`` is the step-path form: the env writes obs / reward / flags straight into
this rank's slot of one preallocated byte buffer ([obs | reward | terminated | truncated],
16-byte aligned segments, padded to the largest shard), and ``step_gather`` is env.step + ONE
``all_gather_into_tensor`` into a preallocated receive buffer: no allocation, no copy, no
host sync, so a whole step + gather can be captured in a HIP graph.  The gathered views are
per rank: obs [world, max_count, N, D], reward / flags [world, max_count] (rows beyond a
rank's count are padding).
"""
from typing import NamedTuple

import torch
import torch.distributed as dist


def shard_range(global_envs: int, world: int, rank: int):
    """Contiguous partition, the remainder spread over the first ranks -> (offset, count)."""
    if global_envs < world:
        raise ValueError(f"{global_envs} envs cannot be sharded over {world} ranks")
    base, extra = divmod(global_envs, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


class Gathered(NamedTuple):
    """global outputs of one packed step: views into the receive buffer, one row block per rank"""
    obs: torch.Tensor      # [world, max_count, N, D] float32
    rew: torch.Tensor      # [world, max_count] float32
    term: torch.Tensor     # [world, max_count] bool
    trunc: torch.Tensor    # [world, max_count] bool
    counts: list           # live rows per rank


def _a16(n):
    return (n + 15) // 16 * 16


class ShardedAviary:
    """One shard of a node-wide vectorised aviary.

    ``make_env(num_envs=..., env_offset=...)`` builds the per-rank env (e.g.
    ``functools.partial(HoverAviary, device=local_rank, seed=...)``); every rank must pass
    the same remaining arguments so the shards form one logical batch."""

    def __init__(self, global_envs: int, make_env, group=None, packed: bool = False):
        if not dist.is_initialized():
            raise RuntimeError("ShardedAviary needs torch.distributed to be initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.global_envs = int(global_envs)
        self.offset, self.count = shard_range(self.global_envs, self.world, self.rank)
        self.counts = [shard_range(self.global_envs, self.world, r)[1] for r in range(self.world)]
        self.max_count = max(self.counts)
        self.env = make_env(num_envs=self.count, env_offset=self.offset)
        self.num_envs = self.count
        self.observation_space = getattr(self.env, "observation_space", None)
        self.action_space = getattr(self.env, "action_space", None)
        self._gbuf = None
        self.packed = bool(packed)
        if self.packed:
            self._bind_packed()

    def _bind_packed(self):
        env, M, c = self.env, self.max_count, self.count
        row = tuple(env._obs.shape[1:])
        nobs = M * int(torch.Size(row).numel()) * 4
        self._o_rew = _a16(nobs)
        self._o_term = self._o_rew + _a16(4 * M)
        self._o_trunc = self._o_term + _a16(M)
        self._seg = self._o_trunc + _a16(M)
        dev = env._obs.device
        self._send = torch.zeros(self._seg, dtype=torch.uint8, device=dev)
        self._recv = torch.zeros(self.world * self._seg, dtype=torch.uint8, device=dev)
        s = self._send
        env.bind_outputs(s[:nobs].view(torch.float32).view((M,) + row)[:c],
                         s[self._o_rew:self._o_rew + 4 * M].view(torch.float32)[:c],
                         s[self._o_term:self._o_term + M].view(torch.bool)[:c],
                         s[self._o_trunc:self._o_trunc + M].view(torch.bool)[:c])
        R = self._recv.view(self.world, self._seg)
        self.gathered = Gathered(R[:, :nobs].view(torch.float32).view((self.world, M) + row),
                                 R[:, self._o_rew:self._o_rew + 4 * M].view(torch.float32),
                                 R[:, self._o_term:self._o_term + M].view(torch.bool),
                                 R[:, self._o_trunc:self._o_trunc + M].view(torch.bool), list(self.counts))

    def _all_gather_packed(self):
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
        elif self._send.is_cuda:   # gloo (tests): staged through host memory
            out = torch.zeros(self._recv.numel(), dtype=torch.uint8)
            dist.all_gather(list(out.chunk(self.world)), self._send.cpu(), group=self.group)
            self._recv.copy_(out)
        else:
            dist.all_gather(list(self._recv.chunk(self.world)), self._send, group=self.group)

    def step_gather(self, action) -> Gathered:
        """packed mode: one env.step of this shard, then one all-gather of every rank's outputs into
        the preallocated receive buffer (graph-capturable on RCCL: nothing allocated, no host sync)"""
        if not self.packed:
            raise RuntimeError("step_gather needs ShardedAviary(..., packed=True)")
        self.step(action)
        self._all_gather_packed()
        return self.gathered

    def gather_packed(self) -> Gathered:
        """packed mode: all-gather the outputs the last step / reset left in the send buffer"""
        self._all_gather_packed()
        return self.gathered

    def local_slice(self, x):
        """rows of a global [global_envs, ...] batch that belong to this rank"""
        return x[self.offset:self.offset + self.count]

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, action):
        """action: this shard's [count, ...] batch, or the global [global_envs, ...] batch."""
        if action.shape[0] == self.global_envs and self.global_envs != self.count:
            action = self.local_slice(action)
        return self.env.step(action)

    def _gather_one(self, x):
        x = x.contiguous()
        if x.shape[0] != self.max_count:
            pad = torch.zeros((self.max_count - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            x = torch.cat([x, pad])
        out = torch.empty((self.world * self.max_count,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, x, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world)), x, group=self.group)
        if all(c == self.max_count for c in self.counts):
            return out
        return torch.cat([out[r * self.max_count:r * self.max_count + c] for r, c in enumerate(self.counts)])

    def gather(self, obs, rew, term, trunc):
        """All-gather one step's outputs into global batches on every rank.

        obs, reward and the two flags travel as one packed float32 buffer (one
        collective per step); flags come back as torch.bool."""
        E = obs.shape[0]
        packed = torch.cat([obs.reshape(E, -1).float(), rew.reshape(E, 1).float(),
                            term.reshape(E, 1).float(), trunc.reshape(E, 1).float()], dim=1)
        g = self._gather_one(packed)
        D = packed.shape[1] - 3
        return (g[:, :D].reshape((self.global_envs,) + tuple(obs.shape[1:])), g[:, D].contiguous(),
                g[:, D + 1] != 0, g[:, D + 2] != 0)

    def close(self):
        if hasattr(self.env, "close"):
            self.env.close()
