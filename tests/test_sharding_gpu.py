"""BASELINE config 5 on the HIP path (one GPU): the 32,768-env level3 / COMPETE / 4-drone / PYB_DW /
disturbed race sharded as 8 handles of 4,096 envs with env_offset = r * 4096 (what rank r of an
8-GPU job builds, gym_pybullet_adrp_amd/sharding.py) against ONE 32,768-env handle.  Reset and
sub-step draws are Philox-keyed by the global env id, so the shards must reproduce the single batch
bit for bit: obs, reward, terminated, truncated, terminal obs and the full SoA state, 40 env.steps
with auto-resets (reference step: envs/MultiRaceAviary.py:171-270).
The packed-buffer gather of ShardedAviary (the learner-side reassembly) is checked on the same
tensors with a one-rank gloo group.  Needs an MI355X: -m gpu."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics, RaceMode  # noqa: E402

SHARDS, E_SHARD, N = 8, 4096, 4
E_GLOBAL = SHARDS * E_SHARD
STEPS = 40


def _make(num_envs, env_offset):
    return MultiRaceAviary("level3", num_drones=N, physics=Physics.PYB_DW, racemode=RaceMode.COMPETE,
                           num_envs=num_envs, env_offset=env_offset, seed=2024, autoreset=True, reward="wrapper")


def _actions(obs0, dev):
    """FULLSTATE targets: start + U(+-0.3) m for 3/4 of the envs (config 3/4's synthetic actions);
    the rest outside the level3 bounds or at the ground, so drones are eliminated, envs terminate
    and auto-reset inside the run.  Re-drawn every 10 steps."""
    g = torch.Generator(device=dev)
    g.manual_seed(55)
    out = []
    for k in range(STEPS // 10):
        tgt = obs0[..., :3] + torch.rand(obs0.shape[:2] + (3,), generator=g, device=dev) * 0.6 - 0.3
        tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
        wild = torch.rand(obs0.shape[:2] + (3,), generator=g, device=dev) * torch.tensor([8.0, 8.0, 2.6], device=dev) \
            - torch.tensor([4.0, 4.0, 0.0], device=dev)
        sel = (torch.arange(obs0.shape[0], device=dev) % 4 == k % 4)[:, None, None]
        tgt = torch.where(sel, wild, tgt)
        a = torch.cat([tgt, torch.zeros(obs0.shape[:2] + (1,), device=dev)], -1).contiguous()
        out += [a] * 10
    return out


def test_config5_shards_bit_identical_to_one_batch():
    one = _make(E_GLOBAL, 0)
    shards = [_make(E_SHARD, r * E_SHARD) for r in range(SHARDS)]
    dev = one.device
    obs1, _ = one.reset()
    obs_s = torch.cat([s.reset()[0] for s in shards])
    assert torch.equal(obs1, obs_s)
    # the reset states differ per env (global-id keyed draws), not per shard-local index
    assert not torch.equal(obs_s[:E_SHARD], obs_s[E_SHARD:2 * E_SHARD])
    acts = _actions(obs1.clone(), dev)
    ep_field = one.state_field_names()[1].index("episode")
    ep_prev = one.get_state()[1][ep_field].reshape(E_GLOBAL, N)[:, 0].clone()
    done_total = 0
    for k in range(STEPS):
        o1, r1, te1, tr1, info1 = one.step(acts[k])
        outs = [s.step(acts[k][r * E_SHARD:(r + 1) * E_SHARD]) for r, s in enumerate(shards)]
        assert torch.equal(o1, torch.cat([o[0] for o in outs])), f"obs differ at step {k}"
        assert torch.equal(r1, torch.cat([o[1] for o in outs])), f"reward differs at step {k}"
        assert torch.equal(te1, torch.cat([o[2] for o in outs])), f"terminated differs at step {k}"
        assert torch.equal(tr1, torch.cat([o[3] for o in outs])), f"truncated differs at step {k}"
        done = te1 | tr1
        tob1 = info1["terminal_observation"][done]
        tobs = torch.cat([o[4]["terminal_observation"] for o in outs])[done]
        assert torch.equal(tob1, tobs), f"terminal obs differ at step {k}"
        # full-size property: exactly the done envs start a new episode in the same launch
        ep = one.get_state()[1][ep_field].reshape(E_GLOBAL, N)[:, 0].clone()
        assert torch.equal(ep - ep_prev, done.to(ep.dtype)), f"episode counters vs done flags at step {k}"
        ep_prev = ep
        done_total += int(done.sum())
        assert torch.isfinite(o1).all()
    assert done_total > 0, "the run should exercise termination + auto-reset"
    f1, i1 = one.get_state()
    fs = torch.cat([s.get_state()[0] for s in shards], 1)
    is_ = torch.cat([s.get_state()[1] for s in shards], 1)
    assert torch.equal(i1, is_)
    np.testing.assert_array_equal(f1.cpu().numpy(), fs.cpu().numpy())    # NaN == NaN (D-term memory)
    for s in shards:
        s.close()
    one.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_packed_gather_one_rank():
    """ShardedAviary(packed=True): the env writes obs / reward / flags straight into the rank's slot
    of the preallocated send buffer; step_gather() is env.step + one all-gather with no allocation,
    and its global views equal the env's own outputs (world 1, gloo)."""
    import functools
    import torch.distributed as dist
    from gym_pybullet_adrp_amd.sharding import ShardedAviary
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        E = 256
        sh = ShardedAviary(E, functools.partial(MultiRaceAviary, "level3", num_drones=N, physics=Physics.PYB_DW,
                                                racemode=RaceMode.COMPETE, seed=5), packed=True)
        ref = MultiRaceAviary("level3", num_drones=N, physics=Physics.PYB_DW, racemode=RaceMode.COMPETE, seed=5,
                              num_envs=E)
        obs, _ = sh.reset()
        obs_r, _ = ref.reset()
        assert torch.equal(obs, obs_r)
        act = torch.cat([obs_r[..., :3] + 0.1, torch.zeros_like(obs_r[..., :1])], -1).contiguous()
        for _ in range(5):
            g = sh.step_gather(act)
            o, r, te, tr, _ = ref.step(act)
            assert torch.equal(g.obs.reshape(E, N, -1), o)
            assert torch.equal(g.rew.reshape(E), r)
            assert torch.equal(g.term.reshape(E), te) and torch.equal(g.trunc.reshape(E), tr)
        sh.close()
        ref.close()
    finally:
        dist.destroy_process_group()


def _nccl_world1():
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    return dist


def test_packed_gather_rccl_graph():
    """the north star's RCCL obs all-gather on the one GPU a box has: a world-1 "nccl" (RCCL) group,
    BASELINE config 5's per-GPU workload (level3 / COMPETE / 4 drones / PYB_DW / disturbances, 4,096
    envs, auto-reset) in ShardedAviary(packed=True); step_gather (env.step + all_gather_into_tensor of
    the packed send buffer) captured in ONE HIP graph and replayed 20 times: after every replay the
    gathered obs / reward / flags equal, bit for bit, an unsharded env stepped eagerly on the same
    actions (sharding.py:98-115)"""
    import functools
    from gym_pybullet_adrp_amd.sharding import ShardedAviary
    dist = _nccl_world1()
    try:
        E = E_SHARD
        make = functools.partial(MultiRaceAviary, "level3", num_drones=N, physics=Physics.PYB_DW,
                                 racemode=RaceMode.COMPETE, seed=2024, autoreset=True, reward="wrapper")
        sh = ShardedAviary(E, make, packed=True)
        ref = make(num_envs=E)
        assert sh.env.kernel_name == ref.kernel_name == "race_step<f64,PYB_DW,G4,Q4>"
        obs, _ = sh.reset()
        obs_r, _ = ref.reset()
        assert torch.equal(obs, obs_r)
        acts = _actions(obs_r.clone(), obs_r.device)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            sh.step_gather(acts[0])                  # warm-up outside the capture (step 0)
        torch.cuda.current_stream().wait_stream(side)
        ref.step(acts[0])
        a_buf = acts[1].clone()
        # no RCCL work pending and a thread-local capture: the ProcessGroupNCCL watchdog's event
        # queries must not meet a global-mode capture (BENCH_r04's abort, bench.quiesce_collectives)
        import bench
        bench.quiesce_collectives()
        g = torch.cuda.CUDAGraph()
        with bench.capture_graph(g):
            out = sh.step_gather(a_buf)
        done = 0
        for k in range(1, 21):
            a_buf.copy_(acts[k])
            g.replay()
            o, r, te, tr, _ = ref.step(acts[k])
            torch.cuda.synchronize()
            assert torch.equal(out.obs.reshape(E, N, -1), o), f"gathered obs differ at replay {k}"
            assert torch.equal(out.rew.reshape(E), r)
            assert torch.equal(out.term.reshape(E), te) and torch.equal(out.trunc.reshape(E), tr)
            done += int((te | tr).sum())
        assert done > 0, "the replays should include auto-resets"
        sh.close()
        ref.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("refuse", [False, True])
def test_bench_gather_record_graph_and_eager_fallback(refuse):
    """bench.py's config-5 all-gather record on a world-1 RCCL group: the graph-captured form (no
    graph_capture_error), and with the capture refused the eager fallback (one launch + one
    collective per step, timed under barriers) that bench.py takes then"""
    import bench
    dist = _nccl_world1()
    try:
        rec = bench.gather_record_world1(0, 64, 8, precision="fp64", E=512, refuse_capture=refuse)
        assert rec["world"] == 1 and rec["backend"] == "nccl" and rec["value"] > 0
        if refuse:
            assert "graph_capture_error" in rec and rec["timed_region"].endswith("eager steps (step kernel + RCCL all-gather each)")
        else:
            assert "graph_capture_error" not in rec and "HIP graph" in rec["timed_region"]
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_hover_ragged_shards_bit_identical(precision):
    """One env's step does not depend on its batch (envs/BaseAviary.py:262-387 steps each env on
    its own): HoverAviary at BASELINE config 2's size, E = 4,096 on ONE handle (the LDS-staged kernel
    with its reset-helper wave, E % 64 == 0) against two ragged env_offset shards of 1,000 + 3,096
    (the row-store kernel, partial last wave).  The hover TUs contract a*b+c only within one source
    expression (csrc/Makefile CONTRACT), so obs, reward, flags, terminal obs and the whole SoA state
    are bit for bit equal over 60 env.steps with auto-resets."""
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    kw = dict(precision=precision, seed=4242, initial_xyzs=[0, 0, 1.0],
              init_noise={"xyz": 0.1, "rpy": 0.3, "vel": 0.3, "omega": 1.0})
    one = HoverAviary(num_envs=4096, **kw)
    parts = [HoverAviary(num_envs=1000, env_offset=0, **kw), HoverAviary(num_envs=3096, env_offset=1000, **kw)]
    cut = [0, 1000, 4096]
    o1, _ = one.reset()
    os_ = torch.cat([p.reset()[0] for p in parts])
    assert torch.equal(o1, os_)
    rng = np.random.default_rng(17)
    done = 0
    for k in range(60):
        a = rng.uniform(-1, 1, (4096, 1, 4)).astype(np.float32)
        if k % 20 >= 12:
            a[::3] = 1.0                       # climb out of bounds: truncations, auto-resets
        at = torch.from_numpy(a).to(one.device)
        o1, r1, te1, tr1, i1 = one.step(at)
        outs = [p.step(at[cut[j]:cut[j + 1]].contiguous()) for j, p in enumerate(parts)]
        assert torch.equal(o1, torch.cat([o[0] for o in outs])), f"obs differ at step {k}"
        assert torch.equal(r1, torch.cat([o[1] for o in outs])), f"reward differs at step {k}"
        assert torch.equal(te1, torch.cat([o[2] for o in outs])) and torch.equal(tr1, torch.cat([o[3] for o in outs]))
        d = te1 | tr1
        tob = torch.cat([o[4]["terminal_observation"] for o in outs])
        assert torch.equal(i1["terminal_observation"][d], tob[d]), f"terminal obs differ at step {k}"
        done += int(d.sum())
    assert done > 0, "the run should exercise auto-reset"
    f1, n1 = one.get_state()
    fs = torch.cat([p.get_state()[0] for p in parts], 1)
    ns = torch.cat([p.get_state()[1] for p in parts], 1)
    assert torch.equal(n1, ns)
    np.testing.assert_array_equal(f1.cpu().numpy(), fs.cpu().numpy())
    for p in parts:
        p.close()
    one.close()


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_hover_one_env_shards_bit_identical(precision):
    """A one-env handle runs its env on the whole wave (csrc/hover_kernel.h SPLIT: three lanes take
    the obs row's three Euler angles): eight env_offset shards of ONE env each against the first eight
    envs of a 64-env batch (the LDS-staged kernel, one angle chain per lane) give the same obs,
    reward, flags, terminal obs and state bit for bit over 60 env.steps with auto-resets
    (envs/BaseAviary.py:262-387 steps each env on its own)."""
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    kw = dict(precision=precision, seed=977, initial_xyzs=[0, 0, 1.0],
              init_noise={"xyz": 0.1, "rpy": 0.3, "vel": 0.3, "omega": 1.0})
    full = HoverAviary(num_envs=64, **kw)
    ones = [HoverAviary(num_envs=1, env_offset=j, **kw) for j in range(8)]
    o64, _ = full.reset()
    assert torch.equal(o64[:8], torch.cat([p.reset()[0] for p in ones]))
    rng = np.random.default_rng(5)
    done = 0
    for k in range(60):
        a = rng.uniform(-1, 1, (64, 1, 4)).astype(np.float32)
        if k % 20 >= 12:
            a[::2] = 1.0                       # climb out of bounds: truncations, auto-resets
        at = torch.from_numpy(a).to(full.device)
        o, r, te, tr, info = full.step(at)
        outs = [p.step(at[j:j + 1].contiguous()) for j, p in enumerate(ones)]
        assert torch.equal(o[:8], torch.cat([x[0] for x in outs])), f"obs differ at step {k}"
        assert torch.equal(r[:8], torch.cat([x[1] for x in outs])), f"reward differs at step {k}"
        assert torch.equal(te[:8], torch.cat([x[2] for x in outs])) and torch.equal(tr[:8], torch.cat([x[3] for x in outs]))
        d = (te | tr)[:8]
        tob = torch.cat([x[4]["terminal_observation"] for x in outs])
        assert torch.equal(info["terminal_observation"][:8][d], tob[d]), f"terminal obs differ at step {k}"
        done += int(d.sum())
    assert done > 0, "the run should exercise auto-reset"
    f, n = full.get_state()
    np.testing.assert_array_equal(f[:, :8].cpu().numpy(), torch.cat([p.get_state()[0] for p in ones], 1).cpu().numpy())
    assert torch.equal(n[:, :8], torch.cat([p.get_state()[1] for p in ones], 1))
    for p in ones:
        p.close()
    full.close()
