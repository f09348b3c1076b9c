"""SB3 VecEnv adapter: host logic on the CPU with a scripted stand-in env (the real envs need
a GPU), and the real HoverAviary / MultiRaceAviary on the GPU (-m gpu)."""
import numpy as np
import pytest
import torch

from gym_pybullet_adrp_amd.utils.spaces import Box
from gym_pybullet_adrp_amd.vec_env import AviaryVecEnv


class _Scripted:
    """stand-in with the batched env interface: E envs, env 1 truncates at step 2, env 2
    terminates at step 3 (auto-reset semantics: obs holds the reset observation)"""

    def __init__(self, E=4, D=5):
        self.num_envs, self.D, self.k = E, D, 0
        self.observation_space = Box(low=-np.ones((1, D)), high=np.ones((1, D)), dtype=np.float32)
        self.action_space = Box(low=-np.ones((1, 4)), high=np.ones((1, 4)), dtype=np.float32)
        self.tobs = torch.zeros((E, 1, D))
        self.closed = False
        self._obs = torch.zeros((E, 1, D))
        self._rew = torch.zeros(E)
        self._term = torch.zeros(E, dtype=torch.bool)
        self._trunc = torch.zeros(E, dtype=torch.bool)
        self._act_shape = (E, 1, 4)
        self.actions = []

    def bind_outputs(self, obs, rew, term, trunc, tobs=None):      # the batched envs' contract
        want = ((self._obs, obs), (self._rew, rew), (self._term, term), (self._trunc, trunc))
        if tobs is not None:
            want += ((self.tobs, tobs),)
        for old, new in want:
            assert new.shape == old.shape and new.dtype == old.dtype and new.is_contiguous()
        self._obs, self._rew, self._term, self._trunc = obs, rew, term, trunc
        if tobs is not None:
            self.tobs = tobs

    def reset(self, seed=None):
        self._obs.zero_()
        return self._obs, {}

    def step(self, action):
        self.actions.append(torch.as_tensor(action).clone())
        self.k += 1
        E = self.num_envs
        self._obs.fill_(float(self.k))
        self._rew.copy_(torch.arange(E, dtype=torch.float32) * self.k)
        self._term.zero_()
        self._trunc.zero_()
        if self.k == 2:
            self._trunc[1] = True
            self.tobs[1] = 100.0
            self._obs[1] = -1.0
        if self.k == 3:
            self._term[2] = True
            self.tobs[2] = 200.0
        return self._obs, self._rew, self._term, self._trunc, {"answer": 42, "terminal_observation": self.tobs}

    def close(self):
        self.closed = True


@pytest.mark.parametrize("packed,zero_copy", [(False, False), (True, False), (True, True)])
def test_vecenv_protocol_and_infos(packed, zero_copy):
    venv = AviaryVecEnv(_Scripted(), packed=packed, zero_copy=zero_copy)
    assert venv._packed == packed
    assert venv.num_envs == 4 and venv.observation_space.shape == (1, 5)
    obs = venv.reset()
    assert isinstance(obs, np.ndarray) and obs.shape == (4, 1, 5)
    o, r, d, infos = venv.step(np.full((4, 1, 4), 0.5, np.float32))
    assert not d.any() and all(i == {} for i in infos)
    np.testing.assert_array_equal(venv.env.actions[-1].cpu().numpy(), np.full((4, 1, 4), 0.5, np.float32))
    if packed:
        with pytest.raises(TypeError):        # the shared empty info of a running env is read-only
            infos[0]["x"] = 1
    o, r, d, infos = venv.step(np.zeros((4, 1, 4), np.float32))
    np.testing.assert_array_equal(d, [False, True, False, False])
    assert infos[1]["TimeLimit.truncated"] is True
    np.testing.assert_array_equal(infos[1]["terminal_observation"], np.full((1, 5), 100.0))
    np.testing.assert_array_equal(o[1], np.full((1, 5), -1.0))     # already the reset observation
    o_prev = o
    o, r, d, infos = venv.step(np.zeros((4, 1, 4), np.float32))
    assert d[2] and infos[2]["TimeLimit.truncated"] is False
    np.testing.assert_array_equal(infos[2]["terminal_observation"], np.full((1, 5), 200.0))
    np.testing.assert_array_equal(o_prev[1], np.full((1, 5), -1.0))  # ring of 2 / copies: still valid
    np.testing.assert_array_equal(r, np.arange(4) * 3.0)
    assert venv.get_attr("num_envs") == [4] * 4 and venv.env_is_wrapped(object) == [False] * 4
    venv.close()
    assert venv.env.closed


def test_vecenv_torch_passthrough():
    venv = AviaryVecEnv(_Scripted(), as_torch=True)
    venv.reset()
    o, r, d, info = venv.step(torch.zeros((4, 1, 4)))
    assert isinstance(o, torch.Tensor) and d.dtype == torch.bool and "terminal_observation" in info


@pytest.mark.gpu
def test_hover_and_race_vecenv_on_gpu():
    from gym_pybullet_adrp_amd.vec_env import HoverAviaryVec, MultiRaceAviaryVec
    v = HoverAviaryVec(n_envs=64, seed=1)
    obs = v.reset()
    assert obs.shape == (64, 1, 72)
    for _ in range(300):   # past the 8 s limit: every env truncates once (242 steps)
        obs, rew, done, infos = v.step(np.random.uniform(-1, 1, (64, 1, 4)).astype(np.float32))
    assert obs.shape == (64, 1, 72) and rew.shape == (64,)
    v.close()
    r = MultiRaceAviaryVec(n_envs=32, race_config="level0", num_drones=2)
    obs = r.reset()
    assert obs.shape == (32, 2, 49)
    act = np.concatenate([obs[..., :3] + [0, 0, 0.5], np.zeros((32, 2, 1))], -1).astype(np.float32)
    obs, rew, done, infos = r.step(act)
    assert obs.shape == (32, 2, 49) and len(infos) == 32
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["hover", "race"])
def test_packed_host_path_matches_legacy(kind):
    """the host paths return the same thing: the direct path (adrp_vec_step: the kernels read / write
    pinned host blocks, views of a ring), the packed pinned-copy path and the per-tensor .cpu() path
    give the same obs, rewards, dones, terminal observations and TimeLimit.truncated (same seed, same
    actions); the direct and packed paths start with 2 terminal rows, so steps with more finished envs
    take the overflow copy and re-bind with a larger region"""
    from gym_pybullet_adrp_amd.vec_env import HoverAviaryVec, MultiRaceAviaryVec
    outs = []
    for mode in ("direct", "packed", "legacy"):
        if kind == "hover":
            v = HoverAviaryVec(n_envs=256, seed=3, initial_xyzs=[0, 0, 1.0], init_noise={"rpy": 0.3, "omega": 1.0})
        else:
            v = MultiRaceAviaryVec(n_envs=128, race_config="level3", num_drones=4, seed=3)
        v = type(v)(v.env, packed=mode != "legacy", direct=mode == "direct",
                    terminal_rows=2 if mode != "legacy" else None)
        assert v._packed == (mode != "legacy") and v._direct == (mode == "direct")
        assert v.zero_copy == (mode == "direct")
        obs = v.reset()
        rng = np.random.default_rng(0)
        seq = [obs.copy()]
        for k in range(60):
            if kind == "hover":
                a = rng.uniform(-1, 1, (256, 1, 4)).astype(np.float32)
            else:
                a = np.concatenate([obs[..., :3] + rng.uniform(-2, 2, obs[..., :3].shape), np.zeros(obs.shape[:2] + (1,))],
                                   -1).astype(np.float32)
            obs, rew, done, infos = v.step(a)
            seq.append((obs.copy(), rew.copy(), done.copy(),
                        [(bool(i.get("TimeLimit.truncated")), None if i.get("terminal_observation") is None
                          else np.array(i.get("terminal_observation"))) for i in infos]))
        outs.append(seq)
        if mode != "legacy":
            assert v._cap > 2   # more finished envs than terminal rows in some step: grown
        v.close()
    for other in outs[1:]:
        np.testing.assert_array_equal(outs[0][0], other[0])
        ndone = 0
        for (o1, r1, d1, i1), (o2, r2, d2, i2) in zip(outs[0][1:], other[1:]):
            np.testing.assert_array_equal(o1, o2)
            np.testing.assert_array_equal(r1, r2)
            np.testing.assert_array_equal(d1, d2)
            ndone += int(d1.sum())
            for (t1, x1), (t2, x2) in zip(i1, i2):
                assert t1 == t2 and (x1 is None) == (x2 is None)
                if x1 is not None:
                    np.testing.assert_array_equal(x1, x2)
        assert ndone > 0


@pytest.mark.gpu
def test_direct_ring_lifetime():
    """direct host path, ring of 3: the obs / rewards / dones a step returned are still intact two
    steps later (SB3 copies obs into its rollout buffer one step after), and the third step after
    reuses the block"""
    from gym_pybullet_adrp_amd.vec_env import HoverAviaryVec
    v = HoverAviaryVec(n_envs=128, seed=5, initial_xyzs=[0, 0, 1.0])
    assert v._direct and v.zero_copy and len(v._host) == 3
    v.reset()
    rng = np.random.default_rng(1)
    hist = []
    for k in range(6):
        o, r, d, _ = v.step(rng.uniform(-1, 1, (128, 1, 4)).astype(np.float32))
        hist.append((o, r, d, o.copy(), r.copy(), d.copy()))
        for j in range(max(0, k - 2), k + 1):          # the last three steps' views are intact
            np.testing.assert_array_equal(hist[j][0], hist[j][3])
            np.testing.assert_array_equal(hist[j][1], hist[j][4])
            np.testing.assert_array_equal(hist[j][2], hist[j][5])
    assert np.shares_memory(hist[0][0], hist[3][0])    # the ring wrapped
    v.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,rf,cap,p", [(4096, 72, 128, 0.004), (5000, 196, 64, 0.3), (1, 5, 1, 1.0), (3000, 7, 0, 0.5)])
def test_compact_rows_kernel(n, rf, cap, p):
    """adrp_compact_rows: count, ascending ids of term | trunc envs (several 1024-env chunks, more
    done envs than cap rows) and their rows, against torch"""
    import ctypes
    from gym_pybullet_adrp_amd import _lib
    g = torch.Generator().manual_seed(n)
    term = (torch.rand(n, generator=g) < p / 2).to(torch.uint8).cuda()
    trunc = (torch.rand(n, generator=g) < p / 2).to(torch.uint8).cuda()
    rows = torch.randn(n, rf, generator=g).cuda()
    cnt = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    idx = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    out = torch.zeros(max(cap, 1), rf, device="cuda")
    V = ctypes.c_void_p
    rc = _lib.load().adrp_compact_rows(V(term.data_ptr()), V(trunc.data_ptr()), V(rows.data_ptr()), n, rf, cap,
                                       V(cnt.data_ptr()), V(idx.data_ptr()), V(out.data_ptr()),
                                       V(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    ref = torch.nonzero((term | trunc).bool()).flatten()
    k = int(cnt.item())
    assert k == ref.numel()
    assert torch.equal(idx[:k].long().cpu(), ref.cpu())
    m = min(k, cap)
    assert torch.equal(out[:m].cpu(), rows[ref[:m]].cpu())


def test_step_infos_iteration_matches_indexing():
    """_StepInfos: iterating (what SB3's info-buffer update does over all envs) yields what indexing
    does, the same dict objects for finished envs and the shared empty mapping for the rest"""
    from gym_pybullet_adrp_amd.vec_env import _StepInfos
    idx = np.array([0, 3, 4, 9])
    tobs = np.arange(4 * 2, dtype=np.float32).reshape(4, 2)
    infos = _StepInfos(10, idx, tobs, np.array([True, False, True, False]))
    it = list(infos)
    assert len(it) == 10 and all(a is b for a, b in zip(it, [infos[i] for i in range(10)]))
    assert it[3]["TimeLimit.truncated"] is False and it[4]["TimeLimit.truncated"] is True
    np.testing.assert_array_equal(it[9]["terminal_observation"], [6.0, 7.0])
    assert it[1] == {} and infos[-1] is it[9] and len(infos[2:5]) == 3
    assert list(_StepInfos(3, np.array([], dtype=np.int64), tobs[:0], np.array([], bool))) == [{}, {}, {}]
