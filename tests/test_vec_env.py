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

    def reset(self, seed=None):
        return torch.zeros((self.num_envs, 1, self.D)), {}

    def step(self, action):
        self.k += 1
        E = self.num_envs
        obs = torch.full((E, 1, self.D), float(self.k))
        rew = torch.arange(E, dtype=torch.float32) * self.k
        term = torch.zeros(E, dtype=torch.bool)
        trunc = torch.zeros(E, dtype=torch.bool)
        if self.k == 2:
            trunc[1] = True
            self.tobs[1] = 100.0
            obs[1] = -1.0
        if self.k == 3:
            term[2] = True
            self.tobs[2] = 200.0
        return obs, rew, term, trunc, {"answer": 42, "terminal_observation": self.tobs}

    def close(self):
        self.closed = True


def test_vecenv_protocol_and_infos():
    venv = AviaryVecEnv(_Scripted())
    assert venv.num_envs == 4 and venv.observation_space.shape == (1, 5)
    obs = venv.reset()
    assert isinstance(obs, np.ndarray) and obs.shape == (4, 1, 5)
    o, r, d, infos = venv.step(np.zeros((4, 1, 4), np.float32))
    assert not d.any() and all(i == {} for i in infos)
    o, r, d, infos = venv.step(np.zeros((4, 1, 4), np.float32))
    np.testing.assert_array_equal(d, [False, True, False, False])
    assert infos[1]["TimeLimit.truncated"] is True
    np.testing.assert_array_equal(infos[1]["terminal_observation"], np.full((1, 5), 100.0))
    np.testing.assert_array_equal(o[1], np.full((1, 5), -1.0))     # already the reset observation
    o, r, d, infos = venv.step(np.zeros((4, 1, 4), np.float32))
    assert d[2] and infos[2]["TimeLimit.truncated"] is False
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
