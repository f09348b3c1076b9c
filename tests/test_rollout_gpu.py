"""On-device PPO rollout collection (csrc/policy_kernel.h policy_sample_kernel, policy.hip adrp_gae,
gym_pybullet_adrp_amd/rollout.py) against the float64 restatement of SB3 2.3.2's
ActorCriticPolicy.forward(deterministic=False) / RolloutBuffer.compute_returns_and_advantage
(oracle/policy.py), with the reference's own zip weights (actor: policy_golden.npz, critic and
log_std: critic_golden.npz, both read from user_controller/*.zip without unpickling).
Needs an MI355X: -m gpu.

Bars: the Gaussian draws are the oracle's bit for bit (Philox + the IEEE-float Box-Muller); the
sampled action, value and log-probability within the actor's f32-MFMA bar (2e-5 absolute on the
action; value / log_prob relative 2e-5 of the pre-activation scale); GAE bit-identical to NumPy's
float32 recursion."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.policy import ACTOR_KEYS, CRITIC_KEYS, DevicePolicy  # noqa: E402
from oracle import policy as OP  # noqa: E402
from tests.test_policy import G, ZIPS, weights  # noqa: E402

C = np.load(os.path.join(os.path.dirname(__file__), "golden", "critic_golden.npz"))
TOL = 2e-5


def critic(name):
    return [C[f"{name}_v{i}"] for i in range(7)]


def make(name, mode):
    w, relu = weights(name)
    v = critic(name)
    wd = dict(zip(ACTOR_KEYS, w))
    wd.update(dict(zip(CRITIC_KEYS, v)))
    return DevicePolicy(wd, "relu" if relu else "tanh", 0, mode), w, v, relu


@pytest.mark.parametrize("name", ZIPS)
@pytest.mark.parametrize("mode", ["raw", "relative"])
def test_sample_matches_sb3_forward(name, mode):
    pol, w, v, relu = make(name, mode)
    assert pol.has_critic
    rng = np.random.default_rng(5)
    for rows, counter in ((1, 0), (17, 3), (1000, 77), (4096, 123456)):
        x = np.zeros((rows, 49), np.float32)
        x[:, :3] = rng.uniform(-3, 3, (rows, 3))
        x[:, 3:6] = rng.uniform(-np.pi, np.pi, (rows, 3))
        x[:, 6:] = rng.uniform(-2, 2, (rows, 43))
        xd = torch.from_numpy(x).cuda()
        eps = torch.empty((rows, 4), device="cuda")
        env_act, act, val, lp = pol.sample(xd, 2024, counter, eps=eps)
        torch.cuda.synchronize()
        e_ref = OP.policy_eps(rows, 2024, counter, 4)
        np.testing.assert_array_equal(eps.cpu().numpy(), e_ref)                 # the draws, bit for bit
        a_ref, v_ref, lp_ref = OP.sample(w, v, x, relu, e_ref)
        std = np.exp(np.asarray(v[6], np.float64))
        assert np.abs(act.cpu().numpy() - a_ref).max() <= TOL * max(1.0, std.max())
        assert np.abs(val.cpu().numpy() - v_ref).max() <= TOL * max(1.0, np.abs(v_ref).max())
        assert np.abs(lp.cpu().numpy() - lp_ref).max() <= 1e-4 * max(1.0, np.abs(lp_ref).max())
        clipped = np.clip(a_ref, -1, 1)
        ref_env = OP.rl_transform(clipped, x, mode) if mode != "raw" else clipped
        err = np.abs(env_act.cpu().numpy() - ref_env)
        if mode != "raw":
            err[:, 3] = np.abs(np.angle(np.exp(1j * (env_act.cpu().numpy()[:, 3] - ref_env[:, 3]))))
        assert err.max() <= TOL * max(1.0, std.max())
    # the draws follow the counter: another step, other samples
    xd = torch.from_numpy(x[:64]).cuda()
    a1 = pol.sample(xd, 2024, 1)[1].cpu().numpy()
    a2 = pol.sample(xd, 2024, 2)[1].cpu().numpy()
    assert not np.array_equal(a1, a2)
    pol.close()


def test_gae_matches_sb3():
    rng = np.random.default_rng(9)
    T, E = 257, 1000
    rew = rng.normal(size=(T, E)).astype(np.float32)
    val = rng.normal(size=(T, E)).astype(np.float32)
    starts = (rng.random((T, E)) < 0.05).astype(np.float32)
    last_v = rng.normal(size=E).astype(np.float32)
    dones = (rng.random(E) < 0.1).astype(np.float32)
    d = [torch.from_numpy(a).cuda() for a in (rew, val, starts, last_v, dones)]
    adv = torch.empty((T, E), device="cuda")
    ret = torch.empty((T, E), device="cuda")
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    assert lib.adrp_gae(*(t.data_ptr() for t in d), T, E, 0.99, 0.95, adv.data_ptr(), ret.data_ptr(), s) == 0
    a_ref, r_ref = OP.gae(rew, val, starts, last_v, dones, 0.99, 0.95)
    np.testing.assert_array_equal(adv.cpu().numpy(), a_ref)
    np.testing.assert_array_equal(ret.cpu().numpy(), r_ref)


def test_collect_race_rollout_matches_oracle_policy():
    """a 64-step rollout of 512 one-drone level0 races driven by the reference's example actor /
    critic (RLController RELATIVE transform), all on the device: every stored step's value,
    log-prob and action equal the oracle's forward of the stored obs with the kernel's draws, the
    env actions drive the env (the stored obs of step t+1 are the env's), and the advantages /
    returns equal SB3's GAE recursion of the stored rewards / values"""
    from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary
    from gym_pybullet_adrp_amd.rollout import RolloutCollector
    env = MultiRaceAviary("level0", num_drones=1, num_envs=512, seed=3, reward="wrapper")
    pol, w, v, relu = make("example_RL_model", "relative")
    col = RolloutCollector(env, pol, 64, seed=11)
    col.reset()
    col.collect()
    torch.cuda.synchronize()
    obs = col.obs.cpu().numpy()
    for t in (0, 1, 31, 63):
        e_ref = OP.policy_eps(512, 11, t, 4)
        a_ref, v_ref, lp_ref = OP.sample(w, v, obs[t, :, :49], relu, e_ref)
        assert np.abs(col.actions[t].cpu().numpy() - a_ref).max() <= 5e-5
        assert np.abs(col.values[t].cpu().numpy() - v_ref).max() <= 5e-5 * max(1, np.abs(v_ref).max())
        assert np.abs(col.log_probs[t].cpu().numpy() - lp_ref).max() <= 1e-4 * max(1, np.abs(lp_ref).max())
    a_ref, r_ref = OP.gae(col.rewards.cpu().numpy(), col.values.cpu().numpy(), col.episode_starts.cpu().numpy(),
                          col.last_values.cpu().numpy(), col.last_dones.cpu().numpy(), 0.99, 0.95)
    np.testing.assert_array_equal(col.advantages.cpu().numpy(), a_ref)
    np.testing.assert_array_equal(col.returns.cpu().numpy(), r_ref)
    assert float(col.episode_starts[0].min()) == 1.0          # SB3: every env starts an episode
    n = 0
    for b in col.batches(4096):
        assert b[0].shape == (min(4096, 64 * 512 - n), 49)
        n += b[0].shape[0]
    assert n == 64 * 512
    pol.close()
    env.close()


def test_collect_hover_one_d_rpm():
    """learn.py's task shape: HoverAviary ONE_D_RPM (obs 27, one action) with a random Tanh 27-64-64-1
    actor / critic; 2 rollouts of 32 steps over 1024 envs with auto-reset and time-limit truncation
    bootstraps; the stored actions drive the env through clip(a) (RAW)"""
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    from gym_pybullet_adrp_amd.rollout import RolloutCollector
    from gym_pybullet_adrp_amd.utils.enums import ActionType
    rng = np.random.default_rng(2)
    env = HoverAviary(act=ActionType.ONE_D_RPM, num_envs=1024, seed=4, initial_xyzs=[0, 0, 1.0],
                      init_noise={"rpy": 0.3, "omega": 1.0})
    shapes = {ACTOR_KEYS[0]: (64, 27), ACTOR_KEYS[1]: (64,), ACTOR_KEYS[2]: (64, 64), ACTOR_KEYS[3]: (64,),
              ACTOR_KEYS[4]: (1, 64), ACTOR_KEYS[5]: (1,), CRITIC_KEYS[0]: (64, 27), CRITIC_KEYS[1]: (64,),
              CRITIC_KEYS[2]: (64, 64), CRITIC_KEYS[3]: (64,), CRITIC_KEYS[4]: (1, 64), CRITIC_KEYS[5]: (1,),
              CRITIC_KEYS[6]: (1,)}
    wd = {k: (rng.normal(size=s) * 0.2).astype(np.float32) for k, s in shapes.items()}
    pol = DevicePolicy(wd, "tanh", 0, "raw")
    assert pol.act_dim == 1 and pol.in_dim == 27
    col = RolloutCollector(env, pol, 32, seed=1)
    col.reset()
    for _ in range(2):
        col.collect()
    torch.cuda.synchronize()
    assert torch.isfinite(col.advantages).all() and torch.isfinite(col.returns).all()
    assert float(col.episode_starts.sum()) > 0                    # auto-resets inside the rollouts
    w = [wd[k] for k in ACTOR_KEYS]
    v = [wd[k] for k in CRITIC_KEYS]
    e_ref = OP.policy_eps(1024, 1, 32 + 5, 1)
    a_ref, v_ref, lp_ref = OP.sample(w, v, col.obs[5].cpu().numpy(), False, e_ref)
    assert np.abs(col.actions[5].cpu().numpy() - a_ref).max() <= 5e-5
    assert np.abs(col.values[5].cpu().numpy() - v_ref).max() <= 5e-5
    pol.close()
    env.close()


def test_truncation_bootstrap_matches_oracle_critic():
    """SB3 collect_rollouts' time-limit bootstrap: the stored reward of step t is the env's reward
    plus gamma * V(terminal obs) exactly on the envs that were truncated and not terminated, and the
    env's reward bit for bit everywhere else.  HoverAviary ONE_D_RPM under a random Tanh
    actor: tilted / out-of-bounds drones are truncated (HoverAviary._computeTruncated), so a
    24-step rollout over 1024 envs holds hundreds of bootstraps.  V is checked against the float64
    critic forward of the recorded terminal rows (oracle/policy.py critic_value) at the actor's bar."""
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    from gym_pybullet_adrp_amd.rollout import RolloutCollector
    from gym_pybullet_adrp_amd.utils.enums import ActionType
    rng = np.random.default_rng(8)
    E, T, gamma = 1024, 24, 0.99
    env = HoverAviary(act=ActionType.ONE_D_RPM, num_envs=E, seed=6, initial_xyzs=[0, 0, 1.0],
                      init_noise={"rpy": 0.35, "omega": 2.0, "vel": 0.5})
    shapes = {ACTOR_KEYS[0]: (64, 27), ACTOR_KEYS[1]: (64,), ACTOR_KEYS[2]: (64, 64), ACTOR_KEYS[3]: (64,),
              ACTOR_KEYS[4]: (1, 64), ACTOR_KEYS[5]: (1,), CRITIC_KEYS[0]: (64, 27), CRITIC_KEYS[1]: (64,),
              CRITIC_KEYS[2]: (64, 64), CRITIC_KEYS[3]: (64,), CRITIC_KEYS[4]: (1, 64), CRITIC_KEYS[5]: (1,),
              CRITIC_KEYS[6]: (1,)}
    wd = {k: (rng.normal(size=s) * 0.3).astype(np.float32) for k, s in shapes.items()}
    pol = DevicePolicy(wd, "tanh", 0, "raw")
    col = RolloutCollector(env, pol, T, gamma=gamma, seed=3)
    raw = []
    step = env.step

    def recording_step(a):
        out = step(a)
        o, r, te, tr, info = out
        raw.append((r.clone(), te.clone(), tr.clone(), info["terminal_observation"].reshape(E, -1).clone()))
        return out
    env.step = recording_step
    col.reset()
    col.collect()
    torch.cuda.synchronize()
    v = [wd[k] for k in CRITIC_KEYS]
    boots = 0
    for t, (r, te, tr, tobs) in enumerate(raw):
        r, te, tr, tobs = r.cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy(), tobs.cpu().numpy()
        stored = col.rewards[t].cpu().numpy()
        boot = tr & ~te
        np.testing.assert_array_equal(stored[~boot], r[~boot])
        if boot.any():
            v_ref = OP.critic_value(v, tobs[boot], False)
            exp = r[boot].astype(np.float64) + gamma * v_ref
            assert np.abs(stored[boot] - exp).max() <= 5e-5 * max(1.0, np.abs(exp).max()), f"step {t}"
            # the bootstrap is the terminal row's value, not the next episode's first row
            assert not np.allclose(tobs[boot], col.obs[t + 1].cpu().numpy()[boot]) if t + 1 < T else True
        boots += int(boot.sum())
    assert boots > 50, f"only {boots} truncations: the test should exercise the bootstrap"
    pol.close()
    env.close()
