"""On-device policy forward (csrc/policy_kernel.h, f32 MFMA) against the float64 oracle
(oracle/policy.py, whose transforms are pinned by the reference) and a torch fp32 forward.
Needs an MI355X: -m gpu.

Tolerance: the kernel computes the MLP in exact-f32 MFMA fma chains; vs the float64 oracle
the clipped action may differ by <= 2e-5 absolute (a few f32 ulps of Σ|w·x| ~ 10), the
FULLSTATE setpoints likewise (the transform itself runs in float64 on the device)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd.policy import ACTOR_KEYS, DevicePolicy, rollout  # noqa: E402
from oracle import policy as OP  # noqa: E402
from tests.test_policy import G, ZIPS, weights  # noqa: E402

TOL = 2e-5


def make(name, mode):
    w, relu = weights(name)
    return DevicePolicy(dict(zip(ACTOR_KEYS, w)), "relu" if relu else "tanh", 0, mode), w, relu


def random_obs(rng, shape):
    x = np.zeros(shape, np.float32)
    x[..., :3] = rng.uniform(-3, 3, shape[:-1] + (3,))
    x[..., 3:6] = rng.uniform(-np.pi, np.pi, shape[:-1] + (3,))
    x[..., 6:] = rng.uniform(-2, 2, shape[:-1] + (shape[-1] - 6,))
    return x


@pytest.mark.parametrize("name", ZIPS)
@pytest.mark.parametrize("mode", ["raw", "relative", "absolute"])
def test_policy_matches_oracle(name, mode):
    pol, w, relu = make(name, mode)
    rng = np.random.default_rng(7)
    for rows in (1, 15, 17, 64, 1000, 16384):                  # ragged tiles and the config-4 batch
        x = random_obs(rng, (rows, 49))
        got = pol.act(torch.from_numpy(x).cuda()).cpu().numpy()
        a = OP.sb3_predict(w, x, relu)
        ref = OP.rl_transform(a, x, mode) if mode != "raw" else a
        err = np.abs(got - ref)
        if mode != "raw":     # a yaw at the +-pi seam may land on the other side: compare on the circle
            err[:, 3] = np.abs(np.angle(np.exp(1j * (got[:, 3] - ref[:, 3]))))
        assert err.max() <= TOL, f"rows={rows}: max err {err.max():.3e}"
    pol.close()


def test_policy_saturation_and_golden_obs():
    """the reference's sample obs (policy_golden) incl. actions beyond the Box (clip)"""
    pol, w, relu = make("twogates", "raw")
    x = G["pol_obs"].astype(np.float32)
    got = pol.act(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = OP.sb3_predict(w, x, relu)
    assert np.abs(got - ref).max() <= TOL
    assert (np.abs(OP.actor_mean(w, x, relu)) > 1).any()       # clipping exercised


def test_obs_stride_prefix():
    """COMPETE rows are 67 wide; the policy reads the first 49 columns of each row."""
    pol, w, relu = make("example_RL_model", "relative")
    rng = np.random.default_rng(3)
    x = random_obs(rng, (4096, 4, 67))
    got = pol.act(torch.from_numpy(x).cuda()).cpu().numpy().reshape(-1, 4)
    xx = x.reshape(-1, 67)[:, :49]
    ref = OP.rl_transform(OP.sb3_predict(w, xx, relu), xx, "relative")
    err = np.abs(got - ref)
    err[:, 3] = np.abs(np.angle(np.exp(1j * (got[:, 3] - ref[:, 3]))))
    assert err.max() <= TOL


def test_closed_loop_race_rollout_graph():
    """MultiRaceAviary level0 COMPARE driven by the example policy entirely on the device, one
    env.step + one policy launch per iteration, captured in a HIP graph; the setpoints fed to
    each step equal the oracle policy of that step's observation."""
    from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary
    env = MultiRaceAviary("level0", num_drones=2, precision="fp32", num_envs=512, seed=5)
    pol, w, relu = make("example_RL_model", "relative")
    obs, _ = env.reset()
    act = torch.empty((512, 2, 4), device=obs.device)
    rollout(env, pol, 3, act)                                  # eager warm-up
    torch.cuda.synchronize()
    x = env._obs.cpu().numpy().reshape(-1, 49)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        rollout(env, pol, 1, act)                             # warm the side stream
        torch.cuda.synchronize()
        x = env._obs.cpu().numpy().reshape(-1, 49)
        with torch.cuda.graph(g, stream=s):
            pol.act(env._obs, out=act)
            env.step(act)
    g.replay()
    torch.cuda.synchronize()
    ref = OP.rl_transform(OP.sb3_predict(w, x, relu), x, "relative")
    got = act.cpu().numpy().reshape(-1, 4)
    err = np.abs(got - ref)
    err[:, 3] = np.abs(np.angle(np.exp(1j * (got[:, 3] - ref[:, 3]))))
    assert err.max() <= TOL
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    assert torch.isfinite(env._obs).all()
    env.close(); pol.close()
