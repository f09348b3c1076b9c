"""TEST INFRASTRUCTURE ONLY — float64 NumPy restatement of the on-device policy path (actor,
critic, Gaussian sample, GAE), the
checker for csrc/policy_kernel.h (never imported by the product package).

* ``actor_mean`` / ``sb3_predict``: stable_baselines3 2.3.2 (the version the reference's
  zips were saved with) ``ActorCriticPolicy._predict(obs, deterministic=True)`` for an
  MlpPolicy with a Flatten extractor: ``action_net(policy_net(obs))`` = the Gaussian mean,
  then ``BasePolicy.predict`` clips it to the Box [-1, 1].  SB3 is not importable here:
  this part is restated from SB3's published code (parity unpinned beyond the reference's
  own weights), the GPU kernel is held to it and to a torch fp32 forward.
* ``rl_transform``: ``RLController._action_transform`` (user_controller/RLController.py:60-73)
  and ``RLControllerTwoGates._action_transform`` (RLControllerTwoGates.py:56-69) with
  ``map2pi`` (utils/utils.py:188-197): pinned by tests/golden/policy_golden.npz, produced by
  running those reference classes (tests/golden/make_golden.py: policy_fixtures).
"""
import numpy as np


def actor_mean(w, obs, relu):
    """w = (W1, b1, W2, b2, W3, b3) in torch Linear layout; obs [..., in_dim] -> mean [..., 4]"""
    act = (lambda x: np.maximum(x, 0.0)) if relu else np.tanh
    x = np.asarray(obs, np.float64)
    h = act(x @ np.asarray(w[0], np.float64).T + np.asarray(w[1], np.float64))
    h = act(h @ np.asarray(w[2], np.float64).T + np.asarray(w[3], np.float64))
    return h @ np.asarray(w[4], np.float64).T + np.asarray(w[5], np.float64)


def sb3_predict(w, obs, relu):
    return np.clip(actor_mean(w, obs, relu), -1.0, 1.0)


def map2pi(a):
    return ((a + np.pi) % (2 * np.pi)) - np.pi


def rl_transform(a, obs, mode):
    """a [..., 4] agent action, obs [..., >= 6] -> FULLSTATE setpoint [..., 4] (float64)"""
    a = np.array(a, np.float32).astype(np.float64)          # SB3 returns float32 actions
    a[..., 3] = 0.0
    scale = np.array([1, 1, 1, np.pi])
    if mode == "raw":
        return np.clip(a, -1, 1)
    if mode == "relative":
        pose = np.asarray(obs, np.float64)[..., [0, 1, 2, 5]]
        t = pose + a * scale
    else:
        t = a * scale
    t[..., 3] = map2pi(t[..., 3])
    return t


# ---- PPO rollout step (stable_baselines3 2.3.2 ActorCriticPolicy.forward, deterministic=False) ----
def critic_value(v, obs, relu):
    """v = (W1, b1, W2, b2, Wv, bv[, log_std]) of mlp_extractor.value_net + value_net -> value [...]"""
    act = (lambda x: np.maximum(x, 0.0)) if relu else np.tanh
    x = np.asarray(obs, np.float64)
    h = act(x @ np.asarray(v[0], np.float64).T + np.asarray(v[1], np.float64))
    h = act(h @ np.asarray(v[2], np.float64).T + np.asarray(v[3], np.float64))
    return (h @ np.asarray(v[4], np.float64).T + np.asarray(v[5], np.float64))[..., 0]


def policy_eps(rows, seed, counter, act_dim):
    """the kernel's standard normals: Philox4x32-10 {row, counter, 0x504f4c00, 0} keyed by seed, the
    Box-Muller of its two word pairs (oracle/race.c normal_pair_f) -> [rows, act_dim] float32"""
    from oracle import oracle as O
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]
    out = np.zeros((rows, 4), np.float32)
    for r in range(rows):
        x = O.philox([r & 0xFFFFFFFF, counter & 0xFFFFFFFF, 0x504F4C00, 0], key)
        out[r, :2] = O.normal_pair(x[0], x[1])
        out[r, 2:] = O.normal_pair(x[2], x[3])
    return out[:, :act_dim]


def sample(w, v, obs, relu, eps):
    """(action = mean + exp(log_std) eps, value, log_prob = sum_i log N(a_i; mean_i, std_i)) in float64"""
    mean = actor_mean(w, obs, relu)
    log_std = np.asarray(v[6], np.float64)
    std = np.exp(log_std)
    a = mean + std * np.asarray(eps, np.float64)
    lp = (-((a - mean) ** 2) / (2 * std * std) - log_std - np.log(np.sqrt(2 * np.pi))).sum(-1)
    return a, critic_value(v, obs, relu), lp


def gae(rewards, values, episode_starts, last_values, dones, gamma, gae_lambda):
    """RolloutBuffer.compute_returns_and_advantage (stable_baselines3 2.3.2), float32 arrays as the
    rollout buffer holds them -> (advantages, returns)"""
    rewards, values, episode_starts = (np.asarray(x, np.float32) for x in (rewards, values, episode_starts))
    last_values, dones = np.asarray(last_values, np.float32), np.asarray(dones, np.float32)
    T = rewards.shape[0]
    adv = np.zeros_like(rewards)
    last = np.zeros_like(last_values)
    for step in reversed(range(T)):
        if step == T - 1:
            next_nt = np.float32(1.0) - dones
            next_v = last_values
        else:
            next_nt = np.float32(1.0) - episode_starts[step + 1]
            next_v = values[step + 1]
        delta = rewards[step] + np.float32(gamma) * next_v * next_nt - values[step]
        last = delta + np.float32(gamma * gae_lambda) * next_nt * last
        adv[step] = last
    return adv, adv + values
