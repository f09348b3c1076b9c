"""TEST INFRASTRUCTURE ONLY — float64 NumPy restatement of the on-device policy path, the
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
