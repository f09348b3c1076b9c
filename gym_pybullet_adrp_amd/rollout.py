"""On-device PPO rollout collection (the consumer side of the hot path).

The reference trains with stable-baselines3 PPO (examples/learn.py:72-94): every rollout step,
``OnPolicyAlgorithm.collect_rollouts`` (stable_baselines3 2.3.2) runs ``policy(obs)`` on the host
batch, clips the actions, steps the VecEnv, bootstraps the value of time-limit truncations into the
reward, and appends (obs, action, reward, episode_start, value, log_prob) to its RolloutBuffer;
``compute_returns_and_advantage`` then runs GAE.  ``RolloutCollector`` does the same with every
tensor resident on the GPU:

* one ``adrp_policy_sample`` launch per step (actor + critic on f32 MFMA, the Gaussian sample, its
  log-probability and the clipped / RLController-transformed env action), written straight into
  the buffer row of the step;
* the env step's reward / flags are copied into the buffer row (device-to-device);
* the truncation bootstrap ``reward += gamma * V(terminal_obs)`` for envs whose episode hit the
  time limit (and not a termination), SB3 collect_rollouts;
* ``adrp_gae`` for the advantages and returns.

One agent per env: HoverAviary (learn.py's task) or a one-drone MultiRaceAviary (the RLController
setting).  ``collect`` can be captured in one HIP graph (every pointer is fixed per step).
"""
import torch

from . import _lib


class RolloutCollector:
    """``n_steps`` x ``num_envs`` PPO rollout buffer on the env's device.

    policy: ``DevicePolicy`` with a critic (``set_critic`` / ``from_zip(critic=True)``), its input
    the first ``policy.in_dim`` obs floats of the agent's row."""

    def __init__(self, env, policy, n_steps, gamma=0.99, gae_lambda=0.95, seed=0):
        if not policy.has_critic:
            raise ValueError("the policy needs a critic (DevicePolicy.set_critic) to collect rollouts")
        if env.NUM_DRONES != 1:
            raise ValueError("one agent per env: HoverAviary or MultiRaceAviary(num_drones=1)")
        self.env, self.policy = env, policy
        self.T, self.E = int(n_steps), env.num_envs
        self.gamma, self.gae_lambda, self.seed = float(gamma), float(gae_lambda), int(seed)
        dev = env.device
        D, A = env.h.D, policy.act_dim
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs = torch.zeros((self.T, self.E, D), **f32)
        self.actions = torch.zeros((self.T, self.E, A), **f32)
        self.rewards = torch.zeros((self.T, self.E), **f32)
        self.episode_starts = torch.zeros((self.T, self.E), **f32)
        self.values = torch.zeros((self.T, self.E), **f32)
        self.log_probs = torch.zeros((self.T, self.E), **f32)
        self.advantages = torch.zeros((self.T, self.E), **f32)
        self.returns = torch.zeros((self.T, self.E), **f32)
        self._env_act = torch.zeros((self.E,) + tuple(env._act_shape[1:]), **f32)
        self._term = torch.zeros((self.T, self.E), dtype=torch.bool, device=dev)
        self._trunc = torch.zeros((self.T, self.E), dtype=torch.bool, device=dev)
        self._last_obs = torch.zeros((self.E, D), **f32)
        self._last_start = torch.ones(self.E, **f32)         # SB3: _last_episode_starts = ones at reset
        self.last_values = torch.zeros(self.E, **f32)
        self.last_dones = torch.zeros(self.E, **f32)
        # value of the terminal observations (scratch outputs of the sampling launch)
        self._tv = torch.zeros(self.E, **f32)
        self._scratch = (torch.zeros((self.E, 4 if policy.mode else A), **f32), torch.zeros((self.E, A), **f32),
                         torch.zeros(self.E, **f32))
        self.rollouts = 0

    def reset(self):
        obs, _ = self.env.reset()
        self._last_obs.copy_(obs.reshape(self.E, -1))
        self._last_start.fill_(1.0)

    def _values_of(self, obs2d, out):
        """critic values of obs rows (the sampling launch; its action outputs go to scratch)"""
        ea, a, lp = self._scratch
        self.policy.sample(obs2d, self.seed, 0xFFFFFFFF, env_act=ea, action=a, value=out, log_prob=lp)

    def collect(self):
        """one rollout of n_steps env.steps -> fills the buffer and runs GAE (SB3 collect_rollouts +
        compute_returns_and_advantage); every tensor stays on the device"""
        # the env's device is the current one for the whole rollout: the launches take that device's
        # current stream (a null stream is the current device's)
        with torch.cuda.device(self.obs.device):
            return self._collect()

    def _collect(self):
        env, pol, E = self.env, self.policy, self.E
        base = self.rollouts * self.T
        env_act = self._env_act.view(E, -1)
        for t in range(self.T):
            self.obs[t].copy_(self._last_obs)
            self.episode_starts[t].copy_(self._last_start)
            pol.sample(self.obs[t], self.seed, base + t, env_act=env_act, action=self.actions[t],
                       value=self.values[t], log_prob=self.log_probs[t])
            obs, rew, term, trunc, info = env.step(self._env_act)
            self.rewards[t].copy_(rew)
            self._term[t].copy_(term)
            self._trunc[t].copy_(trunc)
            # time-limit bootstrap (collect_rollouts): reward += gamma * V(terminal obs) only where the
            # episode was truncated and not terminated; a select, so a stale terminal row of an env
            # that did not finish (even a non-finite one) never reaches its reward
            self._values_of(info["terminal_observation"].reshape(E, -1), self._tv)
            boot = trunc & ~term
            torch.where(boot, self.rewards[t] + self.gamma * self._tv, self.rewards[t], out=self.rewards[t])
            self._last_obs.copy_(obs.reshape(E, -1))
            self._last_start.copy_((term | trunc).to(torch.float32))
        # values of the observations after the last step (SB3: policy.predict_values(new_obs))
        self._values_of(self._last_obs, self.last_values)
        self.last_dones.copy_(self._last_start)
        rc = _lib.load().adrp_gae(self.rewards.data_ptr(), self.values.data_ptr(), self.episode_starts.data_ptr(),
                                  self.last_values.data_ptr(), self.last_dones.data_ptr(), self.T, E, self.gamma,
                                  self.gae_lambda, self.advantages.data_ptr(), self.returns.data_ptr(),
                                  _lib._raw_stream(self.obs.device.index))
        if rc != 0:
            raise _lib.AdrpError(f"adrp_gae: {_lib.load().adrp_last_error(None).decode()}")
        self.rollouts += 1
        return self

    def batches(self, batch_size, generator=None):
        """RolloutBuffer.get(batch_size): shuffled minibatches of (obs, actions, old_values,
        old_log_prob, advantages, returns) over the flattened n_steps x num_envs samples"""
        n = self.T * self.E
        idx = torch.randperm(n, device=self.obs.device, generator=generator)
        flat = (self.obs.reshape(n, -1), self.actions.reshape(n, -1), self.values.reshape(n),
                self.log_probs.reshape(n), self.advantages.reshape(n), self.returns.reshape(n))
        for s in range(0, n, batch_size):
            j = idx[s:s + batch_size]
            yield tuple(x.index_select(0, j) for x in flat)
