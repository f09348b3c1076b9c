"""The reference's gymnasium wrappers (utils/wrapper.py), fused into the race step kernel.

``DroneObservationWrapper(env)`` and ``RewardWrapper(env)`` take a ``MultiRaceAviary`` (or a
wrapper of one) and switch the matching stage of the fused step on (``adrp_set_wrappers``):

* DroneObservationWrapper (wrapper.py:38-65): yaw actions are forced to 0 and an env terminates
  once its drone 0 has passed gate 2 (``current_gate[0] >= 2``), inside the same launch, so the
  auto-reset fires on it.  The reference zeroes ``action[:, 3]`` of the caller's numpy array in
  place; the device action tensor is left untouched here (the kernel reads yaw as 0).
* RewardWrapper (wrapper.py:68-186): gate-progress reward of drone 0 (``info["task_completed"]``,
  absent in the reference, := every drone finished).

Unlike a gymnasium wrapper these switch a stage of the BASE env's fused step: from construction on
the unwrapped env (and every other stack over it) steps with yaw 0 / the early termination / the
gate reward too.  ``detach()`` restores the base env's previous wrapper flags (the wrapper object
must not be stepped afterwards).

Stacking order matters as in the reference: ``RewardWrapper(DroneObservationWrapper(env))`` gives
the reward's terminal terms the early termination, ``DroneObservationWrapper(RewardWrapper(env))``
does not.  Everything else is delegated to the wrapped env (gymnasium 0.28 ``Wrapper`` semantics:
public attributes forward).
"""


class _Wrapper:
    def __init__(self, env):
        self.env = env
        base = self.unwrapped
        self._saved = (base.reward_wrapper, base.obs_wrapper)   # flags before this wrapper

    def detach(self):
        """switch the base env's fused stage back to what it was before this wrapper"""
        self.unwrapped.set_wrappers(*self._saved)

    def __getattr__(self, name):
        if name.startswith("_") or name == "env":
            raise AttributeError(f"accessing private attribute '{name}' is prohibited")
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        e = self.env
        while isinstance(e, _Wrapper):
            e = e.env
        return e

    def reset(self, *args, **kwargs):
        return self.env.reset(*args, **kwargs)

    def step(self, action):
        return self.env.step(action)

    def close(self):
        return self.env.close()


class DroneObservationWrapper(_Wrapper):
    """utils/wrapper.py:12-65 (fused): yaw actions 0, early termination at current_gate[0] >= 2."""

    def __init__(self, env):
        super().__init__(env)
        base = self.unwrapped
        base.set_wrappers(base.reward_wrapper, 2 if base.reward_wrapper else 1)


class RewardWrapper(_Wrapper):
    """utils/wrapper.py:68-186 (fused): the gate-progress reward of drone 0."""

    def __init__(self, env):
        super().__init__(env)
        base = self.unwrapped
        base.set_wrappers(True, base.obs_wrapper)
