"""The gymnasium ``Env`` surface of the batched envs (envs/BaseAviary.py:18-21, 391-420).

The reference's aviaries subclass ``gymnasium.Env``; ``gymnasium.make`` then sets
``env.unwrapped.spec`` and wraps the env (``OrderEnforcing``, whose ``Wrapper.__init__`` requires a
``gymnasium.Env``).  With gymnasium importable the batched envs subclass it too; without it (this
image) they carry the same attributes: ``metadata``, ``render_mode``, ``spec``, ``unwrapped``,
``np_random`` is not provided (the random streams are the device Philox keys, ``reset(seed=...)``).
"""
try:  # pragma: no cover - gymnasium is absent in this image
    from gymnasium import Env as _Env
except ImportError:
    _Env = object


class AviaryEnv(_Env):
    # the reference comments its metadata out (BaseAviary.py:21): gymnasium's defaults
    metadata = {"render_modes": []}
    render_mode = None
    spec = None
    reward_range = (-float("inf"), float("inf"))

    @property
    def unwrapped(self):
        return self

    def render(self):
        """BaseAviary.render prints a text line per drone; GUI / video are out of scope here
        (DESIGN.md §9): nothing to render."""
        return None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __str__(self):
        return f"<{type(self).__name__} x{getattr(self, 'num_envs', '?')} (gym_pybullet_adrp_amd)>"
