"""gym_pybullet_adrp_amd — MI355X-native batched quadrotor step for gym-pybullet-adrp.

The hot path (HoverAviary / MultiRaceAviary env.step: PYB physics sub-steps, force
models, Mellinger controller, collision, obs/reward/termination) runs as one fused HIP
kernel per env.step inside libadrp.so (csrc/), called through the C-ABI in
include/adrp.h.  This package holds the ctypes loader and the gymnasium/SB3-style
vectorised env classes that mirror the reference's surface.
"""
__version__ = "0.1.0"

# Environment registry (gym_pybullet_adrp/__init__.py:5-28): the two envs on the hot path.  With
# gymnasium importable they are registered as the reference registers them, so
# gymnasium.make("multi-race-aviary-v0", ...) builds the batched GPU env; without it, make() below
# resolves the same ids.
ENV_IDS = {
    "hover-aviary-v0": "gym_pybullet_adrp_amd.envs:HoverAviary",
    "multi-race-aviary-v0": "gym_pybullet_adrp_amd.envs:MultiRaceAviary",
}


def make(env_id, **kwargs):
    """gymnasium.make for the registered ids (no wrappers: the envs are batched and autoreset)."""
    import importlib
    if env_id not in ENV_IDS:
        raise KeyError(f"unknown env id {env_id!r}; registered: {sorted(ENV_IDS)}")
    mod, cls = ENV_IDS[env_id].split(":")
    return getattr(importlib.import_module(mod), cls)(**kwargs)


try:  # pragma: no cover - gymnasium is absent in this image
    from gymnasium.envs.registration import register as _register, registry as _registry
    for _id, _entry in ENV_IDS.items():
        if _id not in _registry:
            _register(id=_id, entry_point=_entry, disable_env_checker=True)
except ImportError:
    pass
