"""Environment registry (gym_pybullet_adrp/__init__.py:5-28): hover-aviary-v0 / multi-race-aviary-v0."""
import importlib

import pytest

import gym_pybullet_adrp_amd as pkg


def test_ids_resolve_to_the_env_classes():
    assert set(pkg.ENV_IDS) == {"hover-aviary-v0", "multi-race-aviary-v0"}
    for env_id, entry in pkg.ENV_IDS.items():
        mod, cls = entry.split(":")
        c = getattr(importlib.import_module(mod), cls)
        assert c.__name__ == {"hover-aviary-v0": "HoverAviary", "multi-race-aviary-v0": "MultiRaceAviary"}[env_id]
    with pytest.raises(KeyError):
        pkg.make("ctrl-aviary-v0")


def test_gymnasium_registration_when_available():
    gym = pytest.importorskip("gymnasium")
    for env_id, entry in pkg.ENV_IDS.items():
        assert gym.envs.registration.registry[env_id].entry_point == entry


@pytest.mark.gpu
def test_make_builds_the_batched_env():
    env = pkg.make("multi-race-aviary-v0", race_config="level1", num_drones=2, num_envs=8)
    obs, _ = env.reset()
    assert tuple(obs.shape) == (8, 2, 49)
    env.close()
    env = pkg.make("hover-aviary-v0", num_envs=16)
    obs, _ = env.reset()
    assert tuple(obs.shape) == (16, 1, 72)
    env.close()
