"""Trajectory logging in the reference Logger format (utils/logger.py): the array layout is
pinned by tests/golden/logger_golden.npz (the reference Logger run on scripted states);
the device-side recording needs a GPU (marked)."""
import os

import numpy as np
import pytest

from gym_pybullet_adrp_amd.logger import logger_arrays

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = np.load(os.path.join(ROOT, "tests", "golden", "logger_golden.npz"))


def test_layout_matches_reference_logger():
    st, ct = G["log_state"], G["log_control"]
    T, n = st.shape[:2]
    ts = np.repeat((np.arange(T) / 30)[:, None], n, 1)
    a = logger_arrays(ts, st, ct)
    for got, key in zip(a, ("timestamps", "states", "controls")):
        np.testing.assert_array_equal(got, G[f"log_grow_{key}"])
        pre = G[f"log_prealloc_{key}"]
        np.testing.assert_array_equal(got, pre[..., :T])          # preallocated: same columns,
        assert not pre[..., T:].any()                               # zeros after the last log


@pytest.mark.gpu
@pytest.mark.parametrize("physics,act", [("PYB_DRAG", "RPM"), ("PYB", "RPM"), ("PYB", "ONE_D_RPM")])
def test_device_logger_hover(tmp_path, physics, act):
    import torch
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    from gym_pybullet_adrp_amd.logger import DeviceLogger
    from gym_pybullet_adrp_amd.utils.enums import ActionType, Physics
    from oracle import oracle as O
    env = HoverAviary(physics=Physics[physics], act=ActionType[act], precision="fp32", num_envs=64, initial_xyzs=[0, 0, 1.0],
                      autoreset=False)
    env.reset()
    slots = [0, 5, 63]
    lg = DeviceLogger(env, 30, output_folder=str(tmp_path), slots=slots, duration_steps=16)
    rng = np.random.default_rng(0)
    A = env.h.A
    exp = []
    for t in range(10):
        a = rng.uniform(-1, 1, (64, 1, A)).astype(np.float32)
        env.step(torch.from_numpy(a))
        lg.log(t / 30, controls=np.tile(np.arange(12.0), (3, 1)))
        f, _ = env.get_state()
        names, _ = env.state_field_names()
        ix = {k: j for j, k in enumerate(names)}
        f = f.double().cpu().numpy()
        rows = []
        for s in slots:
            q = f[[ix[f"quat_{c}"] for c in "xyzw"], s]
            rpm = f[[ix[f"last_rpm_{k}"] for k in range(4)], s] if physics == "PYB_DRAG" else \
                env.HOVER_RPM * (1 + np.float32(0.05) * a[s, 0, [0, 1, 2, 3] if A == 4 else [0] * 4]).astype(np.float64)
            rows.append(np.concatenate([f[[ix[f"pos_{c}"] for c in "xyz"], s], q, O.euler_from_quat(q),
                                        f[[ix[f"vel_{c}"] for c in "xyz"], s], f[[ix[f"omega_{c}"] for c in "xyz"], s],
                                        rpm]))
        exp.append(rows)
    ts, states, controls = lg.arrays()
    ets, estates, econtrols = logger_arrays(np.repeat((np.arange(10) / 30)[:, None], 3, 1), np.array(exp),
                                            np.tile(np.arange(12.0), (10, 3, 1)))
    np.testing.assert_allclose(states, estates, rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(ts, ets)
    np.testing.assert_array_equal(controls, econtrols)
    path = lg.save()
    d = np.load(path)
    assert d["states"].shape == (3, 16, 10) and d["controls"].shape == (3, 12, 10) and d["timestamps"].shape == (3, 10)


@pytest.mark.gpu
def test_device_logger_race(tmp_path):
    import torch
    from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary
    from gym_pybullet_adrp_amd.logger import DeviceLogger
    env = MultiRaceAviary("level0", num_drones=2, precision="fp32", num_envs=32, seed=1)
    obs, _ = env.reset()
    lg = DeviceLogger(env, 25, output_folder=str(tmp_path), duration_steps=8)   # env 0's two drones
    act = torch.cat([obs[..., :3] + 0.2, torch.zeros_like(obs[..., :1])], -1).contiguous()
    for t in range(5):
        env.step(act)
        lg.log(t / 25)
    _, states, _ = lg.arrays()
    f, _ = env.get_state()
    names, _ = env.state_field_names()
    ix = {k: j for j, k in enumerate(names)}
    f = f.double().cpu().numpy()
    np.testing.assert_allclose(states[:, 0:3, -1], f[[ix[f"pos_{c}"] for c in "xyz"]][:, :2].T, rtol=1e-12)
    np.testing.assert_allclose(states[:, 12:16, -1], f[[ix[f"rpm_{k}"] for k in range(4)]][:, :2].T, rtol=1e-12)
    assert np.isfinite(states).all()
