"""Persistent HoverAviary step probe (csrc/hover_persist.h): E = 1 synchronised steps/s, and a long
bit-identity run against the launched kernel counting the steps whose outputs differ (a stale output
row is a hand-off bug, not a numerics one).  Run under both ADRP_PERSIST_SYSST settings.

    python tools/persist_probe.py [STEPS_SPEED] [STEPS_IDENTITY]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("ADRP_STAGE_ROWS", "0")
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import ActionType, Physics  # noqa: E402


def speed(n):
    env = HoverAviary(num_envs=1, precision="fp64", seed=3)
    env.reset()
    act = np.zeros((1, 1, 4), np.float32)
    with env.persistent() as p:
        for _ in range(200):
            p.step(act)
        t0 = time.perf_counter()
        for _ in range(n):
            p.step(act)
        dt = time.perf_counter() - t0
    env.close()
    return n / dt


def identity(E, physics, act_type, n):
    kw = dict(num_envs=E, physics=physics, act=act_type, precision="fp64", seed=31, initial_xyzs=[0, 0, 1.0],
              init_noise={"xyz": 0.1, "rpy": 0.2, "vel": 0.3, "omega": 1.0})
    a, b = HoverAviary(**kw), HoverAviary(**kw)
    a.reset()
    b.reset()
    rng = np.random.default_rng(7)
    A = a.h.A
    bad = 0
    with b.persistent() as p:
        for k in range(n):
            act = rng.uniform(-1, 1, (E, 1, A)).astype(np.float32)
            if (k // 40) % 3 == 1:
                act[:] = 1.0
            oa, ra, ta, tra, _ = a.step(torch.from_numpy(act).to(a.device))
            ob, rb, tb, trb, _ = p.step(act)
            same = (np.array_equal(ob, oa.cpu().numpy()) and np.array_equal(rb, ra.cpu().numpy())
                    and np.array_equal(tb, ta.cpu().numpy()) and np.array_equal(trb, tra.cpu().numpy()))
            bad += 0 if same else 1
    a.close()
    b.close()
    return bad


if __name__ == "__main__":
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    ni = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    out = {"sysst": os.environ.get("ADRP_PERSIST_SYSST", "0"), "steps_per_s": [round(speed(ns)) for _ in range(3)]}
    out["mismatched_steps"] = {f"E{E}": identity(E, ph, at, ni) for E, ph, at in
                               [(70, Physics.PYB_GND_DRAG_DW, ActionType.ONE_D_RPM), (1, Physics.PYB, ActionType.RPM),
                                (128, Physics.PYB, ActionType.RPM)]}
    out["identity_steps"] = ni
    print(json.dumps(out), flush=True)
