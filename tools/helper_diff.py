"""Where do hover steps with / without the reset helper wave differ?  (diagnostic)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
noise = {"xyz": [0.1, 0.1, 0.1], "rpy": 0.05, "vel": 0.1, "omega": 0.1}
acts = torch.from_numpy(np.random.default_rng(8).uniform(-1, 1, (60, E, 1, 4)).astype(np.float32))
runs = []
for helper in ("1", "0"):
    os.environ["ADRP_RESET_HELPER"] = helper
    env = HoverAviary(physics=Physics.PYB, num_envs=E, seed=99, initial_xyzs=[0, 0, 1.0], init_noise=noise)
    env.reset()
    seq = []
    for t in range(60):
        obs, rew, te, tr, info = env.step(acts[t].to(env.device))
        seq.append((obs.reshape(E, -1).cpu().numpy().copy(), info["terminal_observation"].reshape(E, -1).cpu().numpy().copy(),
                    rew.reshape(E).cpu().numpy().copy(), (te | tr).reshape(E).cpu().numpy().copy()))
    runs.append(seq)
    env.close()
for t in range(60):
    a, b = runs[0][t], runs[1][t]
    for name, x, y in (("obs", a[0], b[0]), ("tobs", a[1], b[1]), ("rew", a[2], b[2]), ("done", a[3], b[3])):
        if not np.array_equal(x, y):
            d = x != y
            rows = np.nonzero(d.reshape(E, -1).any(1))[0]
            cols = np.nonzero(d.reshape(E, -1).any(0))[0] if x.ndim > 1 else []
            print(f"step {t} {name}: {len(rows)} rows differ, e.g. {rows[:8]}, cols {list(cols)[:20]}, "
                  f"done at those rows {a[3][rows[:8]]}, max abs {np.abs(x - y).max():.3e}")
            if name == "obs":
                r = rows[0]
                print("  helper", a[0][r, :12], "\n  chain ", b[0][r, :12])
    if any(not np.array_equal(x, y) for x, y in zip(a, b)):
        break
