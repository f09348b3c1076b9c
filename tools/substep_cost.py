"""Kernel time vs sub-steps per env.step (E = 4096): slope = cost of one physics sub-step."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402

for pyb in (120, 240, 480, 960):
    ctrl = 30          # ring length 15 everywhere; S = pyb / 30 sub-steps
    env = HoverAviary(num_envs=4096, pyb_freq=pyb, ctrl_freq=ctrl, initial_xyzs=[0, 0, 1.0],
                      init_noise={"xyz": 0.1, "rpy": 0.05, "vel": 0.1, "omega": 0.1})
    env.reset()
    acts = torch.rand((8, 4096, 1, 4), device=env.device) * 2 - 1
    for k in range(50):
        env.step(acts[k % 8])
    torch.cuda.synchronize()
    env.h.profile_begin(400)
    for k in range(400):
        env.step(acts[k % 8])
    ms = env.h.profile_end(400)
    from gym_pybullet_adrp_amd import _lib
    print(json.dumps({"substeps": pyb // ctrl, "kernel": _lib.kernel_name(env.cfg), "kernel_us": float(np.mean(ms)) * 1e3,
                      "kernel_us_median": float(np.median(ms)) * 1e3}), flush=True)
    env.close()
