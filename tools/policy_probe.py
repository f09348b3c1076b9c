"""Launch the on-device policy forward N times per configuration (rocprofv3 --kernel-trace
target):  python tools/policy_probe.py [reps]   (ADRP_POLICY_STAGE=1 selects the LDS variant)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_pybullet_adrp_amd.policy import ACTOR_KEYS, DevicePolicy  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "policy_golden.npz"))
for name, rows in (("example_RL_model", 4096), ("twogates", 16384)):
    w = {k: g[f"{name}_w{i}"] for i, k in enumerate(ACTOR_KEYS)}
    pol = DevicePolicy(w, "relu" if bool(g[f"{name}_relu"]) else "tanh", 0, "relative")
    obs = torch.rand((rows, 49), device="cuda") * 2 - 1
    out = torch.empty((rows, 4), device="cuda")
    for _ in range(reps):
        pol.act(obs, out=out)
    torch.cuda.synchronize()
    pol.close()
print("ok")
