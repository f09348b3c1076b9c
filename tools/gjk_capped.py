"""Dump the GJK queries that reach the 48-iteration cap (GJK-stats build: make -C
gym_pybullet_adrp_amd/csrc devg) under the actor-driven config 3 (or random targets), and save
them for a CPU replay: gpurun_out/gjk_capped_<config>_<prec>[_<policy>].npz with the two shapes (oracle shape layout:
type, c, R row-major, h, r), the cut and the last |v|^2.

usage: ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so [RACE_POLICY=example] [RACE_PRECISION=fp64]
       python tools/gjk_capped.py [LEVEL DRONES PHYSICS MODE E STEPS]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics, RaceMode  # noqa: E402

a = sys.argv[1:] + [None] * 6
level, n, phys, mode = a[0] or "level0", int(a[1] or 2), a[2] or "PYB", a[3] or "COMPARE"
E, steps = int(a[4] or 2048), int(a[5] or 200)
prec = os.environ.get("RACE_PRECISION", "fp32")
lib = ctypes.CDLL(_lib.LIB_PATH)
lib.adrp_gjk_dump_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_int]
lib.adrp_gjk_dump_read.restype = ctypes.c_int
env = MultiRaceAviary(level, num_drones=n, physics=Physics[phys], racemode=RaceMode[mode], num_envs=E, seed=7,
                      precision=prec)
obs0, _ = env.reset()
pol = os.environ.get("RACE_POLICY")
if pol:
    from bench import make_policy
    policy = make_policy(pol, env.device.index or 0)
    pact = torch.empty((E, n, 4), device=env.device)

    def step():
        policy.act(env._obs, out=pact)
        return env.step(pact)
else:
    gen = torch.Generator(device=env.device)
    gen.manual_seed(3)
    tgt = obs0[..., :3] + torch.rand((E, n, 3), generator=gen, device=env.device) * 0.6 - 0.3
    act = torch.cat([tgt, torch.zeros((E, n, 1), device=env.device)], -1).contiguous()

    def step():
        return env.step(act)
buf = (ctypes.c_double * (64 * 40))()
lib.adrp_gjk_dump_read(buf, 64, int(prec == "fp64"), 1)
for _ in range(steps):
    step()
torch.cuda.synchronize()
m = lib.adrp_gjk_dump_read(buf, 64, int(prec == "fp64"), 1)
rec = np.array(list(buf), dtype=np.float64).reshape(64, 40)[:max(m, 0)]
out = []
for r in rec:
    sh = []
    for j in range(2):
        p = r[17 * j:17 * j + 17]
        sh.append(np.concatenate([[p[16]], p[0:3], p[3:12], p[12:15], [p[15]]]))   # oracle layout
    out.append(sh)
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/gjk_capped_{level}_{n}_{phys}_{prec}{'_' + pol if pol else ''}.npz", rec=rec, shapes=np.array(out))
print(json.dumps({"capped": int(m), "cut": [float(x) for x in rec[:, 34]], "last_v": [float(np.sqrt(x)) for x in rec[:, 35]],
                  "kinds": [f"{int(x[16])}/{int(x[33])}" for x in rec]}), flush=True)
