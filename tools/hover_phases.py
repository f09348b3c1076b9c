"""Per-phase cost of hover_step_kernel (needs the timing build: make -C gym_pybullet_adrp_amd/csrc timing).

usage: ADRP_LIB=gym_pybullet_adrp_amd/libadrp_timing.so [HOVER_PRECISION=fp64] python tools/hover_phases.py [E ...]
Workload = bench.py's default (airborne starts around (0,0,1), U[-1,1] RPM actions, auto-reset).
Prints, per E, the s_memtime cycles per wave spent in each phase (mean over waves, and the
slowest wave per launch averaged over launches), the share of waves that ran the auto-reset
path, and the kernel time from dispatch events.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402

PHASES = ["loads", "substeps", "obs_flags", "reset", "obs_row", "state_stores", "total"]
SIZES = [int(x) for x in sys.argv[1:]] or [4096, 65536]

lib = ctypes.CDLL(_lib.LIB_PATH)
lib.adrp_race_phase_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 32)()

for E in SIZES:
    env = HoverAviary(num_envs=E, seed=2024, initial_xyzs=[0, 0, 1.0], precision=os.environ.get("HOVER_PRECISION", "fp32"),
                      init_noise={"xyz": 0.1, "rpy": 0.05, "vel": 0.1, "omega": 0.1})
    env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(1)
    acts = (torch.rand((64, E, 1, 4), generator=gen, device=env.device) * 2 - 1).contiguous()
    for k in range(200):
        env.step(acts[k % 64])
    torch.cuda.synchronize()
    lib.adrp_race_phase_read(buf, 1)
    nk = 200
    sums = np.zeros(32)
    mx = np.zeros(8)
    env.h.profile_begin(nk)
    for k in range(nk):
        env.step(acts[k % 64])
        torch.cuda.synchronize()
        lib.adrp_race_phase_read(buf, 1)
        v = np.array(list(buf), dtype=np.float64)
        sums += v
        mx += v[10:18]
    ms = env.h.profile_end(nk)
    waves = sums[8]
    print(json.dumps({"E": E, "kernel": env.kernel_name, "kernel_us": float(np.mean(ms)) * 1e3,
                      "mean_cycles_per_wave": {p: round(sums[i] / waves) for i, p in enumerate(PHASES)},
                      "max_cycles_per_launch": {p: round(mx[i] / nk) for i, p in enumerate(PHASES)},
                      "waves_with_reset": sums[9] / waves, "done_lanes_per_step": sums[7] / nk}), flush=True)
    env.close()
