"""Per-phase cost of race_step_kernel (needs the timing build: make -C gym_pybullet_adrp_amd/csrc timing).

usage: ADRP_LIB=gym_pybullet_adrp_amd/libadrp_timing.so python tools/race_phases.py [LEVEL DRONES PHYSICS MODE E]
       RACE_POLICY=example|twogates: setpoints from the on-device PPO actor (closed loop) instead of
       fixed random targets; RACE_PRECISION=fp64: the float64 kernel
Prints, per configuration, the s_memtime cycles per wave spent in each phase (mean over
waves, and the slowest wave per launch averaged over launches) and the kernel time from
dispatch events.
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

PHASES = ["setup", "physics", "controller", "rays", "obs", "contacts", "tail", "total"]
CONFIGS = [("level0", 2, "PYB", "COMPARE", 2048), ("level3", 4, "PYB_DW", "COMPETE", 4096),
           ("level3", 4, "PYB_DW", "COMPARE", 4096), ("level0", 4, "PYB", "COMPARE", 4096)]
if len(sys.argv) > 5:
    CONFIGS = [(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]))]

lib = ctypes.CDLL(_lib.LIB_PATH)
lib.adrp_race_phase_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
PREC = os.environ.get("RACE_PRECISION", "fp32")
wave_read = lib.adrp_race_wave_read_f64 if PREC == "fp64" else lib.adrp_race_wave_read
wave_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 32)()
QUAD = os.environ.get("ADRP_RACE_QUAD", "1") != "0"

for level, n, phys, mode, E in CONFIGS:
    env = MultiRaceAviary(level, num_drones=n, physics=Physics[phys], racemode=RaceMode[mode], num_envs=E, seed=7,
                          precision=PREC)
    obs0, _ = env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(3)
    off = torch.rand((16, E, n, 3), generator=gen, device=env.device) * 0.6 - 0.3
    tgt = obs0[..., :3].unsqueeze(0) + off
    tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
    acts = torch.cat([tgt, torch.zeros((16, E, n, 1), device=env.device)], -1).contiguous()
    pol = os.environ.get("RACE_POLICY")
    if pol:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)) + "/..")
        from bench import make_policy
        policy = make_policy(pol, env.device.index or 0)
        pact = torch.empty((E, n, 4), device=env.device)

        def step(_a):
            policy.act(env._obs, out=pact)
            return env.step(pact)
    else:
        step = env.step
    for k in range(100):
        step(acts[k % 16])
    torch.cuda.synchronize()
    lib.adrp_race_phase_read(buf, 1)
    nk = 100
    if QUAD:   # four-lane kernel: per-workgroup slots (no same-address atomics)
        G = 1 if n <= 1 else 2 if n <= 2 else 4 if n <= 4 else 8
        nb = (E * G * 4 + 63) // 64
        wbuf = (ctypes.c_ulonglong * (nb * 8))()
        means, maxs, slowest, pct = [], [], [], []
        done = 0.0
        env.h.profile_begin(nk)
        for k in range(nk):
            _, _, te, tr, _ = step(acts[k % 16])
            torch.cuda.synchronize()
            done += float((te | tr).float().mean())
            assert wave_read(wbuf, nb) == 0
            w = np.array(list(wbuf), dtype=np.float64).reshape(nb, 8)
            means.append(w.mean(0))
            maxs.append(w.max(0))
            slowest.append(w[int(w[:, 7].argmax())])
            pct.append(np.percentile(w[:, 7], [50, 90, 99, 100]))
        ms = env.h.profile_end(nk)
        lib.adrp_race_phase_read(buf, 1)   # GJK counters (timing build with -DADRP_RACE_GJK_STATS)
        gv = np.array(list(buf), dtype=np.float64)
        print(json.dumps({"config": f"{level} N={n} {phys} {mode} E={E}", "kernel": env.kernel_name,
                          "gjk": {"calls_per_launch": gv[9] / nk, "mean_iters": gv[18] / max(gv[9], 1),
                                  "max_iters": gv[19], "contact_calls_per_launch": gv[20] / nk,
                                  "contact_max_iters": gv[21], "capped_calls": gv[22]},
                          "kernel_us_timing_build": float(np.mean(ms)) * 1e3,
                          "kernel_us_median": float(np.median(ms)) * 1e3,
                          "reset_env_fraction_per_step": done / nk,
                          "mean_cycles_per_wave": {p: round(x) for p, x in zip(PHASES, np.mean(means, 0))},
                          "max_cycles_per_launch": {p: round(x) for p, x in zip(PHASES, np.mean(maxs, 0))},
                          "slowest_wave_phases": {p: round(x) for p, x in zip(PHASES, np.mean(slowest, 0))},
                          "wave_total_p50_p90_p99_max": [round(x) for x in np.mean(pct, 0)]}),
              flush=True)
        env.close()
        continue
    sums = np.zeros(32)
    mx = np.zeros(8)
    gjk_max = 0
    env.h.profile_begin(nk)
    for k in range(nk):
        step(acts[k % 16])
        torch.cuda.synchronize()
        lib.adrp_race_phase_read(buf, 1)
        v = np.array(list(buf), dtype=np.float64)
        sums += v
        mx += v[10:18]
        gjk_max = max(gjk_max, v[19])
    ms = env.h.profile_end(nk)
    waves = sums[8]
    mean = {p: sums[i] / waves for i, p in enumerate(PHASES)}
    slow = {p: mx[i] / nk for i, p in enumerate(PHASES)}
    print(json.dumps({"config": f"{level} N={n} {phys} {mode} E={E}", "kernel": _lib.kernel_name(env.cfg),
                      "kernel_us": float(np.mean(ms)) * 1e3,
                      "mean_cycles_per_wave": {k: round(x) for k, x in mean.items()},
                      "max_cycles_per_launch": {k: round(x) for k, x in slow.items()},
                      "gjk": {"calls_per_launch": sums[9] / nk, "mean_iters": sums[18] / max(sums[9], 1),
                              "max_iters": gjk_max}}), flush=True)
    env.close()
