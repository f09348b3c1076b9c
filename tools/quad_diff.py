"""Quad (four lanes per drone) vs one-lane race kernel on the same envs: 40 auto-reset env.steps,
bitwise comparison of obs / reward / terminated / truncated and of the final state.

usage: [ADRP_LIB=...] python tools/quad_diff.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics, RaceMode  # noqa: E402

CASES = [("level0", 2, "PYB", "COMPARE", 300), ("level3", 4, "PYB_DW", "COMPETE", 333),
         ("level0", 2, "PYB", "COMPARE", 2048), ("level3", 4, "PYB_DW", "COMPETE", 4096)]
for level, N, ph, mode, E in CASES:
    runs = []
    for quad in ("1", "0"):
        os.environ["ADRP_RACE_QUAD"] = quad
        env = MultiRaceAviary(level, num_drones=N, physics=Physics[ph], racemode=RaceMode[mode], num_envs=E, seed=3,
                              autoreset=True, reward="wrapper")
        obs, _ = env.reset()
        gen = torch.Generator(device=env.device)
        gen.manual_seed(4)
        tgt = obs[..., :3] + torch.rand((E, N, 3), generator=gen, device=env.device) * 0.6 - 0.3
        tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
        act = torch.cat([tgt, torch.zeros((E, N, 1), device=env.device)], -1).contiguous()
        seq = []
        for _ in range(40):
            o, r, te, tr, _ = env.step(act)
            seq.append(torch.cat([o.reshape(E, -1), r.reshape(E, 1), te.reshape(E, 1).float(), tr.reshape(E, 1).float()], 1).cpu())
        f, i = env.get_state()
        runs.append((torch.stack(seq).numpy(), f.cpu().numpy(), i.cpu().numpy()))
        env.close()
    (sa, fa, ia), (sb, fb, ib) = runs
    same = np.array_equal(sa, sb) and np.array_equal(fa, fb, equal_nan=True) and np.array_equal(ia, ib)
    d = np.abs(sa - sb)
    print(f"{level} N={N} {ph} {mode} E={E}: bit-identical={same} max|dobs|={np.nanmax(d):.3e} "
          f"differing obs entries={(d > 0).sum()} of {d.size}, int state mismatches={(ia != ib).sum()}", flush=True)
