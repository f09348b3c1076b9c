"""Run N eager MultiRaceAviary steps (for rocprofv3 --pmc passes of race_step_kernel).

usage: python tools/pmc_race_steps.py LEVEL DRONES PHYSICS RACEMODE E N [ROOT] [PRECISION]
Actions follow bench.py's race protocol (start pose + U(+-0.3) m targets).
"""
import sys

import torch

level, drones, physics, mode, E, N = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]), \
    int(sys.argv[6])
sys.path.insert(0, sys.argv[7] if len(sys.argv) > 7 else ".")
prec = sys.argv[8] if len(sys.argv) > 8 else "fp32"
from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics, RaceMode  # noqa: E402

env = MultiRaceAviary(level, num_drones=drones, physics=Physics[physics], racemode=RaceMode[mode],
                      num_envs=E, seed=2024, precision=prec)
obs0, _ = env.reset()
gen = torch.Generator(device=env.device)
gen.manual_seed(1)
off = torch.rand((8, E, drones, 3), generator=gen, device=env.device) * 0.6 - 0.3
tgt = obs0[..., :3].unsqueeze(0) + off
tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
acts = torch.cat([tgt, torch.zeros((8, E, drones, 1), device=env.device)], -1).contiguous()
for k in range(N):
    env.step(acts[k % 8])
torch.cuda.synchronize()
print("step_bytes", env.step_bytes(), "E", E, "N", N)
