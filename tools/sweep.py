"""Env-count sweep of the HoverAviary step (graph replay, device time per step)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Physics  # noqa: E402


def run(E, physics="PYB", precision="fp32", G=32, reps=10):
    env = HoverAviary(physics=Physics[physics], num_envs=E, precision=precision, initial_xyzs=[0, 0, 1.0],
                      init_noise={"xyz": 0.1, "rpy": 0.05, "vel": 0.1, "omega": 0.1})
    env.reset()
    acts = torch.rand((8, E, 1, 4), device=env.device) * 2 - 1
    for k in range(3):
        env.step(acts[k])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        env.step(acts[0])
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for k in range(G):
            env.step(acts[k % 8])
    g.replay(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (reps * G)
    by = env.step_bytes()
    env.close()
    return {"E": E, "physics": physics, "precision": precision, "us_per_step": dt * 1e6,
            "env_steps_per_s": E / dt, "GBps_alg": by / dt / 1e9, "frac_hbm": by / dt / 8e12}


if __name__ == "__main__":
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4096, 16384, 65536, 262144, 1048576]
    precs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp32"]
    for p in precs:
        for E in sizes:
            print(json.dumps(run(E, precision=p)), flush=True)
