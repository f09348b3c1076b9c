"""Probe: can torch timing events be recorded inside a captured HIP graph on this stack?"""
import sys
import torch
sys.path.insert(0, ".")
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402

env = HoverAviary(num_envs=4096, initial_xyzs=[0, 0, 1.0])
env.reset()
acts = torch.rand((8, 4096, 1, 4), device=env.device) * 2 - 1
for k in range(3):
    env.step(acts[k])
torch.cuda.synchronize()
G = 16
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    env.step(acts[0])
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g):
        for k in range(G):
            ev[k][0].record()
            env.step(acts[k % 8])
            ev[k][1].record()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print("events in graph OK:", [round(a.elapsed_time(b) * 1e3, 2) for a, b in ev])
except Exception as exc:
    print("events in graph FAILED:", repr(exc)[:300])
