"""Host-path cost breakdown: where the time of a Python-driven env.step goes.

usage: python tools/host_path.py   (one GPU)
E = 1 (BASELINE config 1, examples/pid.py-style loop): env.step launch only, + stream sync, + device
sync, + event spin, the ctypes call alone; E = 4096: the SB3 VecEnv step (packed host path) split
into its parts.  Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.vec_env import AviaryVecEnv  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


out = {}
for prec in ("fp64", "fp32"):
    env = HoverAviary(num_envs=1, precision=prec, initial_xyzs=[0, 0, 1.0], seed=1)
    env.reset()
    a = torch.rand((1, 1, 4), device=env.device) * 2 - 1
    s = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    r = {}
    r["launch_only_us"] = per_call(lambda: env.step(a))
    r["step_stream_sync_us"] = per_call(lambda: (env.step(a), s.synchronize()))
    r["step_device_sync_us"] = per_call(lambda: (env.step(a), torch.cuda.synchronize()))

    def spin():
        env.step(a)
        ev.record(s)
        while not ev.query():
            pass
    r["step_event_spin_us"] = per_call(spin)
    h = env.h
    args = (h.h, a.data_ptr(), env._obs.data_ptr(), env._rew.data_ptr(), env._term.data_ptr(), env._trunc.data_ptr(),
            env._tobs.data_ptr(), s.cuda_stream)
    r["ctypes_step_only_us"] = per_call(lambda: h._step(*args))
    r["obs_to_host_us"] = per_call(lambda: (env.step(a), env._obs.cpu()))
    env.h.profile_begin(500)
    for _ in range(500):
        env.step(a)
    r["kernel_us"] = float(np.mean(env.h.profile_end(500))) * 1e3
    out[f"E1_{prec}"] = r
    env.close()

E = 4096
acts = np.random.default_rng(1).uniform(-1, 1, (16, E, 1, 4)).astype(np.float32)
k = [0]
for name, kw in (("direct", {}), ("packed_copy", {"direct": False})):
    env = HoverAviary(num_envs=E, precision="fp64", initial_xyzs=[0, 0, 1.0], seed=1,
                      init_noise={"rpy": 0.3, "omega": 1.0})
    v = AviaryVecEnv(env, packed=True, **kw)
    v.reset()

    def vstep():
        k[0] += 1
        return v.step(acts[k[0] % 16])

    r = {"vecenv_step_us": per_call(vstep, 300)}
    if name == "direct":
        r["vec_step_call_us"] = per_call(lambda: v._vec_step(v._h, 1, 0), 300)
        r["act_write_us"] = per_call(lambda: v._act_np.__setitem__(Ellipsis, acts[3]), 300)
    else:
        r["act_in_us"] = per_call(lambda: v._act_in(acts[3]), 300)
        r["env_step_us"] = per_call(lambda: env.step(v._act_dev), 300)
        r["copy_out_us"] = per_call(lambda: v._copy_out(), 300)
        o = v._views[0][0]
        r["obs_numpy_copy_us"] = per_call(lambda: o.copy(), 300)
    out[f"E4096_vecenv_fp64_{name}"] = r
    if name == "direct":
        break_v = v
        continue
    v.close()
v = break_v
if os.environ.get("HOST_PATH_PROFILE"):
    import cProfile
    import io
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        vstep()
    torch.cuda.synchronize()
    pr.disable()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(18)
    print(sio.getvalue(), file=sys.stderr, flush=True)
v.close()
print(json.dumps(out), flush=True)
