"""Host-side wait mode vs the driver-form (K = 20) bench line: the config-2 hover step (4,096 envs,
fp64) as one 20-step HIP graph, timed as bench.py's time_graph times it (perf_counter; ev0.record;
replay; ev1.record; torch.cuda.synchronize), per replay; and the same over a 20-node graph of 1-element
adds (the fixed cost).  One child process per device-flag variant (hipSetDeviceFlags must precede the
runtime's device initialisation): 0 auto (the runtime default), 1 spin, 2 yield, 4 blocking sync.

usage: python tools/sync_probe.py [OUT_JSON] [REPS]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(flags, reps):
    import ctypes

    import numpy as np
    import torch
    if flags >= 0:
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(flags))
        assert rc == 0, f"hipSetDeviceFlags({flags}) = {rc}"
    sys.path.insert(0, ROOT)
    import bench
    dev = 0
    torch.cuda.set_device(dev)
    env = bench.hover_make("fp64", "PYB", dev)(num_envs=4096, env_offset=0)
    env.reset()
    acts = bench.hover_actions(4096, dev, 1)
    for k in range(10):
        env.step(acts[k])
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        env.step(acts[0])
        x = torch.zeros(1, device=dev)
        x.add_(1)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g, gt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(20):
            env.step(acts[k])
    with torch.cuda.graph(gt):
        for k in range(20):
            x.add_(1)
    for _ in range(3):
        g.replay()
        gt.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"timed": [], "events": [], "tiny": [], "sync_idle": []}
    pc = time.perf_counter
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = pc(); ev0.record(); g.replay(); ev1.record(); torch.cuda.synchronize(); t1 = pc()
        res["timed"].append(t1 - t0)
        res["events"].append(ev0.elapsed_time(ev1) * 1e-3)
        torch.cuda.synchronize()
        t0 = pc(); ev0.record(); gt.replay(); ev1.record(); torch.cuda.synchronize(); t1 = pc()
        res["tiny"].append(t1 - t0)
        t0 = pc(); torch.cuda.synchronize(); t1 = pc()
        res["sync_idle"].append(t1 - t0)
    out = {k: {"median_us": float(np.median(v)) * 1e6, "p10_us": float(np.percentile(v, 10)) * 1e6,
               "p90_us": float(np.percentile(v, 90)) * 1e6} for k, v in res.items()}
    out["timed_per_step_us"] = out["timed"]["median_us"] / 20
    print(json.dumps(out), flush=True)


def main(out=None, reps=300):
    rec = {"reps": reps}
    for rnd in range(2):   # two interleaved rounds
        for flags in (-1, 1, 2, 4):
            p = subprocess.run([sys.executable, __file__, "--child", str(flags), str(reps)], capture_output=True,
                               text=True, timeout=300)
            line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 and p.stdout.strip() else None
            rec.setdefault(str(flags), []).append(json.loads(line) if line else {"rc": p.returncode,
                                                                               "err": p.stderr[-600:]})
            print(flags, line if line else p.stderr[-600:], flush=True)
    rec["variants"] = {"-1": "no hipSetDeviceFlags call (runtime default)", "1": "hipDeviceScheduleSpin",
                       "2": "hipDeviceScheduleYield", "4": "hipDeviceScheduleBlockingSync"}
    if out:
        with open(out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]))
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else None, int(sys.argv[2]) if len(sys.argv) > 2 else 300)
