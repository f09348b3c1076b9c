"""Where the driver-form (K = 20) bench line's time goes outside the kernels: one 20-step HIP graph
of the config-2 hover step (4,096 envs, fp64) replayed N times per variant, variants interleaved,
host clock per replay (median, us).

usage: python tools/replay_probe.py [OUT_JSON] [REPS]
  timed     perf_counter; ev0.record; replay; ev1.record; synchronize   (bench.py time_graph, K = 20)
  noevent   perf_counter; replay; synchronize
  evsync    perf_counter; ev0.record; replay; ev1.record; ev1.synchronize
  launch    perf_counter around replay() alone (the host cost of the launch call)
  tiny      the timed form over a 20-node graph of 1-element adds (the fixed cost with ~no kernel time)
  events    ev0 -> ev1 device time of the timed form / 20 (the bench's kernel_us)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(out=None, reps=300):
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
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(20):
            env.step(acts[k])
    gt = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gt):
        for k in range(20):
            x.add_(1)
    for _ in range(3):
        g.replay()
        gt.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: [] for k in ("timed", "noevent", "evsync", "launch", "tiny", "events")}
    pc = time.perf_counter
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = pc(); ev0.record(); g.replay(); ev1.record(); torch.cuda.synchronize(); t1 = pc()
        res["timed"].append(t1 - t0)
        res["events"].append(ev0.elapsed_time(ev1) * 1e-3)
        torch.cuda.synchronize()
        t0 = pc(); g.replay(); torch.cuda.synchronize(); t1 = pc()
        res["noevent"].append(t1 - t0)
        torch.cuda.synchronize()
        t0 = pc(); ev0.record(); g.replay(); ev1.record(); ev1.synchronize(); t1 = pc()
        res["evsync"].append(t1 - t0)
        torch.cuda.synchronize()
        t0 = pc(); g.replay(); t1 = pc()
        res["launch"].append(t1 - t0)
        torch.cuda.synchronize()
        t0 = pc(); ev0.record(); gt.replay(); ev1.record(); torch.cuda.synchronize(); t1 = pc()
        res["tiny"].append(t1 - t0)
    rec = {k: {"median_us": float(np.median(v)) * 1e6, "p10_us": float(np.percentile(v, 10)) * 1e6,
               "p90_us": float(np.percentile(v, 90)) * 1e6} for k, v in res.items()}
    rec["env"] = {k: os.environ.get(k) for k in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "DEBUG_HIP_GRAPH_BATCH_SIZE",
                                                 "HIP_FORCE_DEV_KERNARG")}
    rec["reps"] = reps
    print(json.dumps(rec, indent=1))
    if out:
        with open(out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None, int(sys.argv[2]) if len(sys.argv) > 2 else 300)
