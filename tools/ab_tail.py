"""A/B/n of the race step kernel's per-launch time distribution (mean / median / p99 / max of the
dispatch events, adrp_profile_begin / _end), arms interleaved, one child process per (arm, workload).

usage: python tools/ab_tail.py OUT_JSON ROUNDS STEPS LIB[,VAR=value ...] [LIB ...]
workloads: config 3 + actor (fp32, fp64), config 4 (fp64) -- bench.py's shapes and seeds
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORK = {"c3p_fp32": ("level0", 2, "PYB", "COMPARE", 2048, "fp32", "example"),
        "c3p_fp64": ("level0", 2, "PYB", "COMPARE", 2048, "fp64", "example"),
        "c4_fp64": ("level3", 4, "PYB_DW", "COMPETE", 4096, "fp64", None),
        "c3_fp64": ("level0", 2, "PYB", "COMPARE", 2048, "fp64", None)}


def child(work, steps):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import bench
    level, n, phys, mode, E, prec, pol = WORK[work]
    dev = 0
    torch.cuda.set_device(dev)
    env = bench.race_make(level, n, phys, mode, prec, dev)(num_envs=E, env_offset=0)
    obs0, _ = env.reset()
    acts = bench.race_actions(obs0.clone(), dev, 2024)
    if pol:
        policy = bench.make_policy(pol, dev)
        pact = torch.empty((E, n, 4), device=env.device)

        def step(k):
            policy.act(env._obs, out=pact)
            env.step(pact)
    else:
        def step(k):
            env.step(acts[k % acts.shape[0]])
    for k in range(200):
        step(k)
    torch.cuda.synchronize()
    env.h.profile_begin(steps)
    for k in range(steps):
        step(k)
    t = np.asarray(env.h.profile_end(steps), dtype=np.float64) * 1e3   # us
    print(json.dumps({"mean": t.mean(), "p50": float(np.median(t)), "p99": float(np.percentile(t, 99)),
                      "max": float(t.max()), "n": int(len(t))}), flush=True)


def main(out, rounds, steps, arms):
    rec = {"steps": steps, "rounds": rounds, "arms": arms, "res": {}}
    for r in range(rounds):
        for work in ("c3p_fp32", "c3p_fp64", "c4_fp64", "c3_fp64"):
            for arm in arms:
                parts = arm.split(",")
                env = dict(os.environ, ADRP_LIB=parts[0], **dict(p.split("=", 1) for p in parts[1:]))
                p = subprocess.run([sys.executable, __file__, "--child", work, str(steps)], env=env,
                                   capture_output=True, text=True, timeout=240)
                line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 and p.stdout.strip() else None
                res = json.loads(line) if line else {"rc": p.returncode, "err": p.stderr[-400:]}
                rec["res"].setdefault(work, {}).setdefault(arm, []).append(res)
                print(f"{work:9s} {arm:50s} {line or p.stderr[-400:]}", flush=True)
                if not line:
                    json.dump(rec, open(out, "w"), indent=1)
                    sys.exit(1)
    json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
    else:
        main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:])
