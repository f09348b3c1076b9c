"""Benchmark: HoverAviary env.step throughput (BASELINE.json configs[1]) on N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one env.step() of every env on every GPU: per GPU one fused launch over
4096 envs x 8 PYB sub-steps (240 Hz physics, 30 Hz control) incl. obs/reward/
termination and auto-reset.  Envs are sharded across ranks (weak scaling, no collective
on the step path).  Inputs are resident in HBM before the timed region: per-env random
airborne initial states (device RNG) and a pre-generated buffer of U[-1,1] actions.

Prints ONE JSON line on rank 0 with the roofline of the step kernel (per-launch HIP
events on the launching stream) and a CPU baseline (the float64 oracle, one host core,
bounded sample) timed in the same run.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
ENVS_PER_GPU = 4096         # BASELINE.json configs[1]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    p.add_argument("--physics", default="PYB")
    p.add_argument("--precision", default="fp32")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-allgather", action="store_true", help="N>1: skip the obs all-gather variant")
    p.add_argument("--task", default="hover", choices=["hover", "race"],
                   help="hover = BASELINE configs[1] (default); race = configs[2]/[3] (MultiRaceAviary)")
    p.add_argument("--level", default="level0", help="race: track preset (level0 = config 3, level3 = config 4)")
    p.add_argument("--drones", type=int, default=2, help="race: drones per env")
    p.add_argument("--racemode", default="COMPARE", choices=["COMPARE", "COMPETE"])
    p.add_argument("--no-sweep", action="store_true", help="hover: skip the env-count roofline sweep")
    p.add_argument("--policy", default=None,
                   help="race: closed loop with the on-device PPO actor: 'example' / 'twogates' (the reference's "
                        "user_controller zips, weights from tests/golden/policy_golden.npz) or a SB3 zip path")
    return p.parse_args()


def roofline_sweep(make, sizes, launches=30):
    """The same step kernel at larger env counts (one GPU): where the launch leaves the latency-bound
    regime of E = 4096 and becomes HBM-bound.  Kernel time from dispatch-attached events."""
    out = []
    for n in sizes:
        env = make(num_envs=n, env_offset=0)
        env.reset()
        a = torch.rand((4, n, 1, 4), device=env.device) * 2 - 1
        for k in range(5):
            env.step(a[k % 4])
        torch.cuda.synchronize()
        env.h.profile_begin(launches)
        for k in range(launches):
            env.step(a[k % 4])
        us = float(np.mean(env.h.profile_end(launches))) * 1e3
        gbps = env.step_bytes() / (us * 1e-6) / 1e9
        out.append({"envs": n, "kernel_us": us, "env_steps_per_s": n / (us * 1e-6), "achieved_GBps": gbps,
                    "frac": gbps / HBM_PEAK_GBPS})
        env.close()
        del a
    return out


def make_policy(spec, device, racemode):
    from gym_pybullet_adrp_amd.policy import ACTOR_KEYS, DevicePolicy
    mode = "absolute" if spec == "twogates" else "relative"     # RLControllerTwoGates / RLController
    if spec in ("example", "twogates"):
        g = np.load(os.path.join(ROOT, "tests", "golden", "policy_golden.npz"))
        name = "example_RL_model" if spec == "example" else "twogates"
        w = {k: g[f"{name}_w{i}"] for i, k in enumerate(ACTOR_KEYS)}
        return DevicePolicy(w, "relu" if bool(g[f"{name}_relu"]) else "tanh", device, mode)
    return DevicePolicy.from_zip(spec, device, mode)


def cpu_baseline(cfg, seconds):
    """float64 oracle (oracle/oracle.c), single host thread, bounded sample of the same
    workload: 4096 envs stepped until ~`seconds` of CPU time."""
    from oracle import oracle as O
    c = cfg.copy()
    race = c.task == 1
    c.num_envs = 256 if race else ENVS_PER_GPU
    c.env_offset = 0
    orc = O.Oracle(c)
    obs0 = orc.reset()
    rng = np.random.default_rng(1)
    if race:
        t = obs0[None, ..., :3] + rng.uniform(-0.3, 0.3, (8,) + obs0.shape[:2] + (3,))
        t[..., 2] = np.clip(t[..., 2], 0.2, 1.5)
        acts = np.concatenate([t, np.zeros(t.shape[:-1] + (1,))], -1).astype(np.float32)
    else:
        acts = rng.uniform(-1, 1, (8, c.num_envs, 1, 4)).astype(np.float32)
    orc.step(acts[0])                     # warm
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.step(acts[steps % 8])
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": c.num_envs * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{c.num_envs} envs x {steps} env.steps (float64 oracle, {dt:.1f} s, 1 thread, "
                      f"{platform.processor() or platform.machine()})"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    import functools
    from gym_pybullet_adrp_amd import _lib
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    from gym_pybullet_adrp_amd.utils.enums import Physics

    E = args.envs
    if args.task == "race":
        from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary
        from gym_pybullet_adrp_amd.utils.enums import RaceMode
        make = functools.partial(MultiRaceAviary, args.level, num_drones=args.drones, physics=Physics[args.physics],
                                 racemode=RaceMode[args.racemode], device=local, precision=args.precision, seed=2024)
    else:
        make = functools.partial(HoverAviary, physics=Physics[args.physics], device=local, precision=args.precision,
                                 seed=2024, initial_xyzs=[0, 0, 1.0],
                                 init_noise={"xyz": 0.1, "rpy": 0.05, "vel": 0.1, "omega": 0.1})
    sharded = None
    if world > 1:
        from gym_pybullet_adrp_amd.sharding import ShardedAviary
        sharded = ShardedAviary(E * world, make)     # rank r owns global envs [r*E, (r+1)*E)
        env = sharded.env
    else:
        env = make(num_envs=E, env_offset=0)
    dev = env.device
    obs0, _ = env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    nbuf = 64
    if args.task == "race":
        # FULLSTATE targets = start + U(+-0.3) m, z clipped to [0.2, 1.5], yaw 0
        # (re-drawn per buffer slot)
        N = args.drones
        off = (torch.rand((nbuf, E, N, 3), generator=gen, device=dev) * 0.6 - 0.3)
        tgt = obs0[..., :3].unsqueeze(0) + off
        tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
        acts = torch.cat([tgt, torch.zeros((nbuf, E, N, 1), device=dev)], -1).contiguous()
    else:
        acts = (torch.rand((nbuf, E, 1, 4), generator=gen, device=dev) * 2 - 1).contiguous()
    policy = None
    if args.policy:
        if args.task != "race":
            raise SystemExit("--policy drives MultiRaceAviary (FULLSTATE setpoints)")
        policy = make_policy(args.policy, local, args.racemode)
        pact = torch.empty((E, args.drones, 4), device=dev)

        class _Loop:   # one "step" = policy forward on the current obs + env.step on its setpoints
            def step(self, _a):
                policy.act(env._obs, out=pact)
                return env.step(pact)
        stepper = _Loop()
    else:
        stepper = env
    for k in range(args.warmup):
        stepper.step(acts[k % nbuf])
    torch.cuda.synchronize()

    # ---- timed region: exactly K env.steps, replayed from a captured HIP graph ----
    K = args.steps
    G = max(g for g in range(1, min(K, 256) + 1) if K % g == 0)   # steps per graph, G | K
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        stepper.step(acts[0])
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for k in range(G):
            stepper.step(acts[k % nbuf])
    graph.replay()                                           # untimed: warms the graph
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K // G):
        graph.replay()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())

    # ---- kernel duration: HIP start/stop events attached to each step kernel's own
    # dispatch (hipExtLaunchKernelGGL inside libadrp) on the launching stream, over nk launches
    nk = min(K, 512)
    torch.cuda.synchronize()
    env.h.profile_begin(nk)
    for k in range(nk):
        env.step(acts[k % nbuf])
    kern_ms = env.h.profile_end(nk)
    kern_avg_s = float(np.mean(kern_ms)) / 1e3
    policy_rec = None
    if policy is not None:   # policy launches are on torch's current stream: torch events see them
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
        for a, b in ev:
            a.record()
            policy.act(env._obs, out=pact)
            b.record()
        torch.cuda.synchronize()
        pol_us = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
        rows = E * args.drones
        flops = 2 * rows * (policy.in_dim * policy.h1 + policy.h1 * policy.h2 + policy.h2 * 4)
        policy_rec = {"weights": args.policy, "arch": f"{policy.in_dim}-{policy.h1}-{policy.h2}-4",
                      "kernel_us": pol_us, "rows": rows, "flops": flops,
                      "mfma_f32": {"achieved_tflops": flops / pol_us / 1e6, "unit": "TFLOP/s"},
                      "bytes": rows * (env.h.D + 4) * 4,
                      "note": "event pairs around each policy launch on the current stream"}

    # ---- eager (no graph) end-to-end rate, for reference ----
    torch.cuda.synchronize()
    te0 = time.perf_counter()
    ne = min(K, 1000)
    for k in range(ne):
        env.step(acts[k % nbuf])
    torch.cuda.synchronize()
    eager = {"env_steps_per_s_per_gpu": E * ne / (time.perf_counter() - te0),
             "ms_per_step": (time.perf_counter() - te0) / ne * 1e3}

    # ---- config 5 variant (N > 1): every step followed by the RCCL all-gather that
    # reassembles obs/reward/flags for a learner (eager; not part of `value`) ----
    allgather = None
    if sharded is not None and not args.no_allgather:
        ng = min(K, 500)
        for k in range(10):
            sharded.gather(*env.step(acts[k % nbuf])[:4])
        torch.cuda.synchronize()
        dist.barrier()
        tg0 = time.perf_counter()
        for k in range(ng):
            sharded.gather(*env.step(acts[k % nbuf])[:4])
        torch.cuda.synchronize()
        tg = torch.tensor([time.perf_counter() - tg0], dtype=torch.float64, device=dev)
        dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        tg = float(tg.item())
        allgather = {"value": E * world * ng / tg, "unit": "env-steps/s", "ms_per_step": tg / ng * 1e3,
                     "steps": ng, "collective": "all_gather_into_tensor (RCCL) of packed fp32 obs+reward+flags",
                     "bytes_per_rank_per_step": E * (env.h.D + 3) * 4}

    bytes_per_launch = env.step_bytes()
    achieved = bytes_per_launch / kern_avg_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            rec = json.load(fh)
        key = f"{args.physics}_{args.precision}_{E}" if args.task == "hover" else \
            f"race_{args.level}_{args.drones}_{args.physics}_{args.precision}_{E}"
        if key in rec:
            traffic = rec[key]["hbm_bytes_per_launch"]
    result = {
        "metric": "env-steps/sec (N parallel drones) at 1/2/4/8 MI355X; % HBM roofline",
        "value": E * world * K / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "f64",
        "data": "synthetic: device-RNG airborne initial states around (0,0,1), U[-1,1] RPM actions",
        "config": {"workload": f"HoverAviary Physics.{args.physics} 240/30 Hz (8 sub-steps), {E} envs x 1 drone "
                               f"per GPU, RPM actions, auto-reset", "envs_per_gpu": E, "global_envs": E * world,
                   "drones_per_env": 1, "parallelism": f"env-sharded dp{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "bytes_per_launch": bytes_per_launch, "kernel_us": kern_avg_s * 1e6,
                     "kernel_us_median": float(np.median(kern_ms)) * 1e3, "timed_launches": int(len(kern_ms))},
        "timing": {"timed_region": f"{K // G} replays of a {G}-step HIP graph (one fused launch per env.step)",
                   "eager": eager},
        "kernel": _lib.kernel_name(env.cfg),
    }
    if allgather is not None:
        result["with_obs_allgather"] = allgather
    if args.task == "race":
        result["config"] = {"workload": f"MultiRaceAviary {args.racemode} {args.level}, {args.drones} drones x {E} envs "
                                        f"per GPU, Physics.{args.physics} 500/25 Hz (20 sub-steps, Mellinger 500 Hz)",
                            "envs_per_gpu": E, "global_envs": E * world, "drones_per_env": args.drones,
                            "parallelism": f"env-sharded dp{world}"}
        result["data"] = "synthetic: level preset resets (device Philox), FULLSTATE targets start + U(+-0.3) m"
        result["drone_steps_per_s"] = result["value"] * args.drones
        if policy_rec is not None:
            result["config"]["workload"] += f"; closed loop: on-device PPO actor ({args.policy}) each step"
            result["data"] = "synthetic: level preset resets (device Philox); setpoints from the reference's PPO actor"
            result["policy"] = policy_rec
    if args.task == "hover" and world == 1 and not args.no_sweep and policy is None:
        result["roofline"]["sweep"] = roofline_sweep(make, [65536, 262144, 1048576])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(env.cfg, args.cpu_seconds)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if policy is not None:
        policy.close()
    env.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
