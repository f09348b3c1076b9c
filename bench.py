"""Benchmark: vectorised gym-pybullet-adrp env.step throughput on N MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`value` is BASELINE.json configs[1] (HoverAviary, 4096 envs x 1 drone per GPU, PYB, 240/30 Hz =
8 sub-steps, RPM actions, auto-reset) at the reference's precision (float64 kernel; the
reference integrates in float64): one "step" = one env.step() of every env on every GPU, one
fused HIP launch per GPU, envs sharded across ranks (weak scaling, no collective on the step
path).  Inputs are resident in HBM before the timed region.  `--gpus N` without a launcher
starts N ranks itself (a child `torch.distributed.run`), before anything touches the GPU.

The same JSON line carries sub-records (`configs`), each timed the same way:
  config5      every N: MultiRaceAviary COMPETE level3, 4 drones x 4096 envs per GPU, PYB_DW,
               disturbances on (at N = 1 this is configs[3]), float64 physics + wrapper and
               float32 firmware as the reference; kernel-only, and (N > 1) step + RCCL
               all-gather of the packed obs/reward/flags captured in the same HIP graph;
               `strong`: 32,768 envs in total over the N GPUs
  config5_f32  every N: the same with the float32 kernel
  config3 / config3_f32  N = 1: MultiRaceAviary COMPARE level0, 2 drones x 2048 envs, PYB
  config3_policy  N = 1: config 3 (float64) driven by the reference's PPO actor on the device
  config4_gnd_drag_dw  N = 1: config 4 with Physics.PYB_GND_DRAG_DW (float64)
  config2_f32  N = 1: the `value` workload with the float32 kernel
  config1      N = 1: one HoverAviary env (E = 1), per-step latency: a launch per step, graph-replayed,
               and the persistent step kernel (numpy in / out, synchronous); the CPU oracle
Rooflines: the hover kernel is HBM-bound (bytes per launch / kernel time vs 8 TB/s); the race
kernel is VALU/issue-bound (PMC-counted flops per launch / kernel time vs the vector peak;
HBM fraction kept as information).  Kernel time = HIP events on the launching stream around
the timed region (K graph-replayed launches, one per step) / K; the per-dispatch events of
eager launches are kept beside it.  CPU baseline: the float64 oracle (test infrastructure)
on the host, one thread and the job's CPU share (OpenMP over envs), bounded samples.
"""
import argparse
import functools
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
VALU_F32_PEAK_TFLOPS = 157.3    # MI355X fp32 vector (FMA = 2 flops), MI355X_MICROARCH.md
VALU_F64_PEAK_TFLOPS = 78.6
ENVS_PER_GPU = 4096             # BASELINE.json configs[1]
METRIC = "env-steps/sec (N parallel drones) at 1/2/4/8 MI355X; % HBM roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    p.add_argument("--physics", default="PYB")
    p.add_argument("--precision", default="fp64", choices=["fp64", "fp32"],
                   help="main line kernel precision (fp64 = the reference's float64)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="per CPU-baseline leg")
    p.add_argument("--no-allgather", action="store_true", help="N>1: skip the obs all-gather variant")
    p.add_argument("--no-configs", action="store_true", help="only the main line (no config sub-records)")
    p.add_argument("--race-steps", type=int, default=200, help="timed steps of each race sub-record")
    p.add_argument("--task", default="hover", choices=["hover", "race"],
                   help="main line: hover = BASELINE configs[1] (default); race = configs[2]/[3]")
    p.add_argument("--level", default="level0", help="race main line: track preset")
    p.add_argument("--drones", type=int, default=2, help="race main line: drones per env")
    p.add_argument("--racemode", default="COMPARE", choices=["COMPARE", "COMPETE"])
    p.add_argument("--no-sweep", action="store_true", help="hover: skip the env-count roofline sweep")
    p.add_argument("--policy", default=None,
                   help="race main line: closed loop with the on-device PPO actor: 'example' / 'twogates' "
                        "(weights from tests/golden/policy_golden.npz) or a SB3 zip path")
    p.add_argument("--graph-only", action="store_true",
                   help="profiling runs (rocprofv3): no eager event-timed launches after the timed region, so "
                        "the kernel statistics are those of the graph-replayed launches")
    p.add_argument("--launch-check", action="store_true",
                   help="CPU-only check of the rank launch: every rank joins a gloo group, rank 0 prints the "
                        "record of the world it saw, no GPU work")
    p.add_argument("--gather-leg", action="store_true",
                   help="internal: run only config 5's world-1 RCCL step + all-gather record and print it "
                        "(the parent bench runs this as a child process)")
    p.add_argument("--gather-warmup", type=int, default=None, help="internal: --gather-leg warm-up steps")
    return p.parse_args()


# ----------------------------------------------------------------------------------------------
# rank launch
# ----------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without a launcher: run this script under torch.distributed.run as a child and
    return its exit code (no exec: this process never touches the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def launch_check(args, world, rank, out=None):
    dist.init_process_group("gloo")
    seen = dist.get_world_size()
    t = torch.tensor([rank, 1], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_arg": args.gpus, "world_seen": seen,
                          "ranks_reported": int(t[1]), "rank_sum": int(t[0])}), file=out or sys.stdout, flush=True)
    dist.barrier()
    dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------
# CPU side
# ----------------------------------------------------------------------------------------------
def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail
    return {"nproc": os.cpu_count(), "affinity": avail, "threads_allowed": min(share, avail), "model": model}


def _oracle_leg(cfg, E, acts_fn, seconds, threads):
    from oracle import oracle as O
    c = cfg.copy()
    c.num_envs, c.env_offset = E, 0
    O.set_threads(threads)
    try:
        orc = O.Oracle(c)
        obs0 = orc.reset()
        acts = acts_fn(obs0, E)
        orc.step(acts[0])                     # warm
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            orc.step(acts[steps % len(acts)])
            steps += 1
        dt = time.perf_counter() - t0
    finally:
        O.set_threads(1)
    return E * steps / dt, steps, dt


def _hover_acts(obs0, E):
    return np.random.default_rng(1).uniform(-1, 1, (8, E, 1, 4)).astype(np.float32)


def _race_acts(obs0, E):
    rng = np.random.default_rng(1)
    t = obs0[None, ..., :3] + rng.uniform(-0.3, 0.3, (8,) + obs0.shape[:2] + (3,))
    t[..., 2] = np.clip(t[..., 2], 0.2, 1.5)
    return np.concatenate([t, np.zeros(t.shape[:-1] + (1,))], -1).astype(np.float32)


def cpu_baseline(cfg, seconds, race=False):
    """The float64 oracle (oracle/oracle.c, test infrastructure) on the host: one thread and all of
    the job's cores (OpenMP over envs; results bit-identical, tests/test_oracle_threads.py)."""
    info = cpu_info()
    E = 256 if race else ENVS_PER_GPU
    fn = _race_acts if race else _hover_acts
    v1, n1, d1 = _oracle_leg(cfg, E, fn, seconds, 1)
    thr = info["threads_allowed"]
    vN, nN, dN = _oracle_leg(cfg, max(E, 8 * thr), fn, seconds, thr)
    return {"value": vN, "unit": "env-steps/s", "cores": thr, "kind": "port",
            "sample": f"{max(E, 8 * thr)} envs x {nN} env.steps, float64 oracle, {dN:.1f} s, OpenMP {thr} threads "
                      f"over envs (the job's CPU share: OMP_NUM_THREADS / affinity cap {thr} of {info['nproc']} "
                      f"host threads); {info['model']}",
            "one_core": {"value": v1, "cores": 1, "sample": f"{E} envs x {n1} env.steps, {d1:.1f} s, 1 thread"},
            "host": info}


# ----------------------------------------------------------------------------------------------
# GPU timing
# ----------------------------------------------------------------------------------------------
WATCHDOG_POLL_S = 0.25   # > ProcessGroupNCCL's watchdog sleep (100 ms): one poll retires finished works


def quiesce_collectives():
    """Nothing of ProcessGroupNCCL may be pending when a HIP graph capture begins.  Its watchdog
    thread polls every issued Work with an event query; a query from another thread while a
    GLOBAL-mode capture is open fails with hipErrorStreamCaptureUnsupported, the watchdog throws
    and the process terminates (BENCH_r04.json, rc 134).  So: finish the device work, then give the
    watchdog one poll to retire the (completed) works before the capture opens.  The capture itself
    is thread-local (`capture_graph`), so a late poll is legal as well."""
    torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        time.sleep(WATCHDOG_POLL_S)


def capture_graph(graph):
    """torch.cuda.graph in thread-local capture mode: only this thread's capture-unsafe calls are
    refused, so the RCCL watchdog's event queries on its own thread stay legal during a capture"""
    return torch.cuda.graph(graph, capture_error_mode="thread_local")


def time_graph(stepper, acts, K, W, world, dev):
    """W eager warm-up steps, then exactly K steps replayed from captured HIP graphs, bracketed by
    barrier + synchronize; returns the max over ranks of the timed region (s) and the graph size."""
    nbuf = acts.shape[0]
    for k in range(W):
        stepper.step(acts[k % nbuf])
    torch.cuda.synchronize()
    G = max(g for g in range(1, min(K, 256) + 1) if K % g == 0)   # steps per graph, G | K
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        stepper.step(acts[0])
    torch.cuda.current_stream(dev).wait_stream(side)
    quiesce_collectives()
    graph = torch.cuda.CUDAGraph()
    with capture_graph(graph):
        for k in range(G):
            stepper.step(acts[k % nbuf])
    graph.replay()                                           # untimed: warms the graph
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(K // G):
        graph.replay()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    del graph
    time_graph.last_event_ms = ev0.elapsed_time(ev1) / K     # device time per replayed step (this rank)
    return float(el.item()), G


def kernel_times(env, acts, n, stepper=None):
    """per-launch durations (ms) of the step kernel: start/stop events attached to its own
    dispatch (hipExtLaunchKernelGGL in libadrp) on the launching stream.  stepper: what drives the
    steps (the policy loop of a closed-loop bench), default env.step on the synthetic actions"""
    stepper = stepper or env
    torch.cuda.synchronize()
    env.h.profile_begin(n)
    for k in range(n):
        stepper.step(acts[k % acts.shape[0]])
    return np.asarray(env.h.profile_end(n))


def pmc_record(name, key):
    """a per-launch counter summary committed under profiles/ (tools/pmc_summary.py)"""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        rec = json.load(fh)
    return rec.get(key)


def pmc_record_any_envs(name, key):
    """the flop-model record of the same race workload (level, drones, physics) at any env count"""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        rec = json.load(fh)
    stem = "_".join(key.split("_")[:-2]) + "_"   # race_{level}_{drones}_{physics}_
    for k in sorted(rec):
        if k.startswith(stem) and k[len(stem):].count("_") == 1 and "algorithmic_flops_per_drone_step" in rec[k]:
            return rec[k]
    return None


def hover_make(precision, physics, dev, **kw):
    from gym_pybullet_adrp_amd.envs.hover import HoverAviary
    from gym_pybullet_adrp_amd.utils.enums import Physics
    return functools.partial(HoverAviary, physics=Physics[physics], device=dev, precision=precision, seed=2024,
                             initial_xyzs=[0, 0, 1.0], init_noise={"xyz": 0.1, "rpy": 0.05, "vel": 0.1, "omega": 0.1},
                             **kw)


def race_make(level, drones, physics, racemode, precision, dev):
    from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary
    from gym_pybullet_adrp_amd.utils.enums import Physics, RaceMode
    return functools.partial(MultiRaceAviary, level, num_drones=drones, physics=Physics[physics],
                             racemode=RaceMode[racemode], device=dev, precision=precision, seed=2024)


def hover_actions(E, dev, seed, nbuf=64):
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    return (torch.rand((nbuf, E, 1, 4), generator=gen, device=dev) * 2 - 1).contiguous()


def race_actions(obs0, dev, seed, nbuf=64):
    """FULLSTATE targets = start + U(+-0.3) m, z clipped to [0.2, 1.5], yaw 0"""
    E, N = obs0.shape[:2]
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    off = torch.rand((nbuf, E, N, 3), generator=gen, device=dev) * 0.6 - 0.3
    tgt = obs0[..., :3].unsqueeze(0) + off
    tgt[..., 2] = tgt[..., 2].clamp(0.2, 1.5)
    return torch.cat([tgt, torch.zeros((nbuf, E, N, 1), device=dev)], -1).contiguous()


def make_policy(spec, device):
    from gym_pybullet_adrp_amd.policy import ACTOR_KEYS, DevicePolicy
    mode = "absolute" if spec == "twogates" else "relative"     # RLControllerTwoGates / RLController
    if spec in ("example", "twogates"):
        g = np.load(os.path.join(ROOT, "tests", "golden", "policy_golden.npz"))
        name = "example_RL_model" if spec == "example" else "twogates"
        w = {k: g[f"{name}_w{i}"] for i, k in enumerate(ACTOR_KEYS)}
        return DevicePolicy(w, "relu" if bool(g[f"{name}_relu"]) else "tanh", device, mode)
    return DevicePolicy.from_zip(spec, device, mode)


def _kernel_time(step_ms, eager_ms):
    """per-launch kernel time: the timed region's HIP events / K (graph replay, one launch per
    step; what rocprofv3 of the same graph replays averages, plus the graph's inter-launch gaps),
    and the eager per-dispatch events beside it"""
    rec = {"kernel_us": step_ms * 1e3,
           "kernel_time": "HIP events around the timed region (graph replay) / K on the launching stream"}
    if eager_ms is not None and len(eager_ms):
        rec.update({"eager_dispatch_us": float(np.mean(eager_ms)) * 1e3,
                    "eager_dispatch_us_median": float(np.median(eager_ms)) * 1e3, "eager_launches": int(len(eager_ms))})
    return rec


def hbm_roofline(bytes_per_launch, step_ms, eager_ms, traffic_key):
    rec = _kernel_time(step_ms, eager_ms)
    ach = bytes_per_launch / (rec["kernel_us"] * 1e-6) / 1e9
    pmc = pmc_record("pmc_traffic.json", traffic_key)
    out = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
           "traffic": None if pmc is None else pmc["hbm_bytes_per_launch"],
           "traffic_source": None if pmc is None else f"profiles/pmc_traffic.json[{traffic_key}]",
           "bytes_per_launch": bytes_per_launch}
    out.update(rec)
    return out


def valu_roofline(env, step_ms, eager_ms, key, precision):
    """race kernel: flops per launch over the kernel time, vs the vector peak (fp64 kernel: the
    fp64 peak, although its firmware part is fp32 as in the reference).  Flop model: the PMC FLOPS
    counters of the one-lane fp32 kernel per drone-step (profiles/pmc_valu.json
    algorithmic_flops_per_drone_step; tools/pmc_summary.py valu mode): the same algorithm in either
    precision; the kernel's own counters (executed flops, redundant quad lanes included) and VALU
    busy beside it.  HBM fraction for information."""
    hbm = hbm_roofline(env.step_bytes(), step_ms, eager_ms, key)
    kt = _kernel_time(step_ms, eager_ms)
    avg_s = kt["kernel_us"] * 1e-6
    pmc = pmc_record("pmc_valu.json", key)
    peak = VALU_F32_PEAK_TFLOPS if precision == "fp32" else VALU_F64_PEAK_TFLOPS
    drones = env.num_envs * env.NUM_DRONES
    rec = {"bound": "valu", "achieved": None, "peak": peak, "unit": "TFLOP/s", "frac": None, "traffic": hbm["traffic"],
           "hbm": {"achieved_GBps": hbm["achieved"], "frac": hbm["frac"], "bytes_per_launch": hbm["bytes_per_launch"]}}
    rec.update(kt)
    alg = pmc_record("pmc_valu.json", key.replace("_fp64_", "_fp32_")) if pmc is None or "algorithmic_flops_per_drone_step" not in pmc else pmc
    if alg is None or "algorithmic_flops_per_drone_step" not in alg:
        # the flop model is per drone-step: the same workload at another env count carries it
        # (config 5 strong: 32,768 envs on one GPU)
        alg = pmc_record_any_envs("pmc_valu.json", key)
    if alg is not None and "algorithmic_flops_per_drone_step" in alg:
        per_drone = alg["algorithmic_flops_per_drone_step"]
        flops = per_drone * drones
        rec.update({"achieved": flops / avg_s / 1e12, "frac": flops / avg_s / 1e12 / peak,
                    "flops_per_launch": flops, "flops_per_drone_step": per_drone,
                    "source": f"profiles/pmc_valu.json[{key if pmc is alg else key.replace('_fp64_', '_fp32_')}]"
                              + ("" if pmc is alg or pmc_record("pmc_valu.json", key.replace("_fp64_", "_fp32_")) is alg
                                 else " (the same workload's flop model at another env count)")})
    if pmc is not None:
        exe = pmc["flops_per_launch"]
        rec.update({"executed_flops_per_launch": exe, "executed_frac": exe / avg_s / 1e12 / peak,
                    "valu_busy": pmc.get("valu_busy"), "executed_source": f"profiles/pmc_valu.json[{key}]"})
    return rec


def race_key(level, drones, physics, precision, E):
    return f"race_{level}_{drones}_{physics}_{precision}_{E}"


# ----------------------------------------------------------------------------------------------
# workloads
# ----------------------------------------------------------------------------------------------
def _gather_record(sharded, acts, K, W, world, dev, E_rank, row_floats, refuse_capture=False):
    """step + packed all-gather (sharding.ShardedAviary(packed=True).step_gather): env.step and one
    all_gather_into_tensor of the preallocated send buffer, captured together in the HIP graph;
    eager (one launch + one collective per step) if the capture is refused (refuse_capture: act as if
    it were, tests/test_sharding_gpu.py)"""

    class _SG:
        def step(self, a):
            return sharded.step_gather(a)
    rec = {"collective": "all_gather_into_tensor (RCCL) of the packed obs/reward/flags send buffer",
           "bytes_per_rank_per_step": sharded._seg, "obs_floats_per_env": row_floats}
    try:
        if refuse_capture:
            raise RuntimeError("capture refused (forced)")
        el, G = time_graph(_SG(), acts, K, W, world, dev)
        rec["timed_region"] = f"{K // G} replays of a {G}-step HIP graph (step kernel + RCCL all-gather per step)"
    except Exception as exc:   # capture of the collective refused: time it eagerly instead
        torch.cuda.synchronize()
        rec["graph_capture_error"] = repr(exc)[:300]
        for k in range(W):
            sharded.step_gather(acts[k % acts.shape[0]])
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for k in range(K):
            sharded.step_gather(acts[k % acts.shape[0]])
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        rec["timed_region"] = f"{K} eager steps (step kernel + RCCL all-gather each)"
    rec.update({"value": E_rank * world * K / el, "unit": "env-steps/s", "ms_per_step": el / K * 1e3, "steps": K})
    return rec


def gather_record_world1(dev, K, W, precision="fp64", E=ENVS_PER_GPU, refuse_capture=False, seed=4):
    """config 5's step + RCCL all-gather at N = 1: a world-1 "nccl" (RCCL) group (created here unless
    one is already initialised), ShardedAviary(packed=True) over the config-5 per-GPU workload,
    step_gather captured in the HIP graph (the path every rank of an N-GPU job runs)"""
    from gym_pybullet_adrp_amd.sharding import ShardedAviary
    own = not dist.is_initialized()
    if own:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", dev))
    sharded = None
    try:
        sharded = ShardedAviary(E, race_make("level3", 4, "PYB_DW", "COMPETE", precision, dev), packed=True)
        obs0, _ = sharded.env.reset()
        acts = race_actions(obs0.clone(), dev, seed)
        rec = _gather_record(sharded, acts, K, W, 1, dev, E, 4 * sharded.env.h.D, refuse_capture=refuse_capture)
        rec.update({"world": dist.get_world_size(), "backend": dist.get_backend(), "precision": precision,
                    "envs_per_gpu": E, "kernel": sharded.env.kernel_name})
        return rec
    finally:
        if sharded is not None:
            sharded.close()
        if own:
            dist.destroy_process_group()


def gather_leg_child(K, W, timeout_s=300):
    """config 5's world-1 RCCL step + all-gather leg in a FRESH child process (this script with
    --gather-leg): it brings up its own RCCL communicator and HIP graph, and whatever happens to it
    (an abort on a library thread cannot be caught in-process) the parent's record survives and
    says what the child returned.  The parent has synchronised its device work first."""
    torch.cuda.synchronize()
    cmd = [sys.executable, os.path.abspath(__file__), "--gather-leg", "--race-steps", str(K),
           "--gather-warmup", str(W)]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "GROUP_RANK", "ROLE_RANK"):
        env.pop(k, None)
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired as exc:
        return {"child": "timeout", "timeout_s": timeout_s,
                "stderr_tail": (exc.stderr or b"")[-1500:].decode(errors="replace") if isinstance(exc.stderr, bytes)
                else str(exc.stderr or "")[-1500:]}
    sys.stderr.write(p.stderr[-4000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"child": "failed", "rc": p.returncode, "stderr_tail": p.stderr[-1500:]}
    rec = json.loads(lines[-1])
    rec["child"] = {"rc": 0, "wall_s": round(time.perf_counter() - t0, 2),
                    "note": "run in a fresh child process (own RCCL communicator), merged here"}
    return rec


def guarded(fn, *a, **kw):
    """one sub-record: an exception in it is recorded in its place, the rest of the line survives"""
    try:
        return fn(*a, **kw)
    except Exception as exc:   # noqa: BLE001 - the record says what failed
        import traceback
        traceback.print_exc()
        torch.cuda.synchronize()
        return {"error": repr(exc)[:500]}


def bench_race(level, drones, physics, racemode, precision, E, K, W, world, rank, dev, seed,
               sharded_gather=False, policy_spec=None, graph_only=False, global_envs=None):
    """one MultiRaceAviary workload; E envs per GPU, or global_envs in total (strong scaling)"""
    from gym_pybullet_adrp_amd import _lib
    make = race_make(level, drones, physics, racemode, precision, dev)
    sharded = None
    if world > 1:
        from gym_pybullet_adrp_amd.sharding import ShardedAviary
        sharded = ShardedAviary(global_envs or E * world, make, packed=sharded_gather)
        env = sharded.env
    else:
        env = make(num_envs=global_envs or E, env_offset=0)
    E = env.num_envs
    obs0, _ = env.reset()
    acts = race_actions(obs0.clone(), dev, seed + rank)
    policy = None
    stepper = env
    if policy_spec:
        policy = make_policy(policy_spec, dev)
        pact = torch.empty((E, drones, 4), device=dev)

        class _Loop:   # one "step" = policy forward on the current obs + env.step on its setpoints
            def step(self, _a):
                policy.act(env._obs, out=pact)
                return env.step(pact)
        stepper = _Loop()
    elapsed, G = time_graph(stepper, acts, K, W, world, dev)
    step_ms = time_graph.last_event_ms
    # closed loop: the timed region holds the policy launch too, so the step kernel's own time comes
    # from its dispatch events on the actor-driven steps
    eager = None if graph_only else kernel_times(env, acts, min(K, 512), stepper)
    if policy is not None and eager is not None:
        step_ms = float(np.mean(eager))
    key = race_key(level, drones, physics, precision, E)
    total = E * world
    rec = {"workload": f"MultiRaceAviary {racemode} {level}, {drones} drones x {E} envs/GPU ({total} total), "
                       f"{physics}, 20 sub-steps + Mellinger 500 Hz, {precision}"
                       + (" (reference precision)" if precision == "fp64" else ""),
           "value": total * K / elapsed, "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W,
           "ms_per_step": elapsed / K * 1e3, "drone_steps_per_s": total * K / elapsed * drones,
           "envs_per_gpu": E, "global_envs": total, "kernel": env.kernel_name,
           "roofline": valu_roofline(env, step_ms, eager, key, precision),
           "timed_region": f"{K // G} replays of a {G}-step HIP graph"}
    if policy is not None:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
        for a, b in ev:
            a.record()
            policy.act(env._obs, out=pact)
            b.record()
        torch.cuda.synchronize()
        pol_us = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
        rows = E * drones
        flops = 2 * rows * (policy.in_dim * policy.h1 + policy.h1 * policy.h2 + policy.h2 * 4)
        rec["workload"] += f"; closed loop: on-device PPO actor ({policy_spec}) each step"
        rec["policy"] = {"weights": policy_spec, "arch": f"{policy.in_dim}-{policy.h1}-{policy.h2}-4",
                         "kernel_us": pol_us, "rows": rows, "flops": flops,
                         "mfma_f32": {"achieved_tflops": flops / pol_us / 1e6, "unit": "TFLOP/s"},
                         "note": "event pairs around each policy launch on the current stream"}
        policy.close()
    if sharded is not None:
        rec["world"] = dist.get_world_size()
        rec["backend"] = dist.get_backend()
        if sharded_gather:
            rec["with_obs_allgather"] = _gather_record(sharded, acts, K, W, world, dev, E, drones * env.h.D)
    env.close()
    return rec


def bench_hover(args, precision, E, K, W, world, rank, dev, sweep=False, sharded_gather=False):
    from gym_pybullet_adrp_amd import _lib
    make = hover_make(precision, args.physics, dev)
    sharded = None
    if world > 1:
        from gym_pybullet_adrp_amd.sharding import ShardedAviary
        sharded = ShardedAviary(E * world, make, packed=sharded_gather)   # rank r owns global envs [r*E, (r+1)*E)
        env = sharded.env
    else:
        env = make(num_envs=E, env_offset=0)
    env.reset()
    acts = hover_actions(E, dev, 1 + rank)
    elapsed, G = time_graph(env, acts, K, W, world, dev)
    step_ms = time_graph.last_event_ms
    eager = None if args.graph_only else kernel_times(env, acts, min(K, 512))
    rec = {"value": E * world * K / elapsed, "ms_per_step": elapsed / K * 1e3,
           "kernel": env.kernel_name,
           "roofline": hbm_roofline(env.step_bytes(), step_ms, eager, f"{args.physics}_{precision}_{E}"),
           "timing": {"timed_region": f"{K // G} replays of a {G}-step HIP graph (one fused launch per env.step)",
                      "replay_overhead_us_per_step": elapsed / K * 1e6 - step_ms * 1e3,
                      "note": "ms_per_step = host clock around the timed region / K; kernel_us = HIP events around "
                              "the replays / K; the difference is graph launch + final sync, amortised over K"}}
    if not args.graph_only:
        # eager (no graph) end-to-end rate, for reference
        torch.cuda.synchronize()
        ne = min(K, 1000)
        te0 = time.perf_counter()
        for k in range(ne):
            env.step(acts[k % acts.shape[0]])
        torch.cuda.synchronize()
        te = time.perf_counter() - te0
        rec["timing"]["eager"] = {"env_steps_per_s_per_gpu": E * ne / te, "ms_per_step": te / ne * 1e3}
    if sharded is not None and sharded_gather:
        rec["with_obs_allgather"] = _gather_record(sharded, acts, K, W, world, dev, E, env.h.D)
    if sweep:
        rec["roofline"]["sweep"] = roofline_sweep(make, [65536, 262144, 1048576])
    cfg = env.cfg.copy()
    env.close()
    return rec, cfg


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
        us = float(np.mean(kernel_times(env, a, launches))) * 1e3
        gbps = env.step_bytes() / (us * 1e-6) / 1e9
        out.append({"envs": n, "kernel_us": us, "env_steps_per_s": n / (us * 1e-6), "achieved_GBps": gbps,
                    "frac": gbps / HBM_PEAK_GBPS})
        env.close()
        del a
    return out


def bench_config1(args, dev, cpu_seconds, with_cpu):
    """BASELINE configs[0]: one HoverAviary env (E = 1, PYB, 240/30 Hz) stepped from Python like
    examples/pid.py: per-step latency on the GPU (synchronised each step, and graph-replayed)
    and the float64 oracle for one env on one host core."""
    make = hover_make(args.precision, "PYB", dev)
    env = make(num_envs=1, env_offset=0)
    env.reset()
    acts = hover_actions(1, dev, 3)
    for k in range(50):
        env.step(acts[k % acts.shape[0]])
    torch.cuda.synchronize()
    n = 500
    t0 = time.perf_counter()
    for k in range(n):
        env.step(acts[k % acts.shape[0]])
        torch.cuda.synchronize()
    sync_s = (time.perf_counter() - t0) / n
    elapsed, G = time_graph(env, acts, 1000, 10, 1, dev)
    kern = kernel_times(env, acts, 200)
    graph_kernel_us = time_graph.last_event_ms * 1e3
    rec = {"workload": f"HoverAviary 1 env x 1 drone, Physics.PYB 240/30 Hz (8 sub-steps), RPM actions, {args.precision}",
           "gpu_sync_per_step": {"value": 1 / sync_s, "unit": "env-steps/s", "us_per_step": sync_s * 1e6,
                                 "note": "Python env.step + torch.cuda.synchronize each step"},
           "gpu_graph": {"value": 1000 / elapsed, "unit": "env-steps/s", "us_per_step": elapsed / 1000 * 1e6},
           "kernel_us": graph_kernel_us, "eager_dispatch_us": float(np.mean(kern)) * 1e3}
    # the same loop without a launch per step: a resident step kernel polling a host-mapped mailbox
    # (HoverAviary.persistent, include/adrp.h adrp_persistent_*); numpy action in, numpy obs out,
    # the step finished when step() returns
    acts_np = acts.cpu().numpy()
    with env.persistent() as p:
        # warm-up (the first blocks of a fresh mailbox ran slower in tools/persist_probe.py)
        for k in range(3000):
            p.step(acts_np[k % acts_np.shape[0]])
        # three blocks, the median block's rate: single 0.05-s blocks vary by +-6 % on the shared host
        n_p, blocks = 5000, []
        for _ in range(3):
            t0 = time.perf_counter()
            for k in range(n_p):
                p.step(acts_np[k % acts_np.shape[0]])
            blocks.append((time.perf_counter() - t0) / n_p)
        ps = float(np.median(blocks))
    rec["gpu_persistent_sync_per_step"] = {
        "value": 1 / ps, "unit": "env-steps/s", "us_per_step": ps * 1e6, "steps": 3 * n_p, "warmup": 3000,
        "block_rates": [1 / b for b in blocks], "statistic": "median of three 5,000-step blocks",
        "note": "HoverAviary.persistent(): numpy action written to host-mapped memory, one resident step kernel "
                "(no launch per step), numpy obs / reward / flags read from host-mapped memory when step() returns"}
    if with_cpu:
        v, steps, dt = _oracle_leg(env.cfg, 1, _hover_acts, min(cpu_seconds, 3.0), 1)
        rec["cpu_oracle_1env"] = {"value": v, "unit": "env-steps/s", "cores": 1,
                                  "sample": f"1 env x {steps} env.steps, {dt:.1f} s"}
    env.close()
    return rec


def bench_sb3_loop(args, dev, E=ENVS_PER_GPU, K=200, W=20):
    """SB3's side of the boundary (examples/learn.py:53-57 make_vec_env + PPO.collect_rollouts):
    numpy actions in, numpy obs / rewards / dones / infos out, through vec_env.AviaryVecEnv, on
    the `value` workload.  packed = the adapter's default: one C call per step (adrp_vec_step: the
    kernels read the actions from and write the outputs into pinned host blocks, a ring of 3 whose
    views are returned), lazy infos; packed_copy = one packed device buffer, one async copy into
    pinned memory, one wait, fresh arrays (DummyVecEnv's copy semantics); legacy = per-tensor .cpu()
    copies and a dict per env."""
    from gym_pybullet_adrp_amd.vec_env import AviaryVecEnv
    make = hover_make(args.precision, args.physics, dev)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (16, E, 1, 4)).astype(np.float32)
    rec = {"workload": f"HoverAviary {E} envs ({args.precision}) stepped through the SB3 VecEnv protocol "
                       "(numpy actions in, numpy obs / rewards / dones / infos out, auto-reset infos)"}
    for name, kw in (("packed", {}), ("packed_copy", {"direct": False}), ("legacy", {"packed": False})):
        env = make(num_envs=E, env_offset=0)
        v = AviaryVecEnv(env, **kw)
        v.reset()
        for k in range(W):
            v.step(acts[k % 16])
        t0 = time.perf_counter()
        done = 0
        for k in range(K):
            _, _, d, _ = v.step(acts[k % 16])
            done += int(d.sum())
        dt = time.perf_counter() - t0
        rec[name] = {"value": E * K / dt, "unit": "env-steps/s", "us_per_step": dt / K * 1e6, "steps": K,
                     "done_envs": done}
        v.close()
    return rec


_T0 = time.perf_counter()


def progress(msg):
    """one stderr line per finished part (a long default run shows it is alive; stdout stays the one
    JSON line)"""
    print(f"[bench {time.perf_counter() - _T0:6.1f} s] {msg}", file=sys.stderr, flush=True)


def _stdout_to_stderr():
    """keep stdout for the ONE JSON line: libraries (RCCL prints its version banner when a
    communicator comes up) write to fd 1 directly, so fd 1 goes to stderr and the record is printed
    to a duplicate of the original stdout"""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    record_out = _stdout_to_stderr()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launch_check:
        return launch_check(args, world, rank, record_out)
    if torch.cuda.device_count() < world:
        sys.exit(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPUs")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(local)
    if args.gather_leg:
        W = args.gather_warmup if args.gather_warmup is not None else max(10, args.race_steps // 10)
        rec = gather_record_world1(local, args.race_steps, W)
        print(json.dumps(rec), file=record_out, flush=True)
        return
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world
    dev = local
    E, K, W = args.envs, args.steps, args.warmup
    RK, RW = args.race_steps, max(10, args.race_steps // 10)

    result = {"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W,
              "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
              "dtype": "f32" if args.precision == "fp32" else "f64"}
    hover_cfg = None
    if args.task == "race":
        rec = bench_race(args.level, args.drones, args.physics, args.racemode, args.precision, E, K, W, world, rank,
                         local, 2, sharded_gather=world > 1 and not args.no_allgather, policy_spec=args.policy)
        result.update({"value": rec.pop("value"), "ms_per_step": rec.pop("ms_per_step"),
                       "data": "synthetic: level preset resets (device Philox), FULLSTATE targets start + U(+-0.3) m"
                       if not args.policy else "synthetic: level preset resets; setpoints from the reference's PPO actor",
                       "config": {"workload": rec.pop("workload"), "envs_per_gpu": E, "global_envs": E * world,
                                  "drones_per_env": args.drones, "parallelism": f"env-sharded dp{world}"}})
        for k in ("steps", "warmup", "n_gpus", "unit"):
            rec.pop(k, None)
        result.update(rec)
    else:
        rec, hover_cfg = bench_hover(args, args.precision, E, K, W, world, rank, local,
                                     sweep=world == 1 and not args.no_sweep,
                                     sharded_gather=world > 1 and not args.no_allgather)
        result.update({"value": rec.pop("value"), "ms_per_step": rec.pop("ms_per_step"),
                       "data": "synthetic: device-RNG airborne initial states around (0,0,1), U[-1,1] RPM actions",
                       "config": {"workload": f"HoverAviary Physics.{args.physics} 240/30 Hz (8 sub-steps), {E} envs "
                                              f"x 1 drone per GPU, RPM actions, auto-reset", "envs_per_gpu": E,
                                  "global_envs": E * world, "drones_per_env": 1,
                                  "parallelism": f"env-sharded dp{world}"}})
        result.update(rec)
    progress("main line")

    if not args.no_configs and args.task == "hover":
        cf = {}
        gather = world > 1 and not args.no_allgather
        go = args.graph_only
        # config 5 at every N (at N = 1 it is BASELINE configs[3]): reference precision, then fp32;
        # `strong`: the 32,768 envs of config 5 in total over the N GPUs
        # at N > 1 every rank must run the same sequence of collectives, so a sub-record failure is
        # not contained there (guarded only at N = 1)
        run = guarded if world == 1 else (lambda fn, *a, **kw: fn(*a, **kw))
        cf["config5"] = run(bench_race, "level3", 4, "PYB_DW", "COMPETE", "fp64", 4096, RK, RW, world, rank, local, 4,
                            sharded_gather=gather, graph_only=go)
        progress("config5")
        cf["config5"]["strong"] = run(bench_race, "level3", 4, "PYB_DW", "COMPETE", "fp64", None, RK, RW, world, rank,
                                      local, 4, graph_only=go, global_envs=8 * 4096)
        progress("config5 strong")
        cf["config5_f32"] = run(bench_race, "level3", 4, "PYB_DW", "COMPETE", "fp32", 4096, RK, RW, world, rank, local,
                                4, sharded_gather=gather, graph_only=go)
        if world == 1:
            progress("config5_f32")
            cf["config4_gnd_drag_dw"] = run(bench_race, "level3", 4, "PYB_GND_DRAG_DW", "COMPETE", "fp64", 4096, RK, RW,
                                            1, 0, local, 4, graph_only=go)
            progress("config4_gnd_drag_dw")
            cf["config3"] = run(bench_race, "level0", 2, "PYB", "COMPARE", "fp64", 2048, RK, RW, 1, 0, local, 2,
                                graph_only=go)
            progress("config3")
            cf["config3_f32"] = run(bench_race, "level0", 2, "PYB", "COMPARE", "fp32", 2048, RK, RW, 1, 0, local, 2,
                                    graph_only=go)
            progress("config3_f32")
            cf["config3_policy"] = run(bench_race, "level0", 2, "PYB", "COMPARE", "fp64", 2048, RK, RW, 1, 0, local, 2,
                                       policy_spec="example", graph_only=go)
            progress("config3_policy")
            cf["config3_policy_f32"] = run(bench_race, "level0", 2, "PYB", "COMPARE", "fp32", 2048, RK, RW, 1, 0,
                                           local, 2, policy_spec="example", graph_only=go)
            progress("config3_policy_f32")
            other = "fp32" if args.precision == "fp64" else "fp64"

            def _other():
                r2, _ = bench_hover(args, other, E, min(K, 1000), min(W, 100), 1, 0, local)
                r2.update({"workload": f"the `value` workload with the {other} kernel", "unit": "env-steps/s",
                           "dtype": "f32" if other == "fp32" else "f64"})
                return r2
            cf[f"config2_{'f32' if other == 'fp32' else 'f64'}"] = run(_other)
            progress("config2 other precision")
            if not go:
                cf["config1"] = run(bench_config1, args, local, args.cpu_seconds, not args.no_cpu_baseline)
                progress("config1")
                cf["config2_sb3_vecenv"] = run(bench_sb3_loop, args, local)
                progress("config2_sb3_vecenv")
            if not args.no_allgather:
                # the RCCL step + all-gather path of an N-GPU job on a world-1 group, last and in a
                # child process: nothing it does can take the record with it
                cf["config5"]["with_obs_allgather"] = gather_leg_child(RK, RW)
                progress("config5 world-1 RCCL all-gather (child)")
        result["configs"] = cf

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.task == "race":
            result["cpu_baseline"] = cpu_baseline(race_cfg_of(args), args.cpu_seconds, race=True)
        else:
            result["cpu_baseline"] = cpu_baseline(hover_cfg, args.cpu_seconds)
            progress("cpu baseline")
            if "configs" in result:
                from gym_pybullet_adrp_amd.envs.race import race_config
                for name, lv, n, ph, md in (("config5", "level3", 4, "PYB_DW", "COMPETE"),
                                            ("config3", "level0", 2, "PYB", "COMPARE"),
                                            ("config4_gnd_drag_dw", "level3", 4, "PYB_GND_DRAG_DW", "COMPETE")):
                    c = race_config(lv, n, ph, md)
                    result["configs"][name]["cpu_baseline"] = cpu_baseline(c, args.cpu_seconds / 2, race=True)
                    progress(f"cpu baseline {name}")
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        result["summary"] = summary(result)   # last key: the compact per-config view stays in a kept tail
        print(json.dumps(result), file=record_out, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _sig(x, n=4):
    return None if x is None else float(f"{x:.{n}g}")


def summary(result):
    """per workload: value (env-steps/s), ms_per_step, dtype, kernel time (us) and roofline fraction"""
    def one(rec, dtype):
        if not rec or rec.get("value") is None:
            return None
        rf = rec.get("roofline") or {}
        return {"v": _sig(rec["value"]), "ms": _sig(rec.get("ms_per_step")), "dt": dtype,
                "k_us": _sig(rf.get("kernel_us")), "frac": _sig(rf.get("frac"), 3)}
    out = {"value": one(result, result.get("dtype"))}
    cf = result.get("configs") or {}
    for name, dt in (("config5", "f64"), ("config5_f32", "f32"), ("config4_gnd_drag_dw", "f64"), ("config3", "f64"),
                     ("config3_f32", "f32"), ("config3_policy", "f64"), ("config3_policy_f32", "f32"),
                     ("config2_f32", "f32"), ("config2_f64", "f64")):
        if name in cf:
            out[name] = one(cf[name], dt)
    c5 = cf.get("config5") or {}
    if "strong" in c5:
        out["config5_strong"] = one(c5["strong"], "f64")
    if "with_obs_allgather" in c5:
        g = c5["with_obs_allgather"]
        out["config5_allgather"] = {"v": _sig(g.get("value")), "ms": _sig(g.get("ms_per_step")), "dt": "f64",
                                    "graph": g.get("value") is not None and "graph_capture_error" not in g,
                                    "world": g.get("world"),
                                    "child": g["child"] if isinstance(g.get("child"), str) else "ok" if "child" in g
                                    else None}
    if "config1" in cf:
        c1 = cf["config1"]
        out["config1"] = {"persistent_sync_v": _sig((c1.get("gpu_persistent_sync_per_step") or {}).get("value")),
                          "launch_sync_v": _sig((c1.get("gpu_sync_per_step") or {}).get("value")),
                          "graph_v": _sig((c1.get("gpu_graph") or {}).get("value")),
                          "cpu_1core_v": _sig((c1.get("cpu_oracle_1env") or {}).get("value"))} if "error" not in c1 \
            else {"error": c1["error"]}
    if "config2_sb3_vecenv" in cf:
        out["sb3_packed_us"] = _sig(cf["config2_sb3_vecenv"]["packed"]["us_per_step"])
    if result.get("cpu_baseline"):
        out["cpu_baseline_v"] = _sig(result["cpu_baseline"]["value"])
    return out


def race_cfg_of(args):
    from gym_pybullet_adrp_amd.envs.race import race_config
    return race_config(args.level, args.drones, args.physics, args.racemode)


if __name__ == "__main__":
    main()
