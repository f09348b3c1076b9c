"""Persistent-step costs (tools only): random actions vs one constant action copied every step vs
no copy, and the same with the action lines flushed from the CPU caches before the request."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd())
from gym_pybullet_adrp_amd.envs.hover import HoverAviary
res = {}
for trial in range(2):
    env = HoverAviary(num_envs=1, precision="fp64", seed=3); env.reset()
    anp = np.random.default_rng(0).uniform(-1, 1, (3, 1, 1, 4)).astype(np.float32)
    const = anp[0].copy()
    with env.persistent() as p:
        act = p.act
        def run(name, fn, n=20000):
            for k in range(2000): fn(k)
            t0 = time.perf_counter()
            for k in range(n): fn(k)
            res.setdefault(name, []).append(round(n / (time.perf_counter() - t0)))
        run("random_copy", lambda k: p.step(anp[k % 3]))
        run("const_copy", lambda k: p.step(const))
        run("no_copy", lambda k: p._step(p._h))
        run("random_copy_again", lambda k: p.step(anp[k % 3]))
    env.close()
print(json.dumps(res))
