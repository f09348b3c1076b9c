"""Race-track configurations in the reference's YAML schema (config/level*.yaml).

``load_race_config`` accepts a mapping with that schema (a dict or Munch, as
``utils.load_config`` returns), a path to such a YAML file, or one of the preset names
below.  ``fill_track`` writes it into the C-ABI ``adrp_config``.

The presets restate the values of the reference's level files.  Their gates, obstacles,
bounds, episode length and the two drone start states are identical across levels; the
levels differ only in which randomisations are enabled (README table in each file):
  getting_started  nothing randomised
  level0           drone start pos/rot
  level1           + drone mass/inertia, action noise and force disturbances
  level2, level3   + gate/obstacle offsets
Drones 2..7 have no start state in any reference file; the SURVEY §8(d) extension places
drone2 at (0.7, 0.9, 0.05) and drone3 at (1.3, 1.1, 0.05) (further drones on a 0.2 m grid).
"""
import copy
import os

_BASE = {
    "bounds": [[-3, -3, 0], [3, 3, 2]],
    "ctrl_freq": 25,
    "pyb_freq": 500,
    "episode_len_sec": 33,
    "init_states": {
        "drone0": {"pos": [0.9, 0.9, 0.05], "vel": [0, 0, 0], "rpy": [0, 0, 0], "pqr": [0, 0, 0]},
        "drone1": {"pos": [1.1, 1.1, 0.05], "vel": [0, 0, 0], "rpy": [0, 0, 0], "pqr": [0, 0, 0]},
    },
    "gates": [[0.45, -1.0, 0.525, 0, 0, 2.35, 1], [1.0, -1.55, 1.0, 0, 0, -0.78, 0],
              [0.0, 0.5, 0.525, 0, 0, 0, 1], [-0.5, -0.5, 1.0, 0, 0, 3.14, 0]],
    "obstacles": [[1.0, -0.5, 0.525, 0, 0, 0], [0.5, -1.5, 0.525, 0, 0, 0],
                  [-0.5, 0, 0.525, 0, 0, 0], [0, 1.0, 0.525, 0, 0, 0]],
    "random_drone_state": False,
    "random_drone_inertia": False,
    "random_gates_obstacles": False,
    "disturbances": False,
}
_STATE = {"pos": {"distrib": "uniform", "x": [-0.1, 0.1], "y": [-0.1, 0.1], "z": [0.0, 0.02]},
          "rot": {"distrib": "uniform", "r": [-0.1, 0.1], "p": [-0.1, 0.1], "y": [-0.1, 0.1]}}
_INERTIA = {"M": {"distrib": "uniform", "range": [-0.01, 0.01]},
            "Ixx": {"distrib": "uniform", "range": [-0.000001, 0.000001]},
            "Iyy": {"distrib": "uniform", "range": [-0.000001, 0.000001]},
            "Izz": {"distrib": "uniform", "range": [-0.000001, 0.000001]}}
_GATES = {"gates": {"distrib": "uniform", "range": [-0.15, 0.15]},
          "obstacles": {"distrib": "uniform", "range": [-0.15, 0.15]}}
_DIST = {"action": {"distrib": "normal", "std": 0.001},
         "dynamics": {"distrib": "uniform", "low": [-0.1, -0.1, -0.1], "high": [0.1, 0.1, 0.1]}}


def _preset(state=False, inertia=False, gates=False, dist=False):
    c = copy.deepcopy(_BASE)
    if state:
        c.update(random_drone_state=True, random_drone_state_info=copy.deepcopy(_STATE))
    if inertia:
        c.update(random_drone_inertia=True, random_drone_inertia_info=copy.deepcopy(_INERTIA))
    if gates:
        c.update(random_gates_obstacles=True, random_gates_obstacles_info=copy.deepcopy(_GATES))
    if dist:
        c.update(disturbances=True, disturbances_info=copy.deepcopy(_DIST))
    return c


PRESETS = {
    "getting_started": _preset(),
    "level0": _preset(state=True),
    "level1": _preset(state=True, inertia=True, dist=True),
    "level2": _preset(state=True, inertia=True, gates=True, dist=True),
    "level3": _preset(state=True, inertia=True, gates=True, dist=True),
}

EXTRA_DRONES = [[0.7, 0.9, 0.05], [1.3, 1.1, 0.05], [0.7, 1.1, 0.05], [1.3, 0.9, 0.05],
                [0.9, 0.7, 0.05], [1.1, 1.3, 0.05]]


def _get(m, k, default=None):
    if isinstance(m, dict):
        return m.get(k, default)
    return getattr(m, k, default)


def load_race_config(race_config):
    """mapping | YAML path | preset name -> plain dict (reference schema)"""
    if isinstance(race_config, str):
        if race_config in PRESETS:
            return copy.deepcopy(PRESETS[race_config])
        if os.path.exists(race_config):
            import yaml
            with open(race_config) as fh:
                return yaml.safe_load(fh)
        raise ValueError(f"unknown race config {race_config!r} (preset names: {sorted(PRESETS)})")
    return race_config


def fill_track(cfg, race_config, num_drones):
    """Write a reference-schema race config into adrp_config.track (+ freqs)."""
    rc = load_race_config(race_config)
    t = cfg.track
    gates = _get(rc, "gates", [])
    obst = _get(rc, "obstacles", [])
    if len(gates) > 4 or len(obst) > 4:
        raise ValueError("MultiRaceAviary observations hard-code 4 gates and 4 obstacles (MultiRaceAviary.py:591-651)")
    t.num_gates, t.num_obstacles = len(gates), len(obst)
    for g, row in enumerate(gates):
        for j in range(7):
            t.gates[g][j] = float(row[j])
    for k, row in enumerate(obst):
        for j in range(6):
            t.obstacles[k][j] = float(row[j])
    b = _get(rc, "bounds")
    for j in range(3):
        t.bounds_hi[j] = float(b[1][j])
    t.episode_len_sec = float(_get(rc, "episode_len_sec", 33))
    states = _get(rc, "init_states")
    names = list(states.keys()) if isinstance(states, dict) else list(vars(states).keys())
    for i in range(num_drones):
        if i < len(names):
            s = _get(states, names[i])
            pos, vel, rpy, pqr = _get(s, "pos"), _get(s, "vel", [0, 0, 0]), _get(s, "rpy", [0, 0, 0]), _get(s, "pqr", [0, 0, 0])
        else:
            pos, vel, rpy, pqr = EXTRA_DRONES[i - len(names)], [0, 0, 0], [0, 0, 0], [0, 0, 0]
        for j in range(3):
            t.init_pos[i][j] = float(pos[j]); t.init_vel[i][j] = float(vel[j])
            t.init_rpy[i][j] = float(rpy[j]); t.init_pqr[i][j] = float(pqr[j])
    t.random_drone_state = int(bool(_get(rc, "random_drone_state", False)))
    if t.random_drone_state:
        info = _get(rc, "random_drone_state_info")
        p, r = _get(info, "pos"), _get(info, "rot")
        for j, k in enumerate("xyz"):
            t.pos_offset_range[j][0], t.pos_offset_range[j][1] = map(float, _get(p, k))
        for j, k in enumerate("rpy"):
            t.rot_offset_range[j][0], t.rot_offset_range[j][1] = map(float, _get(r, k))
    t.random_drone_inertia = int(bool(_get(rc, "random_drone_inertia", False)))
    if t.random_drone_inertia:
        info = _get(rc, "random_drone_inertia_info")
        for j, k in enumerate(("M", "Ixx", "Iyy", "Izz")):
            t.inertia_offset_range[j][0], t.inertia_offset_range[j][1] = map(float, _get(_get(info, k), "range"))
    t.random_gates_obstacles = int(bool(_get(rc, "random_gates_obstacles", False)))
    if t.random_gates_obstacles:
        info = _get(rc, "random_gates_obstacles_info")
        t.gate_offset_range[0], t.gate_offset_range[1] = map(float, _get(_get(info, "gates"), "range"))
        t.obstacle_offset_range[0], t.obstacle_offset_range[1] = map(float, _get(_get(info, "obstacles"), "range"))
    t.disturbances = int(bool(_get(rc, "disturbances", False)))
    if t.disturbances:
        info = _get(rc, "disturbances_info")
        t.action_noise_std = float(_get(_get(info, "action"), "std"))
        dyn = _get(info, "dynamics")
        for j in range(3):
            t.dyn_dist_low[j] = float(_get(dyn, "low")[j])
            t.dyn_dist_high[j] = float(_get(dyn, "high")[j])
    return rc
