"""MultiRaceAviary CPU oracle (oracle/race.c): self-checks that need no GPU.

The Bullet step and the Crazyflie firmware are restated (parity unpinned);
these tests pin what can be pinned without them: the track/config plumbing against the
reference's level presets, the GJK geometry against brute force, the firmware LPF against
its closed form, the reset semantics of MultiRaceAviary.reset (initial obs at the nominal
pose), shard invariance of the Philox draws, and closed-loop behaviour of the Mellinger
loop (take-off to a FULLSTATE target converges; the pitch/roll sign conventions of the
firmware would make it diverge otherwise).
"""
import numpy as np
import pytest

from gym_pybullet_adrp_amd.envs.tracks import PRESETS, fill_track
from gym_pybullet_adrp_amd.utils import abi
from oracle import oracle as O


def race_cfg(level="level0", N=2, E=4, **kw):
    c = O.default_config(abi.TASK_RACE)
    c.num_drones = N
    fill_track(c, level, N)
    c.num_envs = E
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_level0_preset_is_the_default_config():
    a = O.default_config(abi.TASK_RACE)
    b = O.default_config(abi.TASK_RACE)
    fill_track(b, "level0", 2)
    assert bytes(a) == bytes(b)


def test_presets_follow_the_level_table():
    assert not PRESETS["getting_started"]["random_drone_state"]
    assert PRESETS["level0"]["random_drone_state"] and not PRESETS["level0"]["disturbances"]
    assert PRESETS["level1"]["random_drone_inertia"] and PRESETS["level1"]["disturbances"]
    assert not PRESETS["level1"]["random_gates_obstacles"]
    assert PRESETS["level3"]["random_gates_obstacles"]


def _box(c, R, h):
    return [0, *c, *np.asarray(R).ravel(), *h, 0]


def _cyl(c, R, r, hh):
    return [1, *c, *np.asarray(R).ravel(), 0, 0, hh, r]


def _rot(rpy):
    q = O.quat_from_euler(rpy)
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _samples(s, n, rng):
    """points filling a box / cylinder (for a brute-force upper bound of the distance)"""
    c, R = np.array(s[1:4]), np.array(s[4:13]).reshape(3, 3)
    if s[0] == 0:
        h = np.array(s[13:16])
        p = rng.uniform(-1, 1, (n, 3)) * h
        k = rng.integers(0, 3, n)
        p[np.arange(n), k] = np.sign(p[np.arange(n), k]) * h[k]      # on the surface
    else:
        r, hh = s[16], s[15]
        ang = rng.uniform(0, 2 * np.pi, n)
        rad = np.where(rng.random(n) < 0.5, r, r * np.sqrt(rng.random(n)))
        z = np.where(rad < r, np.sign(rng.uniform(-1, 1, n)) * hh, rng.uniform(-hh, hh, n))
        p = np.stack([rad * np.cos(ang), rad * np.sin(ang), z], 1)
    return c + p @ R.T


def test_gjk_distance_against_brute_force():
    rng = np.random.default_rng(0)
    for _ in range(60):
        a = _cyl(rng.uniform(-0.3, 0.3, 3), _rot(rng.uniform(-1, 1, 3)), 0.06, 0.0125)
        if rng.random() < 0.5:
            b = _box(rng.uniform(-0.3, 0.3, 3), _rot(rng.uniform(-1, 1, 3)), rng.uniform(0.02, 0.3, 3))
        else:
            b = _cyl(rng.uniform(-0.3, 0.3, 3), _rot(rng.uniform(-1, 1, 3)), rng.uniform(0.02, 0.1), rng.uniform(0.05, 0.4))
        d = O.shape_distance(a, b)
        assert d >= 0
        pa, pb = _samples(a, 3000, rng), _samples(b, 3000, rng)
        brute = np.min(np.linalg.norm(pa[:, None, :200] - pb[None, :, :200], axis=-1)) if False else None
        # upper bound from samples (GJK must not exceed it), exact for the sampled extremes
        sub_a, sub_b = pa[rng.choice(3000, 600)], pb[rng.choice(3000, 600)]
        ub = np.min(np.linalg.norm(sub_a[:, None, :] - sub_b[None, :, :], axis=-1))
        assert d <= ub + 1e-9
        if d > 0:   # and no sampled pair is closer than the distance (lower bound)
            assert ub >= d - 1e-9


def test_gjk_separating_distance_is_tight():
    """axis-aligned cases with a closed form"""
    I = np.eye(3)
    box = _box([0, 0, 0], I, [0.25, 0.025, 0.025])
    for z in (0.1, 0.5, 1.0):
        cyl = _cyl([0, 0, z], I, 0.06, 0.0125)
        assert abs(O.shape_distance(cyl, box) - (z - 0.025 - 0.0125)) < 1e-12
    cyl = _cyl([0.5, 0, 0], I, 0.06, 0.0125)
    assert abs(O.shape_distance(cyl, box) - (0.5 - 0.25 - 0.06)) < 1e-12
    cyl = _cyl([0.1, 0, 0], I, 0.06, 0.0125)
    assert O.shape_distance(cyl, box) == 0


def test_gjk_coplanar_discs():
    """two level drone cylinders at one height: the support points are coplanar (flat
    tetrahedra); the distance is the rim gap"""
    I = np.eye(3)
    for gap in (0.0035, 0.02, 0.1):
        a = _cyl([0.0, 0.0, 0.5], I, 0.06, 0.0125)
        b = _cyl([0.12 + gap, 0.0, 0.5], I, 0.06, 0.0125)
        assert abs(O.shape_distance(a, b) - gap) < 1e-9
        b = _cyl([(0.12 + gap) / np.sqrt(2), (0.12 + gap) / np.sqrt(2), 0.5], _rot([0, 0, 0.3]), 0.06, 0.0125)
        assert abs(O.shape_distance(a, b) - gap) < 1e-9
    assert O.shape_distance(_cyl([0, 0, 0.5], I, 0.06, 0.0125), _cyl([0.11, 0, 0.5], I, 0.06, 0.0125)) == 0


def test_gate_distance_geometry():
    c = race_cfg()
    ident = [0, 0, 0, 1]
    # drone centred in a tall gate opening: 0.14 m to the side posts (posts at +-0.2, r 0.06)
    assert abs(O.race_body_distance(c, [0, 0, 1], ident, 0, 0, [0, 0, 1, 0]) - 0.14) < 1e-3
    # overlapping a post
    assert O.race_body_distance(c, [0.3, 0, 1], ident, 0, 0, [0, 0, 1, 0]) == 0
    # low gate box under the opening, obstacle pole
    assert O.race_body_distance(c, [0, 0, 0.125], ident, 0, 1, [0, 0, 0.525, 0]) == 0
    d = O.race_body_distance(c, [0.5, 0, 0.5], ident, 1, 0, [0, 0, 0.525, 0])
    assert abs(d - (0.5 - 0.05 - 0.06)) < 1e-9


def test_lpf2p_coefficients():
    """firmware lpf2pSetCutoffFreq: Butterworth, unit DC gain (float32)"""
    for fs, fc in ((500, 30), (500, 80)):
        b0, b1, b2, a1, a2 = O.lpf_coeffs(fs, fc)
        assert abs((b0 + b1 + b2) / (1 + a1 + a2) - 1) < 1e-5
        ohm = np.tan(np.pi / (fs / fc))
        c = 1 + 2 * np.cos(np.pi / 4) * ohm + ohm * ohm
        assert abs(b0 - ohm * ohm / c) < 1e-6 and abs(a1 - 2 * (ohm * ohm - 1) / c) < 1e-6


def test_reset_obs_at_nominal_pose():
    """MultiRaceAviary.reset returns the obs computed before _drone_init moves the drones"""
    c = race_cfg("level0", N=2, E=8)
    o = O.Oracle(c)
    obs = o.reset()
    assert obs.shape == (8, 2, 49)
    np.testing.assert_allclose(obs[:, 0, :3], [[0.9, 0.9, 0.05]] * 8, atol=1e-7)
    np.testing.assert_allclose(obs[:, 1, :3], [[1.1, 1.1, 0.05]] * 8, atol=1e-7)
    assert (obs[..., 3:12] == 0).all() and (obs[..., 48] == 0).all()
    f, i = o.get_state()
    names, _ = o.field_names()
    pos = f[[names.index(n) for n in ("pos_x", "pos_y", "pos_z")]].T.reshape(8, 2, 3)
    off = pos - obs[..., :3]
    assert (np.abs(off[..., :2]) <= 0.1).all() and (off[..., 2] >= -1e-7).all() and (off[..., 2] <= 0.02).all()
    assert np.abs(off).max() > 1e-3                  # randomised (level0: random_drone_state)
    # nominal gates reported when out of range, actual = nominal at level0
    np.testing.assert_allclose(obs[0, 0, 12:16], [0.45, -1.0, 0.525, 2.35], atol=1e-6)


def test_shard_invariance_of_track_randomisation():
    """level3: gate offsets keyed by the global env id -> a shard equals the slice of a big run"""
    big = O.Oracle(race_cfg("level3", N=4, E=10, race_mode=abi.RACE_COMPETE))
    part = O.Oracle(race_cfg("level3", N=4, E=4, race_mode=abi.RACE_COMPETE, env_offset=6))
    ob, op = big.reset(), part.reset()
    np.testing.assert_array_equal(ob[6:], op)
    fb, _ = big.get_state()
    fp, _ = part.get_state()
    np.testing.assert_array_equal(fb[:, 24:], fp)


@pytest.mark.parametrize("physics", [abi.PHYS_PYB, abi.PHYS_PYB_GND, abi.PHYS_PYB_DRAG])
def test_mellinger_takeoff_converges(physics):
    """FULLSTATE target 0.5 m above the start: the closed loop climbs and settles (x, y
    within 2 cm of the target, z within 10 cm: the firmware's 0.027 kg / 9.81 model vs the
    PWM->thrust map leaves the known steady-state z offset), no elimination.  (Downwash is
    left out: between two drones at almost the same height its (PROP_RADIUS/4dz)^2 term blows
    up, in the reference too.  Physics.DYN is left out as well: its yaw torque has the
    opposite sign of the cf2x_IROS PYB model the Mellinger mixer is wired for
    (BaseAviary.py:700-703 vs 849), so its yaw loop diverges; see the next test.)"""
    E, N = 3, 2
    o = O.Oracle(race_cfg("level0", N=N, E=E, physics=physics, autoreset=0))
    obs = o.reset()
    act = np.zeros((E, N, 4), np.float32)
    act[..., :3] = obs[..., :3] + np.array([0, 0, 0.5])
    for _ in range(75):
        obs, _, te, tr, _ = o.step(act)
    assert not te.any() and not tr.any()
    np.testing.assert_allclose(obs[..., :2], act[..., :2], atol=0.02)
    assert (np.abs(obs[..., 2] - act[..., 2]) < 0.1).all()
    assert (np.abs(obs[..., 3:6]) < 0.05).all()


def test_elimination_out_of_bounds_and_termination():
    E, N = 2, 2
    o = O.Oracle(race_cfg("getting_started", N=N, E=E, autoreset=0))
    obs = o.reset()
    act = np.zeros((E, N, 4), np.float32)
    act[..., :3] = obs[..., :3] + np.array([0, 0, 0.5])
    act[0, :, 2] = 3.0            # env 0: both drones climb through the 2 m ceiling
    term_seen = False
    for _ in range(100):
        obs, _, te, tr, _ = o.step(act)
        if te[0]:
            term_seen = True
            break
    assert term_seen and not te[1]
    _, i = o.get_state()
    _, inames = o.field_names()
    flags = i[inames.index("flags")].reshape(E, N)
    assert (flags[0] & 1).all() and not (flags[1] & 1).any()


def test_dyn_yaw_loop_diverges_like_the_reference():
    """Physics.DYN + Mellinger: the reversed DYN yaw torque turns the yaw loop into positive
    feedback; the drones spin past |w| > 20 rad/s and are eliminated within ~6 env.steps"""
    E, N = 2, 2
    o = O.Oracle(race_cfg("level0", N=N, E=E, physics=abi.PHYS_DYN, autoreset=0))
    obs = o.reset()
    act = np.zeros((E, N, 4), np.float32)
    act[..., :3] = obs[..., :3] + np.array([0, 0, 0.5])
    for _ in range(10):
        obs, _, te, _, _ = o.step(act)
    assert te.all()
    assert (np.abs(obs[..., 11]) > 20).all()


def test_obs_wrapper_full_step():
    """The oracle's env.step with the DroneObservationWrapper fused: yaw actions are ignored (the
    trajectories equal a run with yaw 0 and no wrapper) and an env terminates (and auto-resets) once
    drone 0 has passed gate 2; mode 1 feeds that termination to the RewardWrapper's terminal terms."""
    from gym_pybullet_adrp_amd.envs.race import race_config
    E, N = 8, 2
    base = race_config("level0", N, "PYB", "COMPARE", num_envs=E, seed=5)
    base.autoreset = 0
    cw = base.copy()
    cw.track.obs_wrapper = 1
    a, b = O.Oracle(base), O.Oracle(cw)
    o0 = a.reset()
    b.reset()
    rng = np.random.default_rng(0)
    act = np.concatenate([o0[..., :3] + rng.uniform(-0.2, 0.2, (E, N, 3)), np.zeros((E, N, 1))], -1).astype(np.float32)
    act_yaw = act.copy()
    act_yaw[..., 3] = rng.uniform(-3, 3, (E, N))
    for _ in range(5):
        oa, _, ta, _, _ = a.step(act)
        ob, _, tb, _, _ = b.step(act_yaw)
        np.testing.assert_array_equal(oa, ob)
        np.testing.assert_array_equal(ta, tb)
    # drone 0 of envs 0..3 at gate 2 (the others at 1): early termination exactly there
    f, i = b.get_state()
    names, inames = b.field_names()
    g = i[inames.index("gate")].reshape(E, N)
    g[:, 0] = np.where(np.arange(E) < 4, 2, 1)
    g[:, 1] = 0
    i[inames.index("gate")] = g.ravel()
    b.set_state(f, i)
    _, _, tb, _, _ = b.step(act_yaw)
    np.testing.assert_array_equal(tb, np.arange(E) < 4)
