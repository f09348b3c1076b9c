"""HoverAviary HIP kernel vs the CPU oracle (parity proper).  Needs an MI355X: -m gpu.

Tolerance (BASELINE.json north_star): teacher-forced per-step
|x_gpu - x_cpu| <= 1e-4 * max(|x_cpu|, floor) with floors pos/quat/vel/omega 1e-3,
RPM 1; fp32 kernel.  The fp64 kernel is held to 1e-9 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils import abi  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import ActionType, Physics  # noqa: E402
from oracle import oracle as O  # noqa: E402

PHYSICS = [Physics.PYB, Physics.DYN, Physics.PYB_GND, Physics.PYB_DRAG, Physics.PYB_DW, Physics.PYB_GND_DRAG_DW]
FLOORS = {"pos": 1e-3, "quat": 1e-3, "vel": 1e-3, "omega": 1e-3, "angv": 1e-3, "link_quat": 1e-3, "last_rpm": 1.0}


def pair(num_envs, physics=Physics.PYB, act=ActionType.RPM, precision="fp32", **kw):
    env = HoverAviary(physics=physics, act=act, num_envs=num_envs, precision=precision, **kw)
    cfg = env.cfg.copy()
    return env, O.Oracle(cfg)


def random_states(rng, E, env, oracle, z0=1.0, tilt=0.25, vel=0.5, omega=2.0):
    """Same random airborne state in both (values representable in float32)."""
    f, i = oracle.get_state()
    names, inames = oracle.field_names()
    idx = {n: k for k, n in enumerate(names)}
    pos = np.stack([rng.uniform(-0.5, 0.5, E), rng.uniform(-0.5, 0.5, E), z0 + rng.uniform(-0.3, 0.3, E)], 1)
    rpy = rng.uniform(-tilt, tilt, (E, 3)) * np.array([1, 1, 4])
    q = np.array([O.quat_from_euler(r) for r in rpy])
    v = rng.uniform(-vel, vel, (E, 3))
    w = rng.uniform(-omega, omega, (E, 3))
    lag = np.array([O.quat_from_euler(r + rng.uniform(-0.01, 0.01, 3)) for r in rpy])
    for k, ax in enumerate("xyz"):
        f[idx[f"pos_{ax}"]] = pos[:, k]; f[idx[f"vel_{ax}"]] = v[:, k]
        f[idx[f"omega_{ax}"]] = w[:, k]; f[idx[f"angv_{ax}"]] = w[:, k]
    for k, ax in enumerate("xyzw"):
        f[idx[f"quat_{ax}"]] = q[:, k]; f[idx[f"link_quat_{ax}"]] = lag[:, k]
    for k in range(4):
        f[idx[f"last_rpm_{k}"]] = rng.uniform(0.8, 1.2, E) * 16364.0
    ring_fields = [k for k, n in enumerate(names) if n.startswith("ring_")]
    f[ring_fields] = rng.uniform(-1, 1, (len(ring_fields), E))
    i[inames.index("step_counter")] = rng.integers(0, 200, E) * 8
    i[inames.index("ring_head")] = rng.integers(0, env.ACTION_BUFFER_SIZE, E)
    i[inames.index("episode")] = rng.integers(1, 5, E)
    real = np.float64 if env.cfg.precision else np.float32
    f = f.astype(real).astype(np.float64)      # identical start in both
    oracle.set_state(f, i)
    env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))
    return f, i


GROUPS = {"pos": ["pos_x", "pos_y", "pos_z"], "quat": ["quat_x", "quat_y", "quat_z", "quat_w"],
          "vel": ["vel_x", "vel_y", "vel_z"], "omega": ["omega_x", "omega_y", "omega_z"],
          "angv": ["angv_x", "angv_y", "angv_z"], "link_quat": ["link_quat_x", "link_quat_y", "link_quat_z", "link_quat_w"],
          "last_rpm": ["last_rpm_0", "last_rpm_1", "last_rpm_2", "last_rpm_3"]}


def compare_state(env, oracle, rtol, active):
    """Per-drone relative error of each state vector: |x_gpu - x_cpu| / max(|x_cpu|, floor)
    (2-norms over the vector's components), ring exact, ints exact."""
    fg, ig = env.get_state()
    fg, ig = fg.double().cpu().numpy(), ig.cpu().numpy()
    fo, io = oracle.get_state()
    names, inames = oracle.field_names()
    idx = {n: k for k, n in enumerate(names)}
    for k, n in enumerate(names):
        if n.startswith("ring_"):
            np.testing.assert_array_equal(fg[k], fo[k], err_msg=n)
    worst = {}
    for g in active:
        rows = [idx[n] for n in GROUPS[g]]
        d = np.linalg.norm(fg[rows] - fo[rows], axis=0)
        ref = np.maximum(np.linalg.norm(fo[rows], axis=0), FLOORS[g])
        err = d / ref
        worst[g] = float(err.max())
        assert err.max() <= rtol, f"{g}: max rel err {err.max():.3e} (env {err.argmax()})"
    np.testing.assert_array_equal(ig, io)
    return worst


def trunc_mismatches_at_threshold(tr_g, tr_o, final_o):
    """Truncation (HoverAviary.py:100-117: |x|, |y| > 1.5, z > 2, |roll|, |pitch| > 0.4) may differ
    only for an env whose oracle end state sits within the 1e-4 parity bar of one of these
    thresholds (relative to the threshold): a state inside the bar on the other side of a
    threshold flips the flag legitimately.  final_o: the oracle's obs row at the end of the step
    (the terminal obs of an env it reset).  Returns the number of such envs."""
    bad = np.flatnonzero(tr_g != tr_o)
    for e in bad:
        x = final_o[e, 0].astype(np.float64)
        margin = min(abs(abs(x[0]) - 1.5) / 1.5, abs(abs(x[1]) - 1.5) / 1.5, abs(x[2] - 2.0) / 2.0,
                     abs(abs(x[3]) - 0.4) / 0.4, abs(abs(x[4]) - 0.4) / 0.4)
        assert margin <= 1e-4, (f"env {e}: truncated gpu {tr_g[e]} cpu {tr_o[e]}, oracle pos {x[:3]} rpy {x[3:6]}: "
                                f"{margin:.2e} from the nearest threshold")
    return len(bad)


def active_fields(physics, lag=True):
    a = {"pos", "quat", "vel", "omega"}
    if physics == Physics.DYN:
        a |= {"angv"}
    elif lag:
        a |= {"link_quat"}
    if physics in (Physics.PYB_DRAG, Physics.PYB_GND_DRAG_DW):
        a |= {"last_rpm"}
    return a


@pytest.mark.parametrize("physics", PHYSICS)
def test_teacher_forced_step(physics):
    E = 4096
    rng = np.random.default_rng(100 + PHYSICS.index(physics))
    env, orc = pair(E, physics, autoreset=False)
    random_states(rng, E, env, orc)
    for t in range(3):
        act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
        obs_o, rew_o, te_o, tr_o, _ = orc.step(act)
        obs_g, rew_g, te_g, tr_g, _ = env.step(torch.from_numpy(act))
        torch.cuda.synchronize()
        compare_state(env, orc, 1e-4, active_fields(physics))
        og = obs_g.cpu().numpy()
        np.testing.assert_allclose(og[..., 12:], obs_o[..., 12:], rtol=0, atol=0)   # action ring: exact
        for sl in (slice(0, 3), slice(3, 6), slice(6, 9), slice(9, 12)):   # pos, rpy, vel, ang_v
            d = np.linalg.norm(og[:, 0, sl] - obs_o[:, 0, sl], axis=1)
            assert (d / np.maximum(np.linalg.norm(obs_o[:, 0, sl], axis=1), 1e-3)).max() <= 1e-4
        np.testing.assert_allclose(rew_g.cpu().numpy(), rew_o, rtol=1e-4, atol=1e-5)
        assert (te_g.cpu().numpy() == te_o).all()
        trunc_mismatches_at_threshold(tr_g.cpu().numpy(), tr_o, obs_o)
        # re-sync (teacher forcing): oracle state -> GPU
        f, i = orc.get_state()
        real = np.float64 if env.cfg.precision else np.float32
        env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))
        orc.set_state(f.astype(real).astype(np.float64), i)


@pytest.mark.parametrize("physics", [Physics.PYB, Physics.DYN, Physics.PYB_GND_DRAG_DW])
def test_fp64_kernel_tight(physics):
    """the float64 kernel: states within 1e-9, and reward / terminated / truncated exactly (the flags
    are threshold tests on a state that agrees to 1e-9; none of the sampled states sits that close)"""
    E = 512
    rng = np.random.default_rng(7)
    env, orc = pair(E, physics, precision="fp64", autoreset=False)
    random_states(rng, E, env, orc)
    for t in range(5):
        act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
        _, rew_o, te_o, tr_o, _ = orc.step(act)
        _, rew_g, te_g, tr_g, _ = env.step(torch.from_numpy(act))
        torch.cuda.synchronize()
        compare_state(env, orc, 1e-9, active_fields(physics))
        np.testing.assert_array_equal(te_g.cpu().numpy(), te_o)
        np.testing.assert_array_equal(tr_g.cpu().numpy(), tr_o)
        np.testing.assert_allclose(rew_g.cpu().numpy(), rew_o, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("precision,rtol", [("fp32", 1e-4), ("fp64", 1e-9)])
def test_benched_kernel_teacher_forced(precision, rtol):
    """the instantiations bench.py times (BASELINE config 2): hover_step<f64,PYB,A4,B15,cf2x> (`value`,
    the reference's precision) and its f32 twin, with auto-reset and the helper wave, E = 4096,
    teacher-forced per env.step against the oracle: the whole state within 1e-9 (fp64) / 1e-4 (fp32)
    relative, counters / ring exact; terminated exact, truncation only at a threshold within the bar.
    Envs that end their episode are reset in the same launch on both sides: their reset obs (a Philox
    draw) and terminal obs are compared too.  Obs rows are float32 in both: the fp64 kernel's rows
    are held to one float32 rounding (2.5e-7 relative)."""
    import os
    assert os.environ.get("ADRP_RESET_HELPER", "1") != "0"
    E = 4096
    rng = np.random.default_rng(31)
    noise = {"xyz": [0.1, 0.1, 0.1], "rpy": 0.05, "vel": 0.1, "omega": 0.1}
    env, orc = pair(E, Physics.PYB, precision=precision, seed=2024, initial_xyzs=[0, 0, 1.0], init_noise=noise)
    want = f"hover_step<{'f64' if precision == 'fp64' else 'f32'},PYB,A4,B15,cf2x>"
    assert _lib.kernel_name(env.cfg) == want and env.kernel_name == want and env.cfg.autoreset == 1
    real = np.float64 if precision == "fp64" else np.float32
    orow = 2.5e-7 if precision == "fp64" else 1e-4          # obs rows (float32)
    env.reset()
    orc.reset()
    random_states(rng, E, env, orc, tilt=0.3)
    resets = 0
    for t in range(6):
        act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
        obs_o, rew_o, te_o, tr_o, tobs_o = orc.step(act)
        obs_g, rew_g, te_g, tr_g, info = env.step(torch.from_numpy(act))
        torch.cuda.synchronize()
        og = obs_g.cpu().numpy()
        np.testing.assert_array_equal(te_g.cpu().numpy(), te_o)
        done = te_o | tr_o
        final_o = np.where(tr_o[:, None, None], tobs_o, obs_o)
        trunc_mismatches_at_threshold(tr_g.cpu().numpy(), tr_o, final_o)
        same = ~done & (tr_g.cpu().numpy() == tr_o)
        for sl in (slice(0, 3), slice(3, 6), slice(6, 9), slice(9, 12)):
            d = np.linalg.norm(og[same, 0, sl] - obs_o[same, 0, sl], axis=1)
            assert (d / np.maximum(np.linalg.norm(obs_o[same, 0, sl], axis=1), 1e-3)).max() <= orow
        np.testing.assert_array_equal(og[..., 12:], obs_o[..., 12:])             # action ring
        both = done & (tr_g.cpu().numpy() == tr_o)
        resets += int(both.sum())
        np.testing.assert_allclose(og[both], obs_o[both], rtol=min(orow, 1e-6), atol=1e-6)   # reset obs (Philox)
        tg = info["terminal_observation"].cpu().numpy()
        np.testing.assert_allclose(tg[both, :, :12], tobs_o[both, :, :12], rtol=orow, atol=orow)
        np.testing.assert_allclose(rew_g.cpu().numpy()[same], rew_o[same], rtol=max(rtol, 1e-6), atol=1e-5)
        # the whole state (incl. the next episode's of the reset envs) at the bar, ints exact
        agree = tr_g.cpu().numpy() == tr_o
        fg, ig = env.get_state()
        fg, ig = fg.double().cpu().numpy(), ig.cpu().numpy()
        fo, io = orc.get_state()
        names, _ = orc.field_names()
        idx = {n: k for k, n in enumerate(names)}
        for g in active_fields(Physics.PYB):
            rows = [idx[n] for n in GROUPS[g]]
            err = np.linalg.norm(fg[rows] - fo[rows], axis=0) / np.maximum(np.linalg.norm(fo[rows], axis=0), FLOORS[g])
            assert err[agree].max() <= rtol, f"step {t} {g}: {err[agree].max():.3e}"
        np.testing.assert_array_equal(ig[:, agree], io[:, agree])
        f, i = orc.get_state()
        env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))
        orc.set_state(f.astype(real).astype(np.float64), i)
    assert resets > 0


@pytest.mark.parametrize("precision,rtol", [("fp32", 1e-4), ("fp64", 1e-9)])
def test_single_env(precision, rtol):
    """BASELINE configs[0]: one HoverAviary env (E = 1, a 64-lane block with one live lane),
    free-running 100 env.steps from the reference default start against the oracle"""
    env, orc = pair(1, Physics.PYB, precision=precision, autoreset=False)
    o_g, _ = env.reset()
    o_o = orc.reset()
    np.testing.assert_allclose(o_g.cpu().numpy(), o_o, atol=1e-6)
    rng = np.random.default_rng(12)
    for t in range(100):
        act = rng.uniform(-0.2, 0.6, (1, 1, 4)).astype(np.float32)
        obs_o, rew_o, te_o, tr_o, _ = orc.step(act)
        obs_g, rew_g, te_g, tr_g, _ = env.step(torch.from_numpy(act))
        if t % 10 == 0:
            compare_state(env, orc, rtol, active_fields(Physics.PYB))
        f, i = orc.get_state()
        real = np.float64 if precision == "fp64" else np.float32
        env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))
        orc.set_state(f.astype(real).astype(np.float64), i)
        assert bool(te_g[0]) == bool(te_o[0]) and bool(tr_g[0]) == bool(tr_o[0])


def test_free_running_and_autoreset():
    """50 free-running steps from the reference default start, fixed seeds, with
    auto-reset: trajectories stay within tolerance, resets (RNG draws) agree."""
    E = 2048
    noise = {"xyz": [0.1, 0.1, 0.1], "rpy": 0.05, "vel": 0.1, "omega": 0.1}
    env, orc = pair(E, Physics.PYB, seed=1234, initial_xyzs=[0, 0, 1.0], init_noise=noise)
    o_g, _ = env.reset()
    o_o = orc.reset()
    np.testing.assert_allclose(o_g.cpu().numpy(), o_o, rtol=1e-6, atol=1e-6)
    rng = np.random.default_rng(1)
    resets = 0
    for t in range(60):
        act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
        obs_o, rew_o, te_o, tr_o, tobs_o = orc.step(act)
        obs_g, rew_g, te_g, tr_g, info = env.step(torch.from_numpy(act))
        done_o = te_o | tr_o
        done_g = (te_g | tr_g).cpu().numpy()
        resets += done_o.sum()
        # free-running fp32 vs fp64: chaotic divergence is bounded over this horizon
        same = done_o == done_g
        assert same.mean() > 0.99
        ok = same & ~done_o
        np.testing.assert_allclose(obs_g.cpu().numpy()[ok, :, :12], obs_o[ok, :, :12], rtol=5e-3, atol=5e-3)
        both = same & done_o
        np.testing.assert_allclose(obs_g.cpu().numpy()[both], obs_o[both], rtol=1e-5, atol=1e-5)  # reset obs
        np.testing.assert_allclose(info["terminal_observation"].cpu().numpy()[both, :, 12:],
                                   tobs_o[both, :, 12:])
    assert resets > 0


def test_one_d_rpm():
    E = 1024
    rng = np.random.default_rng(3)
    env, orc = pair(E, Physics.PYB, act=ActionType.ONE_D_RPM, autoreset=False)
    assert env.h.D == 27 and env.h.A == 1
    random_states(rng, E, env, orc)
    act = rng.uniform(-1, 1, (E, 1, 1)).astype(np.float32)
    obs_o, *_ = orc.step(act)
    obs_g, *_ = env.step(torch.from_numpy(act))
    torch.cuda.synchronize()
    compare_state(env, orc, 1e-4, active_fields(Physics.PYB))
    np.testing.assert_array_equal(obs_g.cpu().numpy()[..., 12:], obs_o[..., 12:])


def test_ground_contact_model():
    """Drones resting on / dropped onto the plane: both sides apply the same documented
    contact model.  The model is a projection, discontinuous in
    whether a sub-step touches, so contact steps are held to the model's resolution (one
    sub-step of gravity in v, the projection depth in z) rather than the 1e-4 airborne bar."""
    E = 256
    env, orc = pair(E, Physics.PYB, autoreset=False)   # default start z = 0.1125
    env.reset(); orc.reset()
    act = -np.ones((E, 1, 4), np.float32)              # 0.95 HOVER_RPM: sinks, then rests
    env.h.set_diagnostics(True)
    env.h.contact_count(reset=True)
    touched = 0
    for t in range(40):
        orc.step(act)
        env.step(torch.from_numpy(act))
        touched += orc.contact_count()
    torch.cuda.synchronize()
    assert touched > 0 and env.h.contact_count() > 0
    fg = env.get_state()[0].double().cpu().numpy()
    fo, _ = orc.get_state()
    g_dt = 9.8 / 240
    assert np.abs(fg[0:3] - fo[0:3]).max() < 1e-4            # pos [m]
    assert np.abs(fg[3:7] - fo[3:7]).max() < 1e-4            # quat
    assert np.abs(fg[7:10] - fo[7:10]).max() <= 1.01 * g_dt   # vel [m/s]
    assert np.abs(fg[10:13] - fo[10:13]).max() < 1e-4         # omega [rad/s]


def test_full_size_properties():
    """BASELINE config 2 size and beyond: 2^20 envs, invariants that need no oracle
    (finite state, unit quaternions, identical envs stay identical, ring exact), and a
    random subset re-checked against the oracle."""
    E = 1 << 20
    env = HoverAviary(precision="fp32", num_envs=E, autoreset=False, initial_xyzs=[0, 0, 1.0])
    obs, _ = env.reset()
    a = torch.zeros((E, 1, 4), device=env.device)
    a[:, 0, 0] = 0.3
    for _ in range(5):
        obs, rew, te, tr, _ = env.step(a)
    f, i = env.get_state()
    assert torch.isfinite(f).all()
    qn = (f[3:7] ** 2).sum(0).sqrt()
    assert (qn - 1).abs().max() < 1e-5
    assert (obs[:, 0, :12] == obs[0:1, 0, :12]).all()        # identical inputs, identical lanes
    assert (obs[:, 0, -4:] == a[:, 0, :]).all()              # newest ring entry = this action
    # subset vs oracle from the same start
    rng = np.random.default_rng(0)
    sub = np.sort(rng.choice(E, 256, replace=False))
    cfg = env.cfg.copy(); cfg.num_envs = len(sub)
    orc = O.Oracle(cfg)
    fs, is_ = f[:, sub].double().cpu().numpy(), i[:, sub].cpu().numpy()
    orc.set_state(fs, is_)
    act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
    env.step(torch.from_numpy(act))
    orc.step(act[sub])
    fg = env.get_state()[0][:, sub].double().cpu().numpy()
    fo, _ = orc.get_state()
    np.testing.assert_allclose(fg[:13], fo[:13], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("ctrl_freq", [240, 60])
def test_generic_ring_length(ctrl_freq):
    """ctrl_freq != 30: ring length ctrl_freq // 2 != 15 and S = 240 / ctrl_freq -> the
    generic (runtime ring length, device-constant) kernel"""
    E = 128
    env, orc = pair(E, ctrl_freq=ctrl_freq, autoreset=False, seed=3, initial_xyzs=[0, 0, 1.0],
                    init_noise={"xyz": 0.1, "rpy": 0.1, "vel": 0.2, "omega": 0.5})
    obs_g, _ = env.reset()
    obs_o = orc.reset()
    np.testing.assert_allclose(obs_g.cpu().numpy(), obs_o, atol=1e-6)
    rng = np.random.default_rng(4)
    B = ctrl_freq // 2
    for k in range(B + 3):          # past the ring wrap-around
        act = rng.uniform(-1, 1, (E, 1, 4)).astype(np.float32)
        obs_o, rew_o, te_o, tr_o, _ = orc.step(act)
        obs_g, rew_g, te_g, tr_g, _ = env.step(torch.from_numpy(act).to(env.device))
        torch.cuda.synchronize()
        if k % 10 == 0 or k >= B - 2:
            compare_state(env, orc, 1e-4, active_fields(Physics.PYB))
        np.testing.assert_array_equal(obs_g.cpu().numpy()[..., 12:], obs_o[..., 12:])
        f, i = orc.get_state()
        f = f.astype(np.float32).astype(np.float64)
        orc.set_state(f, i)
        env.set_state(torch.from_numpy(f.astype(np.float32)), torch.from_numpy(i))
    env.close()


PID_GROUPS = {"pid_last_rpy": ["pid_last_rpy_x", "pid_last_rpy_y", "pid_last_rpy_z"],
              "pid_int_pos": ["pid_int_pos_x", "pid_int_pos_y", "pid_int_pos_z"],
              "pid_int_rpy": ["pid_int_rpy_x", "pid_int_rpy_y", "pid_int_rpy_z"]}
GROUPS.update(PID_GROUPS)
FLOORS.update({"pid_last_rpy": 1e-3, "pid_int_pos": 1e-3, "pid_int_rpy": 1e-3})
PID_ACTS = {ActionType.PID: 3, ActionType.VEL: 4, ActionType.ONE_D_PID: 1}


def random_pid_state(rng, env, orc):
    """random_states + a DSLPIDControl state (last_rpy near the pose, integrators inside and
    on their clips) in both."""
    f, i = random_states(rng, env.num_envs, env, orc, tilt=0.15, omega=1.0)
    names, _ = orc.field_names()
    idx = {n: k for k, n in enumerate(names)}
    E = env.num_envs
    rpy = np.array([O.euler_from_quat(f[[idx[f"quat_{a}"] for a in "xyzw"], e]) for e in range(E)])
    for k, ax in enumerate("xyz"):
        f[idx[f"pid_last_rpy_{ax}"]] = rpy[:, k] + rng.uniform(-0.02, 0.02, E)
        f[idx[f"pid_int_pos_{ax}"]] = np.clip(rng.uniform(-2.5, 2.5, E), -2, 2) * (0.075 if ax == "z" else 1)
        f[idx[f"pid_int_rpy_{ax}"]] = rng.uniform(-1, 1, E) * (1 if ax != "z" else 20)
    real = np.float64 if env.cfg.precision else np.float32
    f = f.astype(real).astype(np.float64)
    orc.set_state(f, i)
    env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))


def pid_actions(rng, act, E, obs):
    if act == ActionType.PID:    # waypoints, half of them more than 1 m away (capped step)
        return np.clip(obs[:, :, :3] + rng.uniform(-1.5, 1.5, (E, 1, 3)), -2, 2).astype(np.float32)
    a = rng.uniform(-1, 1, (E, 1, PID_ACTS[act])).astype(np.float32)
    if act == ActionType.VEL:
        a[::9, :, :3] = 0        # zero direction -> zero target velocity
    return a


@pytest.mark.parametrize("precision,rtol", [("fp32", 1e-4), ("fp64", 1e-9)])
@pytest.mark.parametrize("physics", [Physics.PYB_GND_DRAG_DW, Physics.DYN])
@pytest.mark.parametrize("act", list(PID_ACTS))
def test_pid_action_types(act, physics, precision, rtol):
    """HoverAviary PID / VEL / ONE_D_PID (BaseRLAviary.py:193-235): the fused DSLPIDControl
    (control/DSLPIDControl.py:82-259) + sub-steps, teacher-forced per env.step against the
    oracle (itself pinned to the reference by tests/golden/pid_golden.npz).  Controller
    state, RPMs (last_rpm, PYB_GND_DRAG_DW) and the 3- / 4- / 1-wide action ring included."""
    E = 2048 if precision == "fp32" else 256
    rng = np.random.default_rng(500 + list(PID_ACTS).index(act))
    env, orc = pair(E, physics, act=act, precision=precision, autoreset=False)
    assert env.h.A == PID_ACTS[act] and env.h.D == 12 + 15 * PID_ACTS[act]
    assert _lib.kernel_name(env.cfg).endswith({ActionType.PID: "PID>", ActionType.VEL: "VEL>",
                                         ActionType.ONE_D_PID: "ONE_D_PID>"}[act])
    random_pid_state(rng, env, orc)
    active = active_fields(physics) | set(PID_GROUPS)
    obs = orc.hover_eval()[0]
    for t in range(4):
        a = pid_actions(rng, act, E, obs)
        obs, rew_o, te_o, tr_o, _ = orc.step(a)
        obs_g, rew_g, te_g, tr_g, _ = env.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        compare_state(env, orc, rtol, active)
        og = obs_g.cpu().numpy()
        np.testing.assert_array_equal(og[..., 12:], obs[..., 12:])
        np.testing.assert_allclose(rew_g.cpu().numpy(), rew_o, rtol=max(rtol, 1e-6), atol=1e-5)
        f, i = orc.get_state()
        real = np.float64 if env.cfg.precision else np.float32
        env.set_state(torch.from_numpy(f.astype(real)), torch.from_numpy(i))
        orc.set_state(f.astype(real).astype(np.float64), i)
    env.close()


def test_pid_controller_persists_across_resets():
    """The reference builds the DSLPIDControl objects once (BaseRLAviary.py:73-78) and never
    resets them: a masked reset keeps the controller state, as the oracle does."""
    E = 256
    env, orc = pair(E, Physics.PYB, act=ActionType.ONE_D_PID, autoreset=False, initial_xyzs=[0, 0, 1.0])
    env.reset(); orc.reset()
    a = np.full((E, 1, 1), 0.5, np.float32)
    for _ in range(3):
        env.step(torch.from_numpy(a)); orc.step(a)
    names, _ = orc.field_names()
    pid = [k for k, n in enumerate(names) if n.startswith("pid_")]
    f, i = orc.get_state()                    # teacher-force: identical state, then reset half
    env.set_state(torch.from_numpy(f.astype(np.float32)), torch.from_numpy(i))
    orc.set_state(f.astype(np.float32).astype(np.float64), i)
    before = env.get_state()[0][pid].clone()
    mask = np.zeros(E, np.uint8); mask[::2] = 1
    env.reset(mask=torch.from_numpy(mask)); orc.reset(mask)
    torch.cuda.synchronize()
    assert torch.equal(env.get_state()[0][pid], before)
    assert before.abs().sum() > 0
    compare_state(env, orc, 1e-4, {"pos", "quat", "vel", "omega"} | set(PID_GROUPS))


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("E", [4096, 640])
def test_reset_helper_same_results(monkeypatch, E, precision):
    """the staged kernel's helper wave (next-episode states, action ring, half the copy-out)
    changes who computes, not what: 40 auto-reset env.steps with and without it
    (ADRP_RESET_HELPER=0) and on the row-store kernel (ADRP_STAGE_ROWS=0) give bit-identical done
    flags, obs, terminal obs and reward (the hover TUs contract a*b+c only within one source
    expression, csrc/Makefile CONTRACT), in both precisions"""
    noise = {"xyz": [0.1, 0.1, 0.1], "rpy": 0.35, "vel": 0.1, "omega": 0.1}
    rng = np.random.default_rng(8)
    acts = torch.from_numpy(rng.uniform(-1, 1, (40, E, 1, 4)).astype(np.float32))
    runs = []
    for helper, stage in (("1", "1"), ("0", "1"), ("1", "0")):
        monkeypatch.setenv("ADRP_RESET_HELPER", helper)
        monkeypatch.setenv("ADRP_STAGE_ROWS", stage)
        env = HoverAviary(physics=Physics.PYB, precision=precision, num_envs=E, seed=99, initial_xyzs=[0, 0, 1.0], init_noise=noise)
        env.reset()
        seq = []
        for t in range(40):
            obs, rew, te, tr, info = env.step(acts[t].to(env.device))
            seq.append((obs.reshape(E, -1).cpu().numpy().copy(), info["terminal_observation"].reshape(E, -1).cpu().numpy().copy(),
                        rew.reshape(E).cpu().numpy().copy(), (te | tr).reshape(E).cpu().numpy().copy()))
        runs.append(seq)
        env.close()
    resets = 0
    for other in runs[1:]:
        for (o1, t1, r1, d1), (o0, t0, r0, d0) in zip(runs[0], other):
            np.testing.assert_array_equal(d1, d0)
            resets += int(d1.sum())
            np.testing.assert_array_equal(o1, o0)
            np.testing.assert_array_equal(t1[d1], t0[d1])
            np.testing.assert_array_equal(r1, r0)
    assert resets > 0


def test_fp64_batch_invariance():
    """the fp64 hover kernel's short forms (exp-map series, Newton-from-1 norm) are chosen
    per lane, so an env's trajectory does not depend on which envs share its wave.  The same 255 states
    stepped (a) in order, (b) shifted by one env (every wave holds different neighbours) and (c) with
    wave neighbours tumbling at 30 / 150 rad/s (the full series) and at 250 rad/s (the coordinate
    velocity clamp) give bit-identical states for every common env over 4 env.steps."""
    E = 256
    rng = np.random.default_rng(77)
    env, orc = pair(E, Physics.PYB, precision="fp64", autoreset=False)
    f, i = random_states(rng, E, env, orc, omega=3.0)
    names, _ = env.state_field_names()
    acts = rng.uniform(-1, 1, (4, E, 1, 4)).astype(np.float32)

    def run(fs, iis, a):
        env.set_state(torch.from_numpy(fs), torch.from_numpy(iis))
        for k in range(4):
            env.step(torch.from_numpy(a[k]))
        return env.get_state()[0].cpu().numpy()

    base = run(f.copy(), i.copy(), acts)
    sh_f, sh_i, sh_a = np.roll(f, 1, axis=1), np.roll(i, 1, axis=1), np.roll(acts, 1, axis=1)
    shifted = run(sh_f, sh_i, sh_a)
    np.testing.assert_array_equal(shifted[:, 1:], base[:, :-1])
    tumble = f.copy()
    w = [names.index(f"omega_{a}") for a in "xyz"]
    for e, mag in ((5, 30.0), (9, 150.0), (70, 250.0), (133, 30.0)):
        tumble[w, e] = mag / np.sqrt(3)
    got = run(tumble, i.copy(), acts)
    keep = np.setdiff1d(np.arange(E), [5, 9, 70, 133])
    np.testing.assert_array_equal(got[:, keep], base[:, keep])
    assert not np.array_equal(got[:, 5], base[:, 5])
    env.close()
