"""High-level command mode of the race kernel vs the CPU oracle.  Needs an
MI355X: -m gpu.

Both sides restate the firmware's commander / planner (csrc/commander.h, oracle/race.c hl_*;
parity with pycffirmware itself is unpinned).  Teacher forcing as in test_race_gpu.py: every
step starts from the oracle's state (body + command state, float32-representable), one command
per drone is sent to both, one env.step is compared.  Every env follows its own script mixing
all eleven commands, so FLYING / IDLE planners, FULLSTATE / commander / unset setpoints and
overrides on and off all occur in one launch.

Tolerance: the closed-loop 2e-3 of test_race_gpu.py for the fp64 kernel; 5e-3 for fp32.  A TAKEOFF
[h, d] plans from t_begin = d (args[-1], MellingerControl.py:57) while the controller clock starts at
0, so for a while the setpoint is the polynomial extrapolated to negative times, tens of metres away:
the controls saturate, and the fp32 kernel's last-ulp differences cross the PWM clips and int16
truncations more often than in the FULLSTATE flights of test_race_gpu.py (measured 3.5e-3 on level3).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd.commands import encode_commands  # noqa: E402
from gym_pybullet_adrp_amd.envs.race import MultiRaceAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import Command, Physics, RaceMode  # noqa: E402
from oracle import oracle as O  # noqa: E402

from test_race_gpu import check_state, sync  # noqa: E402

PLAN, OVR, MODE = 0, 1, 2
T0, DUR, COEF = 29, 30, 31


def script(e, k, obs0, n):
    """command of drone n of env e at step k"""
    p = obs0[e, n, :3].astype(float)
    z3 = np.zeros(3)
    v = (e + n) % 6
    if k == 0:
        return [(Command.TAKEOFF, [0.5, 1.0]), (Command.TAKEOFFYAW, [0.6, 0.8, 0.4]),
                (Command.TAKEOFFVEL, [0.4, 0.5, True]), (Command.GOTO, [p + [0.2, 0.1, 0.5], 0.2, 1.5, False]),
                (Command.FULLSTATE, [p + [0, 0, 0.5], [0.1, 0, 0.2], [0.5, 0.5, 0.5], 0.3, [0, 0, 0.2], 0.0]),
                (Command.NONE, [])][v]
    if k == 3:
        return [(Command.GOTO, [np.array([0.1, -0.2, 0.2]), 0.5, 1.0, True]), (Command.NOTIFY, [0.12]),
                (Command.LAND, [0.0, 2.0]), (Command.STOP, [0.12]),
                (Command.LANDYAW, [0.1, 1.0, 0.2]), (Command.TAKEOFF, [0.7, 0.5])][v]
    if k == 5:
        return [(Command.FULLSTATE, [p + [0.3, 0, 0.6], z3, z3, -0.2, z3, 0.2]), (Command.LANDVEL, [0.2, 0.3, True]),
                (Command.GOTO, [p + [-0.2, 0.3, 0.6], -0.5, 0.6, False]), (Command.NOTIFY, [0.2]),
                (Command.NONE, []), (Command.GOTO, [np.array([0.0, 0.0, 0.1]), 3.0, 0.4, True])][v]
    return (Command.NONE, [])


def encode_step(k, obs0, E, N):
    return encode_commands([[script(e, k, obs0, n) for n in range(N)] for e in range(E)], E, N)


def sync_cmd(env, orc):
    f, i = orc.get_command_state()
    env.set_command_state(torch.from_numpy(f), torch.from_numpy(i))


CMD_GROUPS = {"sp_pos": range(0, 3), "sp_vel": range(3, 6), "sp_acc": range(6, 9), "sp_rate": range(9, 12),
              "sp_quat": range(12, 14), "sp_yaw": range(14, 15), "c_pos": range(15, 18), "c_vel": range(18, 21),
              "c_yaw": range(21, 22), "st_pos": range(22, 25), "st_vel": range(25, 28), "st_yaw": range(28, 29)}


def cmd_errors(env, orc, worst=None):
    """max |gpu - cpu| / max(|cpu|, floor) per command-state field group (per-group bounds);
    floor 1e-3 (m, m/s, quaternion), 1 degree for the yaw fields (the firmware keeps yaw in degrees)"""
    fg = env.get_command_state()[0].cpu().numpy().astype(np.float64)
    fo = orc.get_command_state()[0].astype(np.float64)
    worst = {} if worst is None else worst
    for g, rows in CMD_GROUPS.items():
        r = list(rows)
        floor = 1.0 if g.endswith("yaw") else 1e-3
        d = np.linalg.norm(fg[r] - fo[r], axis=0) / np.maximum(np.linalg.norm(fo[r], axis=0), floor)
        worst[g] = max(worst.get(g, 0.0), float(d.max()))
    return worst


# per field group, |gpu - cpu| / max(|cpu|, floor) (cmd_errors), measured worst over every teacher-
# forced case of this file (fp32 / fp64): setpoints 1.4e-7 / 1.4e-7 (from float32 FULLSTATE args);
# commander position 3.6e-7 / 9e-9, velocity 1.1e-5 / 6.6e-7, yaw <= 2e-4 / 1.8e-5 (a float atan2 in
# degrees: the kernels' hardware transcendentals vs libm).  The firmware-state copies st_* mirror
# the body state, so they carry the closed-loop bar of the body (int16 moment flips, module doc).
CMD_TOL = {"fp32": {"sp_pos": 1e-6, "sp_vel": 1e-6, "sp_acc": 1e-6, "sp_rate": 1e-6, "sp_quat": 1e-6, "sp_yaw": 1e-6,
                    "c_pos": 1e-5, "c_vel": 1e-4, "c_yaw": 2e-3},
           "fp64": {"sp_pos": 1e-6, "sp_vel": 1e-6, "sp_acc": 1e-6, "sp_rate": 1e-6, "sp_quat": 1e-6, "sp_yaw": 1e-6,
                    "c_pos": 1e-6, "c_vel": 1e-5, "c_yaw": 2e-4}}


def check_cmd(env, orc, rtol):
    fg, ig = (t.cpu().numpy() for t in env.get_command_state())
    fo, io = orc.get_command_state()
    np.testing.assert_array_equal(ig, io)
    np.testing.assert_array_equal(fg[T0], fo[T0])
    np.testing.assert_allclose(fg[DUR], fo[DUR], rtol=1e-6)
    np.testing.assert_allclose(fg[COEF:], fo[COEF:], rtol=1e-4, atol=1e-4)
    # setpoint and commander fields: their own bounds; the firmware-state copies follow the body
    tol = CMD_TOL["fp64" if env.cfg.precision else "fp32"]
    for g, err in cmd_errors(env, orc).items():
        bound = tol.get(g, rtol)
        assert err <= bound, f"command state {g}: {err:.3e} > {bound:.1e}"
    np.testing.assert_allclose(fg[:COEF], fo[:COEF], rtol=rtol, atol=5e-3)


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
@pytest.mark.parametrize("level,N,physics,mode", [("level0", 2, Physics.PYB, RaceMode.COMPARE),
                                                  ("level3", 3, Physics.PYB_DW, RaceMode.COMPETE)])
def test_commands_teacher_forced(level, N, physics, mode, precision):
    E = 48
    env = MultiRaceAviary(level, num_drones=N, physics=physics, racemode=mode, num_envs=E, seed=11,
                          autoreset=False, precision=precision, commands=True)
    orc = O.Oracle(env.cfg.copy())
    env.reset()
    obs0 = orc.reset()
    sync(env, orc)
    sync_cmd(env, orc)
    worst, worst_s = {}, {}
    for k in range(8):
        codes, args = encode_step(k, obs0, E, N)
        orc.command(codes, args)
        obs_o, rew_o, te_o, tr_o, _ = orc.step(None)
        obs_g, rew_g, te_g, tr_g, _ = env.step((codes, args))
        rtol = 5e-3 if precision == "fp32" else 2e-3
        cmd_errors(env, orc, worst)
        check_cmd(env, orc, rtol)
        for g, v in check_state(env, orc, rtol).items():
            worst_s[g] = max(worst_s.get(g, 0.0), v)
        og = obs_g.cpu().numpy()
        np.testing.assert_allclose(og[..., :3], obs_o[..., :3], rtol=rtol, atol=1e-3)
        np.testing.assert_array_equal(te_g.cpu().numpy(), te_o)
        sync(env, orc)
        sync_cmd(env, orc)
    print(f"\n[cmd-errors] {level} {precision} command state {worst} body {worst_s}")
    env.close()


def test_tuple_actions_through_step():
    """the reference's list-of-tuples action (E = 1) through MultiRaceAviary.step, and ndarray
    actions in command mode (FULLSTATE sent by the step kernel) against the oracle"""
    N = 2
    env = MultiRaceAviary("level0", num_drones=N, precision="fp32", num_envs=1, seed=3, autoreset=False)
    orc = O.Oracle(env.cfg.copy())
    env.reset()
    obs0 = orc.reset()
    acts = [[(Command.TAKEOFF, [0.5, 1.0]), (Command.GOTO, [obs0[0, 1, :3] + [0, 0, 0.5], 0.0, 1.0, False])]]
    acts += [[(Command.NONE, []), (Command.NONE, [])]] * 3
    for a in acts:
        codes, args = encode_commands(a, 1, N)
        orc.command(codes, args)
        obs_o, *_ = orc.step(None)
        obs_g, *_ = env.step(a)   # the reference's format: one (Command, args) per drone
        np.testing.assert_allclose(obs_g.cpu().numpy()[..., :12], obs_o[..., :12], rtol=2e-3, atol=2e-3)
        sync(env, orc)
        sync_cmd(env, orc)
    assert env.commands
    tgt = np.concatenate([obs0[:, :, :3] + [0.1, 0, 0.6], np.zeros((1, N, 1))], -1).astype(np.float32)
    for _ in range(3):
        obs_o, *_ = orc.step(tgt)
        obs_g, *_ = env.step(torch.from_numpy(tgt).to(env.device))
        check_cmd(env, orc, 2e-3)
        check_state(env, orc, 2e-3)
        sync(env, orc)
        sync_cmd(env, orc)
    env.close()


def test_enable_commands_matches_reset_state():
    """adrp_enable_commands after a reset leaves what a reset in command mode leaves"""
    E, N = 16, 3
    a = MultiRaceAviary("level2", num_drones=N, precision="fp32", num_envs=E, seed=8, autoreset=False)
    b = MultiRaceAviary("level2", num_drones=N, precision="fp32", num_envs=E, seed=8, autoreset=False, commands=True)
    a.reset()
    b.reset()
    a.enable_commands()
    fa, ia = (t.cpu().numpy() for t in a.get_command_state())
    fb, ib = (t.cpu().numpy() for t in b.get_command_state())
    np.testing.assert_array_equal(ia, ib)
    np.testing.assert_array_equal(fa, fb)
    orc = O.Oracle(b.cfg.copy())
    orc.reset()
    fo, io = orc.get_command_state()
    np.testing.assert_array_equal(ib, io)
    np.testing.assert_allclose(fb, fo, atol=1e-6)
    a.close()
    b.close()


@pytest.mark.parametrize("obs_wrapper", [0, 1])
def test_commands_after_ndarray_steps(obs_wrapper):
    """commands enabled implicitly mid-episode.  After ndarray (FULLSTATE) steps the
    reference's controllers hold the last FULLSTATE setpoint (override on), so a drone given
    Command.NONE keeps flying to it while another gets a GOTO; the enabled command state must match
    the oracle's (which runs the command path on every step) and so must the next steps."""
    from gym_pybullet_adrp_amd.utils.wrapper import DroneObservationWrapper
    E, N = 32, 2
    env = MultiRaceAviary("level0", num_drones=N, precision="fp32", num_envs=E, seed=5, autoreset=False)
    wenv = DroneObservationWrapper(env) if obs_wrapper else env
    orc = O.Oracle(env.cfg.copy())
    wenv.reset()
    obs0 = orc.reset()
    rng = np.random.default_rng(3)
    tgt = np.concatenate([obs0[..., :3] + rng.uniform(-0.3, 0.3, (E, N, 3)) + [0, 0, 0.5],
                          rng.uniform(-1, 1, (E, N, 1))], -1).astype(np.float32)
    at = torch.from_numpy(tgt).to(env.device)
    for _ in range(4):
        orc.step(tgt)
        wenv.step(at)
        sync(env, orc)
    assert not env.commands and env.kernel_name.endswith(",Q4>")
    cmds = [[(Command.NONE, []), (Command.GOTO, [obs0[e, 1, :3] + [0.2, 0.0, 0.6], 0.3, 1.0, False])]
            for e in range(E)]
    codes, args = encode_commands(cmds, E, N)
    orc.command(codes, args)
    obs_o, *_ = orc.step(None)
    obs_g, *_ = wenv.step(cmds)            # implicit enable: re-sends the last FULLSTATE, then the commands
    assert env.commands and env.kernel_name == "race_step<f32,PYB,G8,CMD>"
    check_cmd(env, orc, 2e-3)
    check_state(env, orc, 2e-3)
    for _ in range(3):
        sync(env, orc)
        sync_cmd(env, orc)
        none = [[(Command.NONE, [])] * N] * E
        orc.command(*encode_commands(none, E, N))
        orc.step(None)
        wenv.step(none)
        check_cmd(env, orc, 2e-3)
        check_state(env, orc, 2e-3)
    if obs_wrapper:
        wenv.detach()
        assert env.obs_wrapper == 0
    env.close()


# The scripted flight hovers for seconds (take-off, delay), where the body rates are ~1e-4 rad/s.
# A one-unit flip of the float firmware's int16 moment truncation between the kernel and the oracle
# (hardware vs libm float transcendentals; both precisions run the firmware in float) moves the rates
# by ~2e-5 rad/s within the step (measured: omega_y 2.3e-5 rad/s apart with all four RPMs identical
# at the end of the step, fp64).  So the rates are compared relative to max(|omega|, 0.05 rad/s).
OMEGA_FLOOR = 0.05


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_hardcoded_controller_teacher_forced(precision):
    """the reference's HardCodedController command stream (tests/golden/
    hardcoded_golden.npz, made from user_controller/HardCodedController.py itself) through the
    tensor-in command path: HardCodedCommander.predict on the device (its stream must equal the
    fixture's) -> MultiRaceAviary.step((codes, args)) -> adrp_race_command, against the oracle given
    the fixture's commands; teacher-forced for the whole flight (take-off, 12 s of FULLSTATE
    setpoints, NOTIFY, LAND) on getting_started, where it passes all four gates."""
    from gym_pybullet_adrp_amd.hardcoded import HardCodedCommander
    from test_hardcoded import fixture_commands, G
    E, N = 8, 2
    env = MultiRaceAviary("getting_started", num_drones=N, racemode=RaceMode.COMPARE, num_envs=E, seed=1,
                          autoreset=False, precision=precision)
    orc = O.Oracle(env.cfg.copy())
    obs, _ = env.reset()
    orc.reset()
    hc = HardCodedCommander(obs)
    f = float(G["hc_ctrl_freq"])
    worst, worst_s = {}, {}
    rtol = 5e-3 if precision == "fp32" else 2e-3
    for k in range(460):
        codes, args = hc.predict(k / f)
        want_c, want_a = fixture_commands(k, E)
        np.testing.assert_array_equal(codes.cpu().numpy(), want_c)
        # planned from the env's float32 reset obs (the reference plans from float64): 1e-8 m apart
        np.testing.assert_allclose(args.cpu().numpy(), want_a, rtol=0, atol=1e-6)
        orc.command(want_c, want_a)
        obs_o, _, te_o, tr_o, _ = orc.step(None)
        obs_g, _, te_g, tr_g, _ = env.step((codes, args))
        try:
            cmd_errors(env, orc, worst)
            check_cmd(env, orc, rtol)
            for g, v in check_state(env, orc, rtol, floors={"omega": OMEGA_FLOOR}).items():
                worst_s[g] = max(worst_s.get(g, 0.0), v)
        except AssertionError as e:
            raise AssertionError(f"step {k} (commands {want_c[0].tolist()}): {e}") from None
        np.testing.assert_array_equal(te_g.cpu().numpy(), te_o, err_msg=f"step {k}")
        if te_o.all():
            break
        sync(env, orc)
        sync_cmd(env, orc)
    assert te_o.all(), "the scripted flight finishes the track"
    assert env.current_gate.cpu().numpy().tolist() == [[4, 4]] * E
    print(f"\n[cmd-errors] hardcoded {precision} steps {k + 1} command state {worst} body {worst_s}")
    env.close()


def test_hardcoded_controller_free_flight():
    """no teacher forcing: 256 envs fly the device-side HardCodedCommander stream in fp64 and finish
    the track at the step the oracle's free flight (fixture stream) finishes it, +-3 steps"""
    from gym_pybullet_adrp_amd.hardcoded import HardCodedCommander
    from test_hardcoded import fixture_commands, G
    E, N = 256, 2
    env = MultiRaceAviary("getting_started", num_drones=N, racemode=RaceMode.COMPARE, num_envs=E, seed=1,
                          autoreset=False, precision="fp64")
    orc = O.Oracle(MultiRaceAviary("getting_started", num_drones=N, racemode=RaceMode.COMPARE, precision="fp32", num_envs=1,
                                   seed=1, autoreset=False).cfg.copy())
    obs, _ = env.reset()
    orc.reset()
    hc = HardCodedCommander(obs)
    f = float(G["hc_ctrl_freq"])
    done_o = None
    done_g = torch.full((E,), -1, dtype=torch.int64, device=env.device)
    for k in range(G["hc_cmd"].shape[0]):
        if done_o is None:
            orc.command(*fixture_commands(k))
            _, _, te_o, _, _ = orc.step(None)
            if te_o.any():
                done_o = k
        _, _, te_g, tr_g, _ = env.step(hc.predict(k / f))
        assert not tr_g.any()
        done_g = torch.where((done_g < 0) & te_g, k, done_g)
        if done_o is not None and bool((done_g >= 0).all()):
            break
    assert done_o is not None
    dg = done_g.cpu().numpy()
    assert (np.abs(dg - done_o) <= 3).all(), (done_o, np.unique(dg))
    print(f"\n[hardcoded] oracle finished at step {done_o}, gpu fp64 at {np.unique(dg)}")
    env.close()
