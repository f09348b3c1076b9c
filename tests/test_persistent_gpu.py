"""The persistent HoverAviary step (include/adrp.h adrp_persistent_*, csrc/hover_persist.h) against
the launched step kernel: BASELINE config 1's loop (examples/pid.py:101-147 stepping
envs/BaseAviary.py:262-387 one env at a time) without a launch per step.  Two envs built alike,
one stepped with HoverAviary.step (a launch each), one through HoverAviary.persistent(): obs,
reward, flags, terminal obs and, after the persistent kernel ends, the whole SoA state are bit for
bit the launched kernel's over 100 steps with auto-resets.  Needs an MI355X: -m gpu."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.envs.hover import HoverAviary  # noqa: E402
from gym_pybullet_adrp_amd.utils.enums import ActionType, Physics  # noqa: E402


def _pair(E, precision, physics=Physics.PYB, act=ActionType.RPM):
    """the launched env on its default kernel (the LDS-staged one with the reset-helper wave when
    E % 64 == 0, the row-store one otherwise) and its persistent twin: the hover TUs contract a*b+c
    only within one source expression (csrc/Makefile CONTRACT), so every dispatch form of the step
    body gives the same bits"""
    kw = dict(num_envs=E, physics=physics, act=act, precision=precision, seed=31, initial_xyzs=[0, 0, 1.0],
              init_noise={"xyz": 0.1, "rpy": 0.2, "vel": 0.3, "omega": 1.0})
    return HoverAviary(**kw), HoverAviary(**kw)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("E,physics,act", [(1, Physics.PYB, ActionType.RPM), (100, Physics.PYB, ActionType.RPM),
                                           (128, Physics.PYB, ActionType.RPM),
                                           (70, Physics.PYB_GND_DRAG_DW, ActionType.ONE_D_RPM),
                                           (3, Physics.DYN, ActionType.RPM),
                                           (192, Physics.PYB, ActionType.RPM),
                                           (5, Physics.PYB_GND, ActionType.ONE_D_RPM)])
def test_persistent_bit_identical_to_launched(E, physics, act, precision):
    a, b = _pair(E, precision, physics, act)
    a.reset()
    b.reset()
    A = a.h.A
    rng = np.random.default_rng(5)
    acts = rng.uniform(-1, 1, (100, E, 1, A)).astype(np.float32)
    acts[40:60] = 1.0                    # climb out of bounds: truncations and auto-resets
    done = 0
    with b.persistent() as p:
        for k in range(100):
            oa, ra, ta, tra, ia = a.step(torch.from_numpy(acts[k]).to(a.device))
            ob, rb, tb, trb, ib = p.step(acts[k])
            oa, ra, ta, tra = oa.cpu().numpy(), ra.cpu().numpy(), ta.cpu().numpy(), tra.cpu().numpy()
            np.testing.assert_array_equal(ob, oa, err_msg=f"obs at step {k}")
            np.testing.assert_array_equal(rb, ra, err_msg=f"reward at step {k}")
            np.testing.assert_array_equal(tb, ta, err_msg=f"terminated at step {k}")
            np.testing.assert_array_equal(trb, tra, err_msg=f"truncated at step {k}")
            d = ta | tra
            np.testing.assert_array_equal(ib["terminal_observation"][d], ia["terminal_observation"].cpu().numpy()[d])
            done += int(d.sum())
        with pytest.raises(_lib.AdrpError):
            b.step(torch.from_numpy(acts[0]).to(b.device))     # refused while the kernel is resident
    assert done > 0, "the run should exercise auto-reset"
    fa, ia_ = a.get_state()
    fb, ib_ = b.get_state()
    np.testing.assert_array_equal(fa.cpu().numpy(), fb.cpu().numpy())
    np.testing.assert_array_equal(ia_.cpu().numpy(), ib_.cpu().numpy())
    # the env steps normally again after the persistent kernel ended
    a.step(torch.from_numpy(acts[0]).to(a.device))
    b.step(torch.from_numpy(acts[0]).to(b.device))
    assert torch.equal(a._obs, b._obs)
    a.close()
    b.close()


def test_persistent_restart_and_close_order():
    """begin / end twice on one env, and an env closed while its persistent kernel is resident
    (adrp_destroy ends it)"""
    env = HoverAviary(num_envs=1, seed=3)
    env.reset()
    act = np.zeros((1, 1, 4), np.float32)
    for _ in range(2):
        with env.persistent() as p:
            for _ in range(5):
                p.step(act)
    p = env.persistent()
    p.step(act)
    env.close()          # ends the resident kernel
    p.close()            # no-op after the env is gone


@pytest.mark.parametrize("E,physics,act,steps", [(70, Physics.PYB_GND_DRAG_DW, ActionType.ONE_D_RPM, 3000),
                                                 (1, Physics.PYB, ActionType.RPM, 5000)])
def test_persistent_long_run_no_stale_outputs(E, physics, act, steps):
    """3,000 steps at E = 70 (the case where, without the release before `done`, the host once read
    the previous step's obs rows), and 5,000 at E = 1 in line mode (the action and its request tag
    in one 64-byte line, read by one load: a torn read would step on a stale action): every step's
    outputs bit for bit the launched kernel's, with a fresh random action every step"""
    a, b = _pair(E, "fp64", physics, act)
    a.reset()
    b.reset()
    A = a.h.A
    rng = np.random.default_rng(9)
    bad = []
    with b.persistent() as p:
        for k in range(steps):
            act = rng.uniform(-1, 1, (E, 1, A)).astype(np.float32)
            if (k // 50) % 4 == 1:
                act[:] = 1.0
            oa, ra, ta, tra, _ = a.step(torch.from_numpy(act).to(a.device))
            ob, rb, tb, trb, _ = p.step(act)
            if not (np.array_equal(ob, oa.cpu().numpy()) and np.array_equal(rb, ra.cpu().numpy())
                    and np.array_equal(tb, ta.cpu().numpy()) and np.array_equal(trb, tra.cpu().numpy())):
                bad.append(k)
    assert not bad, f"{len(bad)} steps differ, first {bad[:5]}"
    a.close()
    b.close()


def test_persistent_refuses_reseed_and_state_changes():
    """while the resident kernel owns the env, reset(seed=...) (adrp_reseed), reset(),
    set_state and step are refused before any change: the persistent run continues bit for bit like
    a launched twin that never saw the calls"""
    a, b = _pair(64, "fp64")
    a.reset()
    b.reset()
    rng = np.random.default_rng(3)
    acts = rng.uniform(-1, 1, (30, 64, 1, 4)).astype(np.float32)
    with b.persistent() as p:
        for k in range(30):
            if k == 10:
                with pytest.raises(_lib.AdrpError):
                    b.reset(seed=123)
                with pytest.raises(_lib.AdrpError):
                    b.reset()
                with pytest.raises(_lib.AdrpError):
                    b.get_state()
            oa, ra, _, _, _ = a.step(torch.from_numpy(acts[k]).to(a.device))
            ob, rb, _, _, _ = p.step(acts[k])
            np.testing.assert_array_equal(ob, oa.cpu().numpy(), err_msg=f"obs at step {k}")
            np.testing.assert_array_equal(rb, ra.cpu().numpy(), err_msg=f"reward at step {k}")
    fa, ia_ = a.get_state()
    fb, ib_ = b.get_state()
    np.testing.assert_array_equal(fa.cpu().numpy(), fb.cpu().numpy())
    np.testing.assert_array_equal(ia_.cpu().numpy(), ib_.cpu().numpy())
    a.close()
    b.close()
