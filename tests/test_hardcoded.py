"""The reference's HardCodedController (user_controller/HardCodedController.py:14-190), driven as
scripts/sim.py:68-106 drives it, pinned by tests/golden/hardcoded_golden.npz (made by
tests/golden/make_golden.py, GOLDEN_ONLY=hardcoded: the reference controller itself under the
pybullet / gymnasium stand-ins, getting_started, 2 drones, delay = drone index, 990 steps).

* gym_pybullet_adrp_amd.hardcoded.HardCodedCommander (the batched, tensor-out restatement)
  reproduces the reference's command stream for every env of a batch;
* the getting_started reset observation the controllers are built from matches the reference's;
* closed loop on the CPU oracle: the reference's command stream, sent through the command path
  (adrp_race_command semantics, commands.py encoding), flies both drones through all four gates
  and the episode terminates on completion.
"""
import os

import numpy as np
import pytest
import torch

from gym_pybullet_adrp_amd.commands import COMMAND_CODE, TIME_SLOT, CMD_ARGS
from gym_pybullet_adrp_amd.envs.race import race_config
from gym_pybullet_adrp_amd.hardcoded import HardCodedCommander
from gym_pybullet_adrp_amd.utils.enums import Command
from oracle import oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "hardcoded_golden.npz"))
K = G["hc_cmd"].shape[0]
DT = 1.0 / float(G["hc_ctrl_freq"])


def fixture_commands(k, E=1):
    """step k of the fixture as (codes [E, 2], args [E, 2, 14]) in the commands.py layout:
    positional arguments flattened in slots 0.., args[-1] in the clock slot"""
    codes = np.array([COMMAND_CODE[Command(v)] for v in G["hc_cmd"][k]], np.int32)
    args = np.zeros((2, CMD_ARGS))
    for n in range(2):
        m = int(G["hc_nflat"][k, n])
        args[n, :m] = G["hc_flat"][k, n, :m]
        if m:
            args[n, TIME_SLOT] = G["hc_flat"][k, n, m - 1]
    return np.broadcast_to(codes, (E, 2)).copy(), np.broadcast_to(args, (E, 2, CMD_ARGS)).copy()


def test_commander_reproduces_reference_stream():
    E = 3
    obs0 = np.broadcast_to(G["hc_obs0"], (E, 2, G["hc_obs0"].shape[1])).copy()
    hc = HardCodedCommander(torch.from_numpy(obs0))
    np.testing.assert_allclose(hc.reference_trajectory[0].numpy(), G["hc_ref"], rtol=0, atol=1e-12)
    for k in range(K):
        codes, args = hc.predict(k / float(G["hc_ctrl_freq"]))   # scripts/sim.py:79
        want_c, want_a = fixture_commands(k, E)
        np.testing.assert_array_equal(codes.numpy(), want_c, err_msg=f"step {k}")
        np.testing.assert_allclose(args.numpy(), want_a, rtol=0, atol=1e-12, err_msg=f"step {k}")


def test_commander_per_env_clocks_and_replan():
    """envs in different episodes: a [E] ep_time, and replan(mask) restarts a controller"""
    obs0 = np.broadcast_to(G["hc_obs0"], (2, 2, G["hc_obs0"].shape[1])).copy()
    hc = HardCodedCommander(obs0)
    f = float(G["hc_ctrl_freq"])
    for k in range(200):
        codes, args = hc.predict(torch.tensor([k / f, k / f]))
    hc.replan(obs0, mask=np.array([0, 1], np.uint8))
    codes, args = hc.predict(torch.tensor([200 / f, 0.0]))
    want0 = fixture_commands(200)
    want1 = fixture_commands(0)
    np.testing.assert_array_equal(codes[0].numpy(), want0[0][0])
    np.testing.assert_array_equal(codes[1].numpy(), want1[0][0])
    np.testing.assert_allclose(args[0].numpy(), want0[1][0], atol=1e-12)
    np.testing.assert_allclose(args[1].numpy(), want1[1][0], atol=1e-12)


def test_getting_started_reset_obs_matches_reference():
    cfg = race_config("getting_started", 2, "PYB", "COMPARE", num_envs=1, seed=1)
    obs = O.Oracle(cfg).reset()[0]
    ref = G["hc_obs0"]
    np.testing.assert_allclose(obs[:, :12], ref[:, :12], atol=1e-6)      # drone kinematics
    np.testing.assert_allclose(obs[:, 12:], ref[:, 12:], atol=1e-6)      # gates, obstacles, flags, gate id


def test_reference_stream_flies_the_track_on_oracle():
    cfg = race_config("getting_started", 2, "PYB", "COMPARE", num_envs=1, seed=1)
    cfg.autoreset = 0
    orc = O.Oracle(cfg)
    orc.reset()
    gate = orc.field_names()[1].index("gate")
    done_at = None
    for k in range(K):
        orc.command(*fixture_commands(k))
        _, _, te, tr, _ = orc.step(None)
        assert not tr.any()
        if te.any():
            done_at = k
            break
    assert done_at is not None, "the scripted flight should finish the track inside the episode"
    assert orc.get_state()[1][gate].tolist() == [4, 4]
    # drone 1 starts 1 s later (delay); it finishes last, after the end of its spline's 12 s
    assert (2 + 1 + 11) / DT < done_at < (2 + 1 + 12.5) / DT, done_at
