"""Generate golden fixtures from the reference's own Python code (run HERE only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

The reference (FelixWaiblinger/gym-pybullet-adrp @ 2024-10-08) imports pybullet,
gymnasium and munch, none of which exist in this image.  Its pure-numpy code paths are
executed unchanged under minimal stand-ins installed into ``sys.modules``:

* ``pybullet``: a kinematic pose store (loadURDF / resetBase* / getBase*), the three
  math helpers (getQuaternionFromEuler / getEulerFromQuaternion / getMatrixFromQuaternion
  via scipy's extrinsic 'xyz' convention, which is pybullet's away from gimbal lock),
  getLinkStates by forward kinematics of the URDF prop offsets, and *recorders* for
  applyExternalForce / applyExternalTorque.  Anything else raises.  stepSimulation is
  not available, so the Bullet integration itself is NOT pinned by these fixtures.
* ``gymnasium`` (Env, Wrapper, spaces.Box, envs.registration.register) and ``munch``.
* ``gym_pybullet_adrp.envs`` / ``.control`` are registered as bare packages so that their
  ``__init__`` files (which import Betaflight / pycffirmware code paths) are bypassed.
* MellingerControl gets a fake ``firm`` object that records what the wrapper hands the
  firmware and returns preset control outputs.

Only data (inputs and the reference's outputs) is written, to tests/golden/*.npz.
"""
import importlib
import math
import os
import sys
import types

import numpy as np
from scipy.spatial.transform import Rotation

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"

# --------------------------------------------------------------------------------------
# stand-ins
# --------------------------------------------------------------------------------------
PROP_OFFSETS = {  # inertial origins of prop0..3 / center_of_mass links, cf2x_IROS.urdf:41-99
    0: (0.028, 0.028, 0.0), 1: (-0.028, 0.028, 0.0), 2: (-0.028, -0.028, 0.0),
    3: (0.028, -0.028, 0.0), 4: (0.0, 0.0, 0.0)}


class _PB(types.ModuleType):
    DIRECT, GUI = 1, 2
    LINK_FRAME, WORLD_FRAME = 1, 2
    URDF_USE_INERTIA_FROM_FILE = 8

    def __init__(self):
        super().__init__("pybullet")
        self.reset_store()

    def reset_store(self):
        self.bodies = {}
        self.next_id = 0
        self.forces = []       # (body, link, force, pos, flags)
        self.torques = []      # (body, link, torque, flags)
        self.contacts = {}     # (bodyA, bodyB) -> bool
        self.closest = {}      # (bodyA, bodyB) -> bool
        self.rays = None

    # --- client / world ---
    def connect(self, *a, **k): return 0
    def disconnect(self, *a, **k): pass
    def resetSimulation(self, *a, **k):
        self.bodies = {}
        self.next_id = 0
    def setGravity(self, *a, **k): pass
    def setRealTimeSimulation(self, *a, **k): pass
    def setTimeStep(self, *a, **k): pass
    def setAdditionalSearchPath(self, *a, **k): pass
    def changeDynamics(self, *a, **k): pass
    def setCollisionFilterPair(self, *a, **k): pass

    def loadURDF(self, name, basePosition=(0, 0, 0), baseOrientation=(0, 0, 0, 1), **k):
        bid = self.next_id
        self.next_id += 1
        self.bodies[bid] = dict(name=str(name), pos=np.array(basePosition, float),
                                quat=np.array(baseOrientation, float),
                                vel=np.zeros(3), ang=np.zeros(3))
        return bid

    def resetBasePositionAndOrientation(self, bid, pos, quat, physicsClientId=0):
        self.bodies[bid]["pos"] = np.array(pos, float)
        self.bodies[bid]["quat"] = np.array(quat, float)

    def resetBaseVelocity(self, bid, linearVelocity, angularVelocity=(0, 0, 0), physicsClientId=0):
        self.bodies[bid]["vel"] = np.array(linearVelocity, float)
        self.bodies[bid]["ang"] = np.array(angularVelocity, float)

    def getBasePositionAndOrientation(self, bid, physicsClientId=0):
        b = self.bodies[bid]
        return tuple(b["pos"]), tuple(b["quat"])

    def getBaseVelocity(self, bid, physicsClientId=0):
        b = self.bodies[bid]
        return tuple(b["vel"]), tuple(b["ang"])

    # --- math helpers ---
    def getQuaternionFromEuler(self, rpy):
        r, p, y = rpy
        cr, sr = math.cos(r / 2), math.sin(r / 2)
        cp, sp = math.cos(p / 2), math.sin(p / 2)
        cy, sy = math.cos(y / 2), math.sin(y / 2)
        return (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy)

    def getEulerFromQuaternion(self, q):
        return tuple(Rotation.from_quat(np.asarray(q, float)).as_euler("xyz"))

    def getMatrixFromQuaternion(self, q):
        return tuple(Rotation.from_quat(np.asarray(q, float)).as_matrix().reshape(9))

    def getLinkStates(self, bid, linkIndices, computeLinkVelocity=0, computeForwardKinematics=0,
                      physicsClientId=0):
        b = self.bodies[bid]
        R = Rotation.from_quat(b["quat"]).as_matrix()
        out = []
        for i in linkIndices:
            w = b["pos"] + R @ np.array(PROP_OFFSETS[i])
            out.append((tuple(w), tuple(b["quat"])))
        return out

    # --- recorders / scripted queries ---
    def applyExternalForce(self, bid, linkIndex, forceObj, posObj, flags, physicsClientId=0):
        self.forces.append((bid, linkIndex, np.array(forceObj, float), np.array(posObj, float), flags))

    def applyExternalTorque(self, bid, linkIndex, torqueObj, flags, physicsClientId=0):
        self.torques.append((bid, linkIndex, np.array(torqueObj, float), flags))

    def getContactPoints(self, bodyA=None, bodyB=None, physicsClientId=0):
        return [1] if self.contacts.get((bodyA, bodyB), False) else []

    def getClosestPoints(self, bodyA, bodyB, distance, physicsClientId=0):
        return [1] if self.closest.get((bodyA, bodyB), False) else []

    def rayTestBatch(self, rayFromPositions, rayToPositions, physicsClientId=0):
        self.rays = (np.array(rayFromPositions), np.array(rayToPositions))
        return self.ray_result

    def stepSimulation(self, *a, **k):
        raise RuntimeError("stepSimulation is not available: Bullet is not in this image")

    def __getattr__(self, name):
        raise AttributeError(f"pybullet stand-in has no {name}")


def install_stubs():
    pb = _PB()
    sys.modules["pybullet"] = pb
    pbd = types.ModuleType("pybullet_data")
    pbd.getDataPath = lambda: "/nonexistent"
    sys.modules["pybullet_data"] = pbd

    gym = types.ModuleType("gymnasium")

    class Env:
        _np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.default_rng(0)
            return self._np_random

    class Wrapper(Env):
        def __init__(self, env):
            self.env = env

        def __getattr__(self, name):   # gymnasium 0.28 (pyproject.toml:21): public attributes forward
            if name.startswith("_") or name == "env":
                raise AttributeError(f"accessing private attribute '{name}' is prohibited")
            return getattr(self.env, name)

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low = np.broadcast_to(np.asarray(low), shape) if shape else np.asarray(low)
            self.high = np.broadcast_to(np.asarray(high), shape) if shape else np.asarray(high)
            self.shape = self.low.shape
            self.dtype = np.dtype(dtype)

    spaces = types.ModuleType("gymnasium.spaces")
    spaces.Box = Box
    envs = types.ModuleType("gymnasium.envs")
    reg = types.ModuleType("gymnasium.envs.registration")
    reg.register = lambda **k: None
    gym.Env, gym.Wrapper, gym.spaces = Env, Wrapper, spaces
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces, "gymnasium.envs": envs,
                        "gymnasium.envs.registration": reg})

    munch = types.ModuleType("munch")

    class Munch(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    def munchify(x):
        if isinstance(x, dict):
            return Munch({k: munchify(v) for k, v in x.items()})
        if isinstance(x, list):
            return [munchify(v) for v in x]
        return x

    munch.Munch, munch.munchify = Munch, munchify
    sys.modules["munch"] = munch
    return pb


def import_reference(pb):
    sys.path.insert(0, REF)
    import gym_pybullet_adrp  # noqa: F401  (registry, stubbed)
    for sub in ("envs", "control"):
        mod = types.ModuleType(f"gym_pybullet_adrp.{sub}")
        mod.__path__ = [os.path.join(REF, "gym_pybullet_adrp", sub)]
        sys.modules[f"gym_pybullet_adrp.{sub}"] = mod
    ctrl = sys.modules["gym_pybullet_adrp.control"]
    ctrl.BaseControl = importlib.import_module("gym_pybullet_adrp.control.BaseControl").BaseControl
    ctrl.low_level_control = lambda *a, **k: None
    m = types.SimpleNamespace()
    m.enums = importlib.import_module("gym_pybullet_adrp.utils.enums")
    m.utils = importlib.import_module("gym_pybullet_adrp.utils.utils")
    m.BaseAviary = importlib.import_module("gym_pybullet_adrp.envs.BaseAviary")
    m.Hover = importlib.import_module("gym_pybullet_adrp.envs.HoverAviary")
    m.Mellinger = importlib.import_module("gym_pybullet_adrp.control.MellingerControl")
    m.MultiRace = importlib.import_module("gym_pybullet_adrp.envs.MultiRaceAviary")
    m.wrapper = importlib.import_module("gym_pybullet_adrp.utils.wrapper")
    return m


# --------------------------------------------------------------------------------------
# fixtures
# --------------------------------------------------------------------------------------
def set_drone_state(pb, env, i, pos, quat, vel, ang):
    did = env.DRONE_IDS[i]
    pb.resetBasePositionAndOrientation(did, pos, quat)
    pb.resetBaseVelocity(did, vel, ang)


def random_state(rng, center=(0, 0, 1), tilt=0.3):
    pos = np.asarray(center) + rng.uniform(-0.5, 0.5, 3)
    rpy = rng.uniform(-tilt, tilt, 3) * np.array([1, 1, 3])
    quat = np.array(sys.modules["pybullet"].getQuaternionFromEuler(rpy))
    return pos, quat, rng.uniform(-1, 1, 3), rng.uniform(-2, 2, 3)


def hover_fixtures(pb, m):
    E = m.enums
    out = {}
    env = m.Hover.HoverAviary(physics=E.Physics.PYB, act=E.ActionType.RPM)
    out["derived"] = np.array([env.HOVER_RPM, env.MAX_RPM, env.MAX_THRUST, env.GND_EFF_H_CLIP,
                               env.MAX_XY_TORQUE, env.MAX_Z_TORQUE])
    obs0, _ = env.reset()
    out["reset_obs"] = np.asarray(obs0)
    rng = np.random.default_rng(7)

    # (1) preprocess + obs assembly + reward / terminated / truncated on sampled states
    n = 200
    acts = rng.uniform(-1, 1, (n, 1, 4)).astype(np.float32)
    states = np.zeros((n, 13))
    rpms = np.zeros((n, 4)); obs = np.zeros((n, 72)); rew = np.zeros(n)
    term = np.zeros(n, bool); trunc = np.zeros(n, bool); counters = np.zeros(n, np.int64)
    for k in range(n):
        pos, quat, vel, ang = random_state(rng, tilt=0.3)
        if k % 17 == 0:
            pos = np.array([0.0, 0.0, 1.0]) + rng.uniform(-5e-5, 5e-5, 3)   # terminated case
        if k % 23 == 0:
            pos[0] = 1.5 + rng.uniform(-0.01, 0.01)                          # bound edge
        counter = int(rng.choice([0, 8, 1920, 1928, 1936, int(rng.integers(0, 2000))]))
        set_drone_state(pb, env, 0, pos, quat, vel, ang)
        env.step_counter = counter
        rpm = env._preprocessAction(acts[k])
        env._updateAndStoreKinematicInformation()
        states[k] = np.concatenate([pos, quat, vel, ang])
        rpms[k] = rpm[0]
        obs[k] = env._computeObs()[0]
        rew[k] = env._computeReward()
        term[k] = env._computeTerminated()
        trunc[k] = env._computeTruncated()
        counters[k] = counter
    out.update(pp_act=acts, pp_rpm=rpms, task_state=states, task_obs=obs, task_rew=rew,
               task_term=term, task_trunc=trunc, task_counter=counters)

    # ONE_D_RPM preprocess
    env1 = m.Hover.HoverAviary(physics=E.Physics.PYB, act=E.ActionType.ONE_D_RPM)
    a1 = rng.uniform(-1, 1, (64, 1, 1)).astype(np.float32)
    out["pp1_act"] = a1
    out["pp1_rpm"] = np.array([env1._preprocessAction(a)[0] for a in a1])
    return out


def force_fixtures(pb, m):
    """PYB force assembly: what _physics/_groundEffect/_drag/_downwash hand to pybullet."""
    E = m.enums
    rng = np.random.default_rng(11)
    out = {}
    for name, phys in (("pyb", E.Physics.PYB), ("gnd", E.Physics.PYB_GND), ("drag", E.Physics.PYB_DRAG),
                       ("dw", E.Physics.PYB_DW), ("all", E.Physics.PYB_GND_DRAG_DW)):
        nd = 3 if phys in (E.Physics.PYB_DW, E.Physics.PYB_GND_DRAG_DW) else 1
        # HoverAviary is single-drone; use its base classes directly for N > 1
        env = m.Hover.HoverAviary(physics=phys) if nd == 1 else _multi(m, phys, nd)
        env.reset()
        n = 64
        S = np.zeros((n, nd, 13)); RPM = np.zeros((n, 4)); PREV = np.zeros((n, 4))
        LF = np.zeros((n, 5, 3)); LT = np.zeros((n, 5, 3))
        for k in range(n):
            for i in range(nd):
                low = 0.02 if (k % 5 == 0 and i == 0) else 0.3
                pos, quat, vel, ang = random_state(rng, center=(0, 0, low + 0.4), tilt=0.4)
                if i > 0:
                    pos = S[k, 0, :3] + np.array([rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3),
                                                  rng.uniform(0.02, 0.6)])
                set_drone_state(pb, env, i, pos, quat, vel, ang)
                S[k, i] = np.concatenate([pos, quat, vel, ang])
            env._updateAndStoreKinematicInformation()
            rpm = rng.uniform(0.5, 1.2, 4) * env.HOVER_RPM
            prev = rng.uniform(0.5, 1.2, 4) * env.HOVER_RPM
            pb.forces.clear(); pb.torques.clear()
            env._physics(rpm, 0)
            if phys in (E.Physics.PYB_GND, E.Physics.PYB_GND_DRAG_DW):
                env._groundEffect(rpm, 0)
            if phys in (E.Physics.PYB_DRAG, E.Physics.PYB_GND_DRAG_DW):
                env._drag(prev, 0)
            if phys in (E.Physics.PYB_DW, E.Physics.PYB_GND_DRAG_DW):
                env._downwash(0)
            for (bid, link, f, p, fl) in pb.forces:
                assert bid == env.DRONE_IDS[0] and fl == pb.LINK_FRAME and not np.any(p)
                LF[k, link] += f
            for (bid, link, t, fl) in pb.torques:
                assert fl == pb.LINK_FRAME
                LT[k, link] += t
            RPM[k], PREV[k] = rpm, prev
        out.update({f"{name}_state": S, f"{name}_rpm": RPM, f"{name}_prev": PREV,
                    f"{name}_link_force": LF, f"{name}_link_torque": LT})
    return out


def _multi(m, phys, nd):
    """A BaseRLAviary with nd drones (MultiHoverAviary is out of scope; reuse Hover's
    task hooks on drone 0 only, the force models are per-drone)."""
    E = m.enums
    BRL = importlib.import_module("gym_pybullet_adrp.envs.BaseRLAviary").BaseRLAviary

    class _Multi(BRL):
        def _computeReward(self): return 0
        def _computeTerminated(self): return False
        def _computeTruncated(self): return False
        def _computeInfo(self): return {}

    return _Multi(num_drones=nd, physics=phys, pyb_freq=240, ctrl_freq=30, act=E.ActionType.RPM)


def dyn_fixtures(pb, m):
    """Physics.DYN full episodes through HoverAviary.step (fully reference code)."""
    E = m.enums
    rng = np.random.default_rng(3)
    env = m.Hover.HoverAviary(physics=E.Physics.DYN, act=E.ActionType.RPM)
    n_ep, T = 12, 40
    init = np.zeros((n_ep, 13)); acts = rng.uniform(-1, 1, (n_ep, T, 1, 4)).astype(np.float32)
    obs = np.zeros((n_ep, T, 72)); rew = np.zeros((n_ep, T)); term = np.zeros((n_ep, T), bool)
    trunc = np.zeros((n_ep, T), bool)
    ring0 = np.zeros((n_ep, 15, 4), np.float32)
    states = np.zeros((n_ep, T, 13))
    for ep in range(n_ep):
        env.reset()
        pos, quat, vel, ang = random_state(rng, center=(0, 0, 1.0), tilt=0.1)
        set_drone_state(pb, env, 0, pos, quat, vel, np.zeros(3))
        init[ep] = np.concatenate([pos, quat, vel, np.zeros(3)])
        ring0[ep] = np.array([np.asarray(a).reshape(4) for a in env.action_buffer])
        for t in range(T):
            o, r, te, tr, _ = env.step(acts[ep, t])
            obs[ep, t] = o[0]; rew[ep, t] = r; term[ep, t] = te; trunc[ep, t] = tr
            states[ep, t] = np.concatenate([env.pos[0], env.quat[0], env.vel[0], env.rpy_rates[0]])
    return dict(dyn_init=init, dyn_ring0=ring0, dyn_act=acts, dyn_obs=obs, dyn_rew=rew,
                dyn_term=term, dyn_trunc=trunc, dyn_state=states)


class _FakeFirm:
    """Records what MellingerControl hands the firmware; returns preset outputs."""

    class _Obj:
        def __init__(self, **kw):
            self.__dict__.update(kw)

    def __init__(self):
        self.calls = []
        self.preset = (0.0, 0.0, 0.0, 0.0)
        self.modeAbs, self.modeDisable = 1, 0

    def _vec(self):
        return self._Obj(x=0.0, y=0.0, z=0.0, timestamp=0)

    def lpf2pData(self): return self._Obj()
    def lpf2pInit(self, d, fs, fc): d.fs, d.fc = fs, fc
    def lpf2pApply(self, d, v): return v
    def control_t(self): return self._Obj(roll=0, pitch=0, yaw=0, thrust=0.0)

    def setpoint_t(self):
        o = self._Obj()
        o.position, o.velocity, o.acceleration = self._vec(), self._vec(), self._vec()
        o.attitudeRate = self._Obj(roll=0.0, pitch=0.0, yaw=0.0)
        o.attitudeQuaternion = self._Obj(x=0.0, y=0.0, z=0.0, w=1.0)
        o.mode = self._Obj(x=0, y=0, z=0, quat=0, roll=0, pitch=0, yaw=0)
        return o

    def sensorData_t(self):
        return self._Obj(acc=self._vec(), gyro=self._vec(), interruptTimestamp=0)

    def state_t(self):
        return self._Obj(attitude=self._Obj(roll=0.0, pitch=0.0, yaw=0.0, timestamp=0),
                         attitudeQuaternion=self._Obj(x=0.0, y=0.0, z=0.0, w=1.0, timestamp=0),
                         position=self._vec(), velocity=self._vec(), acc=self._vec())

    def controllerMellingerInit(self): pass
    def crtpCommanderHighLevelInit(self): pass
    def crtpCommanderHighLevelTellState(self, s): pass
    def crtpCommanderHighLevelStop(self): pass
    def crtpCommanderHighLevelUpdateTime(self, t): pass

    def controllerMellinger(self, control, setpoint, sensor, state, tick):
        self.calls.append(dict(
            tick=tick,
            quat=[state.attitudeQuaternion.x, state.attitudeQuaternion.y, state.attitudeQuaternion.z,
                  state.attitudeQuaternion.w],
            att=[state.attitude.roll, state.attitude.pitch, state.attitude.yaw],
            pos=[state.position.x, state.position.y, state.position.z],
            vel=[state.velocity.x, state.velocity.y, state.velocity.z],
            acc=[state.acc.x, state.acc.y, state.acc.z],
            sacc=[sensor.acc.x, sensor.acc.y, sensor.acc.z],
            sgyro=[sensor.gyro.x, sensor.gyro.y, sensor.gyro.z],
            sp_pos=[setpoint.position.x, setpoint.position.y, setpoint.position.z],
            sp_quat=[setpoint.attitudeQuaternion.x, setpoint.attitudeQuaternion.y,
                     setpoint.attitudeQuaternion.z, setpoint.attitudeQuaternion.w]))
        control.roll, control.pitch, control.yaw, control.thrust = self.preset


def mellinger_fixtures(pb, m):
    Mel = m.Mellinger
    firm = _FakeFirm()
    Mel.load_firmware = lambda *_: firm
    ctrl = Mel.MellingerControl(0, m.enums.DroneModel.CF2X)
    rng = np.random.default_rng(5)
    out = {}
    # _compute_pwms on int16-valued control outputs
    n = 512
    cin = np.stack([rng.integers(-32000, 32001, n), rng.integers(-32000, 32001, n),
                    rng.integers(-32000, 32001, n), rng.uniform(-5000, 90000, n)], 1).astype(float)
    cin[:8, :3] = 0
    pw = np.array([ctrl._compute_pwms(types.SimpleNamespace(roll=int(c[0]), pitch=int(c[1]), yaw=int(c[2]),
                                                           thrust=c[3])) for c in cin])
    out.update(mel_control=cin, mel_pwms=pw)
    # full computeControl chain with a scripted firmware: state/sensor packing + PWM->RPM
    init_obs = np.zeros((1, 12)); init_obs[0, :3] = [0.9, 0.9, 0.05]
    ctrl.reset(init_obs)
    ctrl._sendFullStateCmd([0.5, -0.3, 1.0], np.zeros(3), np.zeros(3), 0.3, np.zeros(3), 0)
    T = 120
    ins = np.zeros((T, 12)); noise = rng.normal(0, 0.001, (T, 4)); presets = np.zeros((T, 4)); rpms = np.zeros((T, 4))
    pos = np.array([0.9, 0.9, 0.05]); rpy = np.zeros(3); vel = np.zeros(3)
    for t in range(T):
        pos = pos + rng.uniform(-0.01, 0.01, 3); rpy = rpy + rng.uniform(-0.02, 0.02, 3)
        vel = vel + rng.uniform(-0.05, 0.05, 3)
        if t == 60:
            rpy[2] = math.pi - 0.001   # yaw wrap spike in the finite-difference "gyro"
        if t == 61:
            rpy[2] = -math.pi + 0.001
        presets[t] = [int(rng.integers(-3000, 3000)), int(rng.integers(-3000, 3000)),
                      int(rng.integers(-3000, 3000)), rng.uniform(20000, 60000)]
        firm.preset = tuple(presets[t])
        ins[t] = np.concatenate([pos, rpy, vel, np.zeros(3)])
        rpms[t] = ctrl.computeControl(t, pos.copy(), rpy.copy(), vel.copy(), np.zeros(3), noise[t])
    keys = ("tick", "quat", "att", "pos", "vel", "acc", "sacc", "sgyro", "sp_pos", "sp_quat")
    for k in keys:
        out[f"melrec_{k}"] = np.array([c[k] for c in firm.calls], float)
    out.update(mel_in=ins, mel_noise=noise, mel_preset=presets, mel_rpm=rpms)
    # the float64 tick schedule the wrapper passes to controllerMellinger (33 s x 500 Hz)
    firm.calls.clear()
    ctrl.reset(init_obs)
    for _ in range(16500):
        ctrl.state.acc.z = 1.0
        ctrl._step_controller()
    out["tick_schedule"] = np.array([c["tick"] for c in firm.calls], np.uint8)
    # get_quaternion_from_euler
    e = rng.uniform(-math.pi, math.pi, (256, 3))
    out["q_from_e_in"] = e
    out["q_from_e_out"] = np.array([m.utils.get_quaternion_from_euler(*x) for x in e])
    # LPF init arguments (swapped cut-offs)
    out["lpf_acc"] = np.array([ctrl.acclpf[0].fs, ctrl.acclpf[0].fc], float)
    out["lpf_gyro"] = np.array([ctrl.gyrolpf[0].fs, ctrl.gyrolpf[0].fc], float)
    return out


# --------------------------------------------------------------------------------------
# MultiRaceAviary decision logic: obs assembly, termination, truncation, gate progress
# (rays), RewardWrapper -- with the Bullet queries answered from scripted tables
# --------------------------------------------------------------------------------------
class _Conn:
    def send(self, x): pass
    def recv(self): return np.zeros(4)
    def close(self): pass


class _Proc:
    def __init__(self, *a, **k): pass
    def start(self): pass
    def join(self): pass


RACE_CFG = {   # config/level3.yaml track with the two SURVEY §8(d) extension drones
    "bounds": [[-3, -3, 0], [3, 3, 2]], "episode_len_sec": 33, "done_on_completion": True,
    "init_states": {f"drone{k}": {"pos": p, "vel": [0, 0, 0], "rpy": [0, 0, 0], "pqr": [0, 0, 0]}
                    for k, p in enumerate([[0.9, 0.9, 0.05], [1.1, 1.1, 0.05], [0.7, 0.9, 0.05], [1.3, 1.1, 0.05]])},
    "gates": [[0.45, -1.0, 0.525, 0, 0, 2.35, 1], [1.0, -1.55, 1.0, 0, 0, -0.78, 0],
              [0.0, 0.5, 0.525, 0, 0, 0, 1], [-0.5, -0.5, 1.0, 0, 0, 3.14, 0]],
    "obstacles": [[1.0, -0.5, 0.525, 0, 0, 0], [0.5, -1.5, 0.525, 0, 0, 0], [-0.5, 0, 0.525, 0, 0, 0],
                  [0, 1.0, 0.525, 0, 0, 0]],
    "random_gates_obstacles": False, "random_drone_state": False, "random_drone_inertia": False,
    "disturbances": False,
}


def race_fixtures(pb, m):
    E = m.enums
    MR = m.MultiRace
    MR.mp = types.SimpleNamespace(Pipe=lambda: (_Conn(), _Conn()), Process=_Proc)   # no controller processes
    cfg = sys.modules["munch"].munchify(RACE_CFG)
    rng = np.random.default_rng(21)
    out = {}
    for mode_name, mode in (("compete", E.RaceMode.COMPETE), ("compare", E.RaceMode.COMPARE)):
        N = 4 if mode_name == "compete" else 2
        env = MR.MultiRaceAviary(race_config=cfg, num_drones=N, racemode=mode)
        env.reset()
        gates_nom = np.array(env.gates_nominal, float)
        obst_nom = np.array(env.obstacles_nominal, float)
        # (a) _computeObs with scripted getClosestPoints answers
        n = 96
        D = env._computeObs().shape[1]
        kin = np.zeros((n, N, 12)); gact = np.zeros((n, 4, 4)); oact = np.zeros((n, 4, 3))
        gin = np.zeros((n, N, 4), np.uint8); oin = np.zeros((n, N, 4), np.uint8)
        cur = np.zeros((n, N), np.int64); obs = np.zeros((n, N, D))
        for k in range(n):
            for i in range(N):
                pos, quat, vel, ang = random_state(rng, center=(0, 0, 1), tilt=0.4)
                set_drone_state(pb, env, i, pos, quat, vel, ang)
            env._updateAndStoreKinematicInformation()
            ga = gates_nom.copy(); ga[:, [0, 1, 5]] += rng.uniform(-0.15, 0.15, (4, 3))
            oa = obst_nom.copy(); oa[:, :2] += rng.uniform(-0.15, 0.15, (4, 2))
            env.gates_actual = ga.tolist(); env.obstacles_actual = oa.tolist()
            env.current_gate = rng.integers(0, 5, N).astype(float)
            gi = rng.random((N, 4)) < 0.5; oi = rng.random((N, 4)) < 0.5
            pb.closest = {}
            for i in range(N):
                for g in range(4):
                    pb.closest[(env.gates_urdf[g], env.DRONE_IDS[i])] = bool(gi[i, g])
                    pb.closest[(env.obstacles_urdf[g], env.DRONE_IDS[i])] = bool(oi[i, g])
            obs[k] = env._computeObs()
            kin[k] = np.hstack([env.pos, env.rpy, env.vel, env.ang_v])
            gact[k] = ga[:, [0, 1, 2, 5]]; oact[k] = oa[:, :3]
            gin[k] = gi; oin[k] = oi; cur[k] = env.current_gate
        out.update({f"{mode_name}_obs_kin": kin, f"{mode_name}_obs_gact": gact, f"{mode_name}_obs_oact": oact,
                    f"{mode_name}_obs_gin": gin, f"{mode_name}_obs_oin": oin, f"{mode_name}_obs_cur": cur,
                    f"{mode_name}_obs": obs})
        # (b) _computeTerminated with scripted getContactPoints answers
        env.collision_objects = env.gates_urdf + env.obstacles_urdf + [env.PLANE_ID]
        if mode == E.RaceMode.COMPETE:
            env.collision_objects += env.DRONE_IDS.tolist()
        n = 128
        tpos = np.zeros((n, N, 3)); tang = np.zeros((n, N, 3)); tcon = np.zeros((n, N), np.uint8)
        telim0 = np.zeros((n, N), np.uint8); telim = np.zeros((n, N), np.uint8); tfin = np.zeros((n, N), np.uint8)
        tterm = np.zeros(n, bool)
        for k in range(n):
            for i in range(N):
                pos = rng.uniform(-3.3, 3.3, 3); pos[2] = rng.uniform(-0.2, 2.3)
                ang = rng.uniform(-25, 25, 3) * (rng.random() < 0.3) + rng.uniform(-1, 1, 3)
                set_drone_state(pb, env, i, pos, np.array([0, 0, 0, 1.0]), np.zeros(3), ang)
            env._updateAndStoreKinematicInformation()
            pb.contacts = {}
            con = rng.random(N) < 0.2
            for i in range(N):
                if con[i]:
                    obj = env.collision_objects[int(rng.integers(0, len(env.collision_objects)))]
                    pb.contacts[(obj, env.DRONE_IDS[i])] = True
            e0 = rng.random(N) < 0.2
            f0 = rng.random(N) < 0.3
            env.drones_eliminated = e0.copy(); env.drones_finished = f0.copy()
            tterm[k] = env._computeTerminated()
            tpos[k] = env.pos; tang[k] = env.ang_v
            tcon[k] = [any(pb.contacts.get((o, env.DRONE_IDS[i]), False) for o in env.collision_objects) for i in range(N)]
            telim0[k] = e0; telim[k] = env.drones_eliminated; tfin[k] = f0
        out.update({f"{mode_name}_term_pos": tpos, f"{mode_name}_term_angv": tang, f"{mode_name}_term_contact": tcon,
                    f"{mode_name}_term_elim0": telim0, f"{mode_name}_term_elim": telim,
                    f"{mode_name}_term_fin": tfin, f"{mode_name}_term": tterm})
    # (c) _computeTruncated around 33 s x 500 Hz
    counters = np.array([0, 20, 16480, 16499, 16500, 16501, 16520, 16540, 20000])
    tr = []
    for sc in counters:
        env.step_counter = int(sc)
        tr.append(env._computeTruncated())
    out.update(trunc_counter=counters, trunc=np.array(tr))
    # (d) _gate_progress with scripted rayTestBatch answers
    N = env.NUM_DRONES
    n = 160
    pg_gate0 = np.zeros((n, N), np.int64); pg_gate = np.zeros((n, N), np.int64); pg_fin = np.zeros((n, N), np.uint8)
    pg_gact = np.zeros((n, 4, 6)); pg_from = np.zeros((n, N, 7, 3)); pg_to = np.zeros((n, N, 7, 3))
    pg_id = np.zeros((n, N, 7), np.int64); pg_frac = np.zeros((n, N, 7))
    for k in range(n):
        ga = gates_nom.copy(); ga[:, [0, 1, 5]] += rng.uniform(-0.15, 0.15, (4, 3))
        env.gates_actual = ga.tolist()
        g0 = rng.integers(0, 5, N)
        env.current_gate = g0.astype(float)
        env.drones_finished = np.zeros(N, bool)
        for i in range(N):
            ids = rng.choice(list(env.DRONE_IDS) + [-1], 7)
            fr = np.where(rng.random(7) < 0.15, 0.99995, rng.uniform(0, 1.0, 7))
            fr[ids == -1] = 1.0
            pb.ray_result = [(int(ids[r]), -1, float(fr[r]), (0, 0, 0), (0, 0, 1)) for r in range(7)]
            pb.rays = None
            env._gate_progress(i)
            if pb.rays is not None:
                pg_from[k, i], pg_to[k, i] = pb.rays
            pg_id[k, i] = [list(env.DRONE_IDS).index(x) if x in list(env.DRONE_IDS) else -1 for x in ids]
            pg_frac[k, i] = fr
        pg_gate0[k] = g0; pg_gate[k] = env.current_gate; pg_fin[k] = env.drones_finished; pg_gact[k] = ga
    out.update(pg_gate0=pg_gate0, pg_gate=pg_gate, pg_fin=pg_fin, pg_gact=pg_gact, pg_from=pg_from, pg_to=pg_to,
               pg_id=pg_id, pg_frac=pg_frac)
    # (e) RewardWrapper on a scripted episode (info["task_completed"] supplied: the env has none)
    T = 40

    class _Scripted(sys.modules["gymnasium"].Env):
        def __init__(self, seq, obs0):
            self.seq, self.obs0, self.k = seq, obs0, 0
        def reset(self, *a, **k):
            return self.obs0, {}
        def step(self, action):
            r = self.seq[self.k]
            self.k += 1
            return r
    obs_seq = np.zeros((T + 1, 2, 49))
    obs_seq[:, :, :12] = rng.uniform(-1, 1, (T + 1, 2, 12))
    obs_seq[:, :, 12:28] = np.tile(np.array(RACE_CFG["gates"])[:, [0, 1, 2, 5]].ravel(), (T + 1, 2, 1))
    g = 0
    for t in range(T + 1):
        if t > 0 and rng.random() < 0.2 and g < 4:
            g += 1
        obs_seq[t, :, 48] = g
    term_seq = np.zeros(T, bool); term_seq[[15, 31, 39]] = True
    comp_seq = np.zeros(T, bool); comp_seq[31] = True
    seq = [(obs_seq[t + 1], 0, bool(term_seq[t]), False, {"task_completed": bool(comp_seq[t])}) for t in range(T)]
    w = m.wrapper.RewardWrapper(_Scripted(seq, obs_seq[0]))
    w.reset()
    rewards = []
    for t in range(T):
        if obs_seq[t + 1, 0, 48] >= 4 and obs_seq[t + 1, 0, 48] > w.current_gate_id % 4:
            # the reference raises KeyError (gate_positions has keys 0..3); stop the script here
            break
        rewards.append(w.step(np.zeros((2, 4)))[1])
    out.update(rw_obs=obs_seq, rw_term=term_seq, rw_completed=comp_seq, rw_reward=np.array(rewards))
    return out


def obswrap_fixtures(pb, m):
    """DroneObservationWrapper (utils/wrapper.py:38-65) on a scripted env: the in-place yaw zeroing
    of ndarray actions, the early termination at current_gate[0] >= 2, and both stackings with the
    RewardWrapper (the reward's terminal terms see the early termination only from outside)."""
    rng = np.random.default_rng(21)
    T, N = 30, 2

    class _Scripted(sys.modules["gymnasium"].Env):
        def __init__(self, seq, gates, obs0):
            self.seq, self.gates, self.obs0, self.k = seq, gates, obs0, 0
            self.current_gate = gates[0]
        def reset(self, *a, **k):
            self.k = 0
            self.current_gate = self.gates[0]
            return self.obs0, {}
        def step(self, action):
            r = self.seq[self.k]
            self.current_gate = self.gates[self.k + 1]
            self.k += 1
            return r
    obs_seq = np.zeros((T + 1, N, 49))
    obs_seq[:, :, :12] = rng.uniform(-1, 1, (T + 1, N, 12))
    obs_seq[:, :, 12:28] = np.tile(np.array(RACE_CFG["gates"])[:, [0, 1, 2, 5]].ravel(), (T + 1, N, 1))
    gates = np.zeros((T + 1, N), int)
    gates[:, 0] = [0] * 5 + [1] * 7 + [2] * 13 + [3] * 6      # drone 0 reaches gate 2 at step 12
    gates[:, 1] = [0] * 9 + [1] * 22
    obs_seq[:, :, 48] = gates
    term_env = np.zeros(T, bool); term_env[[7, 22]] = True
    seq = [(obs_seq[t + 1], 0.0, bool(term_env[t]), False, {"task_completed": False}) for t in range(T)]
    acts = rng.uniform(-1, 1, (T, N, 4))
    acts_after = np.zeros_like(acts)
    term_out = np.zeros(T, bool)
    W = m.wrapper
    env = W.DroneObservationWrapper(_Scripted(seq, gates, obs_seq[0]))
    env.reset()
    for t in range(T):
        a = acts[t].copy()
        _, _, term_out[t], _, _ = env.step(a)
        acts_after[t] = a
    rew = {}
    for name, make in (("inner", lambda e: W.RewardWrapper(W.DroneObservationWrapper(e))),
                       ("outer", lambda e: W.DroneObservationWrapper(W.RewardWrapper(e)))):
        env = make(_Scripted(seq, gates, obs_seq[0]))
        env.reset()
        r = []
        for t in range(T):
            if obs_seq[t + 1, 0, 48] >= 4:
                break
            r.append(env.step(acts[t].copy())[1])
        rew[name] = np.array(r)
    return dict(ow_obs=obs_seq, ow_gates=gates, ow_term_env=term_env, ow_act=acts, ow_act_after=acts_after,
                ow_term=term_out, ow_rew_inner=rew["inner"], ow_rew_outer=rew["outer"])


def pid_fixtures(pb, m):
    """DSLPIDControl (control/DSLPIDControl.py:82-259) and the HoverAviary PID / VEL /
    ONE_D_PID action types (BaseRLAviary.py:193-235), fully reference code."""
    E = m.enums
    DSL = importlib.import_module("gym_pybullet_adrp.control.DSLPIDControl").DSLPIDControl
    rng = np.random.default_rng(13)
    out = {}
    # (1) computeControl sequences from a fresh controller: inputs, RPM, controller state
    n_seq, T = 48, 12
    dt = 1 / 30
    cin = np.zeros((n_seq, T, 19))    # pos 3, quat 4, vel 3, target_pos 3, target_rpy 3, target_vel 3
    crpm = np.zeros((n_seq, T, 4)); cst = np.zeros((n_seq, T, 9))
    for s in range(n_seq):
        ctrl = DSL(drone_model=E.DroneModel.CF2X)
        big = s % 4 == 0                                   # saturate integrators / torques / PWM
        for t in range(T):
            pos, quat, vel, _ = random_state(rng, center=(0, 0, 1), tilt=0.6 if big else 0.2)
            tp = pos + rng.uniform(-3, 3, 3) * (4.0 if big else 0.3)
            trpy = np.array([0.0, 0.0, rng.uniform(-math.pi, math.pi) if s % 3 == 0 else 0.0])
            tv = rng.uniform(-1, 1, 3) * (s % 2)
            rpm, _, _ = ctrl.computeControl(control_timestep=dt, cur_pos=pos, cur_quat=quat, cur_vel=vel,
                                            cur_ang_vel=np.zeros(3), target_pos=tp, target_rpy=trpy,
                                            target_vel=tv)
            cin[s, t] = np.concatenate([pos, quat, vel, tp, trpy, tv])
            crpm[s, t] = rpm
            cst[s, t] = np.concatenate([ctrl.last_rpy, ctrl.integral_pos_e, ctrl.integral_rpy_e])
    out.update(dsl_in=cin, dsl_rpm=crpm, dsl_state=cst)
    # (2) closed-loop HoverAviary(physics=DYN) episodes per action type; the controller is
    # built once per env (BaseRLAviary.py:73-78) and never reset, so it carries across episodes
    for name, at, A in (("pid", E.ActionType.PID, 3), ("vel", E.ActionType.VEL, 4),
                        ("onedpid", E.ActionType.ONE_D_PID, 1)):
        env = m.Hover.HoverAviary(physics=E.Physics.DYN, act=at)
        n_ep, T = 4, 30
        init = np.zeros((n_ep, 13)); acts = np.zeros((n_ep, T, 1, A), np.float32)
        obs = np.zeros((n_ep, T, 12 + 15 * A)); rew = np.zeros((n_ep, T)); term = np.zeros((n_ep, T), bool)
        trunc = np.zeros((n_ep, T), bool); states = np.zeros((n_ep, T, 13)); rpms = np.zeros((n_ep, T, 4))
        ctl0 = np.zeros((n_ep, 9)); ctl = np.zeros((n_ep, T, 9)); ring0 = np.zeros((n_ep, 15, A), np.float32)
        for ep in range(n_ep):
            env.reset()
            pos, quat, vel, _ = random_state(rng, center=(0, 0, 1.0), tilt=0.1)
            set_drone_state(pb, env, 0, pos, quat, vel, np.zeros(3))
            env._updateAndStoreKinematicInformation()      # _preprocessAction reads the stored state
            init[ep] = np.concatenate([pos, quat, vel, np.zeros(3)])
            c = env.ctrl[0]
            ctl0[ep] = np.concatenate([c.last_rpy, c.integral_pos_e, c.integral_rpy_e])
            ring0[ep] = np.array([np.asarray(a, np.float32).reshape(A) for a in env.action_buffer])
            if name == "pid":
                a = np.clip(pos + rng.uniform(-0.6, 0.6, 3), -1, 1)
                a[2] = rng.uniform(0.5, 1.0)
                if ep == 3:
                    a = np.array([-1.0, 1.0, 1.0])          # > 1 m away: _calculateNextStep caps the step
                seq = np.repeat(a[None], T, 0) + rng.uniform(-0.05, 0.05, (T, 3)) * (ep % 2)
            elif name == "vel":
                seq = rng.uniform(-1, 1, (T, 4))
                seq[::7, :3] = 0                              # zero direction -> zero target velocity
            else:
                seq = rng.uniform(-1, 1, (T, 1))
            acts[ep] = seq.astype(np.float32)[:, None, :]
            for t in range(T):
                o, r, te, tr, _ = env.step(acts[ep, t])
                obs[ep, t] = o[0]; rew[ep, t] = r; term[ep, t] = te; trunc[ep, t] = tr
                states[ep, t] = np.concatenate([env.pos[0], env.quat[0], env.vel[0], env.rpy_rates[0]])
                rpms[ep, t] = env.last_clipped_action[0]
                ctl[ep, t] = np.concatenate([c.last_rpy, c.integral_pos_e, c.integral_rpy_e])
        out.update({f"{name}_init": init, f"{name}_act": acts, f"{name}_obs": obs, f"{name}_rew": rew,
                    f"{name}_term": term, f"{name}_trunc": trunc, f"{name}_state": states,
                    f"{name}_rpm": rpms, f"{name}_ctl0": ctl0, f"{name}_ctl": ctl, f"{name}_ring0": ring0})
    return out


def policy_fixtures(pb, m):
    """On-device policy: the actor weights of the reference's two SB3 zips
    (user_controller/*.zip, read with torch.load(weights_only=True), nothing unpickled) and
    the RLController / RLControllerTwoGates action transforms (user_controller/*.py:56-73)
    run on scripted agent outputs (stable_baselines3 is absent: PPO.load returns a stand-in
    whose predict hands back preset actions)."""
    import io
    import json
    import zipfile
    import torch
    out = {}
    keys = ("mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
            "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
            "action_net.weight", "action_net.bias")
    for name in ("example_RL_model", "twogates"):
        with zipfile.ZipFile(os.path.join(REF, "user_controller", name + ".zip")) as zf:
            sd = torch.load(io.BytesIO(zf.read("policy.pth")), map_location="cpu", weights_only=True)
            kw = json.loads(zf.read("data")).get("policy_kwargs") or {}
        for i, k in enumerate(keys):
            out[f"{name}_w{i}"] = sd[k].float().numpy()
        out[f"{name}_relu"] = np.array("ReLU" in str(kw.get("activation_fn", "Tanh")))

    class _Agent:
        preset = None

        def predict(self, obs, deterministic=True):
            return _Agent.preset.copy(), None

    sb3 = types.ModuleType("stable_baselines3")
    sb3.PPO = types.SimpleNamespace(load=lambda *_a, **_k: _Agent())
    sys.modules["stable_baselines3"] = sb3
    uc = types.ModuleType("user_controller")          # bypass the package __init__
    uc.__path__ = [os.path.join(REF, "user_controller")]
    sys.modules["user_controller"] = uc
    uc.BaseController = importlib.import_module("user_controller.BaseController").BaseController
    RL = importlib.import_module("user_controller.RLController").RLController
    RL2 = importlib.import_module("user_controller.RLControllerTwoGates").RLControllerTwoGates
    rng = np.random.default_rng(31)
    n = 256
    obs = np.zeros((n, 49))
    obs[:, :3] = rng.uniform(-3, 3, (n, 3))
    obs[:, 3:6] = rng.uniform(-math.pi, math.pi, (n, 3))
    obs[:, 6:12] = rng.uniform(-2, 2, (n, 6))
    obs[:, 12:] = rng.uniform(-1.5, 1.5, (n, 37))
    obs[:8, 5] = [math.pi, -math.pi, math.pi - 1e-7, -math.pi + 1e-7, 0.0, 3.0, -3.0, 1e-9]   # map2pi edges
    obs = obs.astype(np.float32).astype(np.float64)
    acts = rng.uniform(-1.2, 1.2, (n, 4)).astype(np.float32)
    rel = np.zeros((n, 4)); ab = np.zeros((n, 4))
    for k in range(n):
        c = RL(0, initial_obs=obs[k], initial_info={})
        _Agent.preset = acts[k]
        cmd, args = c.predict(obs[k], ep_time=0.0)
        rel[k] = np.concatenate([np.asarray(args[0], float), [args[3]]])
        c2 = RL2(0, initial_obs=obs[k], initial_info={})
        _Agent.preset = acts[k][None, :].astype(np.float64)
        cmd2, args2 = c2.predict(obs[k], ep_time=0.0)
        ab[k] = np.concatenate([np.asarray(args2[0], float), [args2[3]]])
    out.update(pol_obs=obs, pol_agent_act=acts, pol_relative=rel, pol_absolute=ab)
    return out


def critic_fixtures():
    """On-device PPO rollout: the critic (mlp_extractor.value_net, value_net) and
    the Gaussian log_std of the reference's two SB3 zips (user_controller/*.zip; policy.pth read with
    torch.load(weights_only=True), the `data` member as JSON: nothing unpickled), and the PPO
    hyper-parameters the zips were trained with (gamma, gae_lambda, n_steps)."""
    import io
    import json
    import zipfile
    import torch
    out = {}
    keys = ("mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
            "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
            "value_net.weight", "value_net.bias", "log_std")
    for name in ("example_RL_model", "twogates"):
        with zipfile.ZipFile(os.path.join(REF, "user_controller", name + ".zip")) as zf:
            sd = torch.load(io.BytesIO(zf.read("policy.pth")), map_location="cpu", weights_only=True)
            data = json.loads(zf.read("data"))
        for i, k in enumerate(keys):
            out[f"{name}_v{i}"] = sd[k].float().numpy()
        out[f"{name}_hp"] = np.array([float(data["gamma"]), float(data["gae_lambda"]), float(data["n_steps"])])
    return out


def hardcoded_fixtures(pb, m):
    """HardCodedController (user_controller/HardCodedController.py:14-190) as scripts/sim.py:68-106
    drives it: config/getting_started.yaml, 2 drones, COMPARE, info["delay"] = drone_id, one
    predict(obs[i], ep_time=episode_step / ctrl_freq) per drone per step, for the 33 s episode.
    Recorded: the reset observation the controllers are built from, and per step and drone the
    command's value string and its arguments flattened in the reference's order (args[-1] last)."""
    import yaml
    E = m.enums
    MR = m.MultiRace
    MR.mp = types.SimpleNamespace(Pipe=lambda: (_Conn(), _Conn()), Process=_Proc)
    with open(os.path.join(REF, "config", "getting_started.yaml")) as f:
        cfg = sys.modules["munch"].munchify(yaml.safe_load(f))
    N = 2
    env = MR.MultiRaceAviary(race_config=cfg, num_drones=N, racemode=E.RaceMode.COMPARE)
    obs, info = env.reset()
    obs = np.asarray(obs, float)
    uc = types.ModuleType("user_controller")          # bypass the package __init__ (SB3 imports)
    uc.__path__ = [os.path.join(REF, "user_controller")]
    sys.modules["user_controller"] = uc
    uc.BaseController = importlib.import_module("user_controller.BaseController").BaseController
    HC = importlib.import_module("user_controller.HardCodedController").HardCodedController
    agents = []
    for i in range(N):
        inf = dict(info)
        inf["delay"] = i
        agents.append(HC(i, obs[i], inf))
    K = int(cfg.episode_len_sec * cfg.ctrl_freq)
    cmd = np.zeros((K, N), "<U3")
    flat = np.zeros((K, N, 14))
    nflat = np.zeros((K, N), np.int32)
    for k in range(K):
        t = k / cfg.ctrl_freq
        for i, a in enumerate(agents):
            c, args = a.predict(obs[i], ep_time=t)
            v = np.concatenate([np.atleast_1d(np.asarray(x, float)).reshape(-1) for x in args]) if args else np.zeros(0)
            cmd[k, i] = c.value
            flat[k, i, :v.size] = v
            nflat[k, i] = v.size
    return {"hc_obs0": obs, "hc_cmd": cmd, "hc_flat": flat, "hc_nflat": nflat,
            "hc_ref": np.stack([np.stack([a.ref_x, a.ref_y, a.ref_z], -1) for a in agents]),
            "hc_ctrl_freq": np.array(cfg.ctrl_freq)}


def logger_fixtures(pb, m):
    """utils/logger.py Logger.log / save array layout (states reordered, controls, timestamps),
    on scripted 20-d state vectors, for both the growing and the preallocated mode."""
    import tempfile
    L = importlib.import_module("gym_pybullet_adrp.utils.logger").Logger
    rng = np.random.default_rng(41)
    n, T = 3, 7
    st = rng.normal(size=(T, n, 20)); ct = rng.normal(size=(T, n, 12))
    out = {"log_state": st, "log_control": ct}
    for tag, dur in (("grow", 0), ("prealloc", 1)):
        with tempfile.TemporaryDirectory() as d:
            lg = L(logging_freq_hz=30, output_folder=os.path.join(d, "r"), num_drones=n, duration_sec=dur)
            for t in range(T):
                for j in range(n):
                    lg.log(drone=j, timestamp=t / 30, state=st[t, j], control=ct[t, j])
            out[f"log_{tag}_timestamps"] = lg.timestamps
            out[f"log_{tag}_states"] = lg.states
            out[f"log_{tag}_controls"] = lg.controls
    return out


def main():
    if os.environ.get("GOLDEN_ONLY") == "critic":   # weights only: no reference module is imported
        px = critic_fixtures()
        path = os.path.join(HERE, "critic_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    os.chdir(REF)   # MultiRaceAviary resolves URDF_DIR relative to the cwd (read only)
    pb = install_stubs()
    m = import_reference(pb)
    if os.environ.get("GOLDEN_ONLY") == "logger":
        px = logger_fixtures(pb, m)
        path = os.path.join(HERE, "logger_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    if os.environ.get("GOLDEN_ONLY") == "policy":
        px = policy_fixtures(pb, m)
        path = os.path.join(HERE, "policy_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    if os.environ.get("GOLDEN_ONLY") == "obswrap":
        px = obswrap_fixtures(pb, m)
        path = os.path.join(HERE, "obswrap_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    if os.environ.get("GOLDEN_ONLY") == "hardcoded":
        px = hardcoded_fixtures(pb, m)
        path = os.path.join(HERE, "hardcoded_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    if os.environ.get("GOLDEN_ONLY") == "pid":
        px = pid_fixtures(pb, m)
        path = os.path.join(HERE, "pid_golden.npz")
        np.savez_compressed(path, **px)
        print("wrote", path, len(px), "arrays")
        return
    fx = {}
    fx.update(hover_fixtures(pb, m))
    fx.update(force_fixtures(pb, m))
    fx.update(dyn_fixtures(pb, m))
    fx.update(mellinger_fixtures(pb, m))
    path = os.path.join(HERE, "hover_golden.npz")
    np.savez_compressed(path, **fx)
    print("wrote", path, len(fx), "arrays")
    rx = race_fixtures(pb, m)
    path = os.path.join(HERE, "race_golden.npz")
    np.savez_compressed(path, **rx)
    print("wrote", path, len(rx), "arrays")
    px = pid_fixtures(pb, m)
    path = os.path.join(HERE, "pid_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")
    px = policy_fixtures(pb, m)
    path = os.path.join(HERE, "policy_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")
    px = logger_fixtures(pb, m)
    path = os.path.join(HERE, "logger_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")
    px = obswrap_fixtures(pb, m)
    path = os.path.join(HERE, "obswrap_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")
    px = hardcoded_fixtures(pb, m)
    path = os.path.join(HERE, "hardcoded_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")
    px = critic_fixtures()
    path = os.path.join(HERE, "critic_golden.npz")
    np.savez_compressed(path, **px)
    print("wrote", path, len(px), "arrays")


if __name__ == "__main__":
    main()
