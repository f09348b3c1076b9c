"""The closed forms of tests/test_closed_form.py on the HIP kernels (fp32 and fp64), through the
C-ABI.  Needs an MI355X: -m gpu.  Tolerances: float32 rounding for the fp32 kernels (stated per
test), 1e-11 for the fp64 kernels."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd import _lib  # noqa: E402
from test_closed_form import (G, free_fall_reference, field, gyro_identity_residual, hover_cfg,  # noqa: E402
                              hover_rest_state, newton_reference, newton_state, race_cfg, set_fields,
                              spin_state, spin_z_reference)

TOL = {"fp32": 1e-5, "fp64": 1e-11}


class Dev:
    """one libadrp handle with its I/O buffers (float64 numpy state in / out)"""

    def __init__(self, cfg, precision):
        cfg = cfg.copy()
        cfg.precision = 1 if precision == "fp64" else 0
        self.h = _lib.Handle(cfg, 0)
        self.cfg = cfg
        E, N, D = cfg.num_envs, cfg.num_drones, self.h.D
        dev = self.h.device
        self.obs = torch.zeros((E, N, D), device=dev)
        self.rew = torch.zeros(E, device=dev)
        self.term = torch.zeros(E, dtype=torch.bool, device=dev)
        self.trunc = torch.zeros(E, dtype=torch.bool, device=dev)
        self.h.reset(self.obs)
        self.names = self.h.field_names()

    def get(self):
        f, i = self.h.get_state()
        return f.double().cpu().numpy(), i.cpu().numpy()

    def put(self, f, i):
        self.h.set_state(torch.from_numpy(f), torch.from_numpy(i))

    def step(self, act):
        self.h.step(torch.from_numpy(np.ascontiguousarray(act, np.float32)).to(self.h.device), self.obs, self.rew,
                    self.term, self.trunc)

    def close(self):
        self.h.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_hover_equilibrium(precision):
    E = 256
    d = Dev(hover_cfg(E), precision)
    f0, _ = set_fields(d.get, d.put, hover_rest_state(d.names, E))
    act = np.zeros((E, 1, 4), np.float32)
    for _ in range(100):
        d.step(act)
    f, _ = d.get()
    n = d.names[0]
    drift = np.abs(field(f, n, "pos_", "xyz") - field(f0, n, "pos_", "xyz")).max()
    # fp32: thrust - m g = O(1e-7 m g) rounding => drift <= 1/2 1e-6 m/s^2 (3.3 s)^2 ~ 5e-6 m
    assert drift < (1e-4 if precision == "fp32" else 1e-11), drift
    # the lever arms cancel exactly in the oracle's order; the kernels' FMA contraction leaves O(ulp)
    assert np.abs(field(f, n, "omega_", "xyz")).max() < (1e-6 if precision == "fp32" else 1e-12)
    d.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
@pytest.mark.parametrize("a", [0.6, -0.6])
def test_constant_thrust_vertical(precision, a):
    E = 128
    cfg = hover_cfg(E)
    d = Dev(cfg, precision)
    set_fields(d.get, d.put, hover_rest_state(d.names, E))
    dc = cfg.drone
    hover = np.sqrt(G * dc.m / (4 * dc.kf))
    rpm = hover * float(np.float32(1.0) + np.float32(0.05) * np.float32(a))
    thrust_acc = 4 * dc.kf * rpm * rpm / dc.m - G
    dt = 1.0 / cfg.pyb_freq
    z, vz = 1.0, 0.0
    act = np.full((E, 1, 4), a, np.float32)
    for _ in range(30):
        d.step(act)
        for _ in range(cfg.pyb_freq // cfg.ctrl_freq):
            vz = vz + dt * (thrust_acc - 0.04 * (1 + abs(vz)) * vz)
            z = z + dt * vz
    f, _ = d.get()
    np.testing.assert_allclose(f[d.names[0].index("pos_z")], z, rtol=TOL[precision])
    np.testing.assert_allclose(f[d.names[0].index("vel_z")], vz, rtol=10 * TOL[precision])
    d.close()


@pytest.mark.parametrize("spin", [False, True])
@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_free_fall(precision, spin):
    """race kernels, motors off (eliminated drones): the damped free fall; with spin the same
    recurrence holds (Newton: w does not turn v)"""
    E, N = 512, 2
    cfg = race_cfg(E)
    d = Dev(cfg, precision)
    rng = np.random.default_rng(0)
    p0 = np.stack([rng.uniform(-2.5, -2.0, E * N), rng.uniform(-2.5, -2.0, E * N), rng.uniform(8, 9, E * N)], 1)
    v0 = rng.uniform(-3, 3, (E * N, 3))
    if precision == "fp32":
        p0, v0 = p0.astype(np.float32).astype(float), v0.astype(np.float32).astype(float)
    vals = {"_names": d.names, "flags": np.ones(E * N, np.int32)}
    for k, ax in enumerate("xyz"):
        vals[f"pos_{ax}"], vals[f"vel_{ax}"], vals[f"omega_{ax}"] = p0[:, k], v0[:, k], np.zeros(E * N)
        if spin:
            vals[f"omega_{ax}"] = rng.uniform(-8, 8, E * N).astype(np.float32).astype(float)
    for m in range(4):
        vals[f"rpm_{m}"] = vals[f"prev_rpm_{m}"] = np.zeros(E * N)
    set_fields(d.get, d.put, vals)
    ref = free_fall_reference(p0, v0, 1.0 / cfg.pyb_freq, 10 * 20)
    act = np.zeros((E, N, 4), np.float32)
    for _ in range(10):
        d.step(act)
    f, _ = d.get()
    p, v = ref[-1]
    np.testing.assert_allclose(field(f, d.names[0], "pos_", "xyz"), p, rtol=TOL[precision], atol=TOL[precision])
    np.testing.assert_allclose(field(f, d.names[0], "vel_", "xyz"), v, rtol=10 * TOL[precision], atol=TOL[precision])
    d.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_torque_free_spin_z(precision):
    E = 128
    d = Dev(hover_cfg(E, gravity=0.0, pyb=240, ctrl=240), precision)
    w0 = np.linspace(-9, 9, E)
    if precision == "fp32":
        w0 = w0.astype(np.float32).astype(float)
    vals = hover_rest_state(d.names, E)
    vals["omega_z"] = vals["angv_z"] = w0
    set_fields(d.get, d.put, vals)
    ref = spin_z_reference(w0, 1.0 / 240, 300)
    act = np.zeros((E, 1, 4), np.float32)
    for _ in range(300):
        d.step(act)
    f, _ = d.get()
    w, th = ref[-1]
    np.testing.assert_allclose(f[d.names[0].index("omega_z")], w, rtol=TOL[precision])
    q = field(f, d.names[0], "quat_", "xyzw")
    want = np.stack([np.zeros(E), np.zeros(E), np.sin(th / 2), np.cos(th / 2)], 1)
    # fp32: 300 exp-map steps of float32 rounding in the angle
    np.testing.assert_allclose(q * np.sign(q[:, 3:4]), want * np.sign(want[:, 3:4]),
                               atol=3e-5 if precision == "fp32" else 1e-11)
    d.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_torque_free_spin_gyro(precision):
    E = 512
    cfg = hover_cfg(E, gravity=0.0, pyb=240, ctrl=240)
    d = Dev(cfg, precision)
    rng = np.random.default_rng(1)
    set_fields(d.get, d.put, spin_state(d.names, E, rng.uniform(-8, 8, (E, 3)), rng))
    dc = cfg.drone
    J = np.array([dc.ixx, dc.iyy, dc.izz])
    act = np.zeros((E, 1, 4), np.float32)
    worst = 0.0
    for _ in range(50):
        f0, _ = d.get()
        d.step(act)
        f1, _ = d.get()
        r = gyro_identity_residual(J, field(f0, d.names[0], "quat_", "xyzw"), field(f0, d.names[0], "omega_", "xyz"),
                                   field(f1, d.names[0], "omega_", "xyz"), 1.0 / 240)
        worst = max(worst, r.max())
    assert worst < (2e-5 if precision == "fp32" else 1e-11), worst
    d.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_quaternion_norm(precision):
    E = 1024
    d = Dev(hover_cfg(E, gravity=0.0, pyb=240, ctrl=240), precision)
    rng = np.random.default_rng(2)
    set_fields(d.get, d.put, spin_state(d.names, E, rng.uniform(-15, 15, (E, 3)), rng))
    act = np.zeros((E, 1, 4), np.float32)
    for _ in range(10000):
        d.step(act)
    q = field(d.get()[0], d.names[0], "quat_", "xyzw")
    assert np.abs(np.linalg.norm(q, axis=1) - 1).max() < (1e-6 if precision == "fp32" else 1e-14)
    d.close()


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_newton_first_law(precision):
    """no force, no gravity, spinning (|w| up to 14 rad/s) and translating: the kernels keep v on
    its damped straight line (the "+ w x v" reading of btMultiBody, pinned by this law)"""
    E = 512
    d = Dev(hover_cfg(E, gravity=0.0, pyb=240, ctrl=240), precision)
    rng = np.random.default_rng(8)
    vals, v0 = newton_state(d.names, E, rng)
    if precision == "fp32":
        for k in list(vals):
            if k != "_names":
                vals[k] = np.asarray(vals[k]).astype(np.float32).astype(float)
        v0 = v0.astype(np.float32).astype(float)
    f0, _ = set_fields(d.get, d.put, vals)
    n = d.names[0]
    ref = newton_reference(field(f0, n, "pos_", "xyz"), v0, 1.0 / 240, 240)
    act = np.zeros((E, 1, 4), np.float32)
    for _ in range(240):
        d.step(act)
    f, _ = d.get()
    p, v = ref[-1]
    vg = field(f, n, "vel_", "xyz")
    turn = np.linalg.norm(np.cross(vg, v0), axis=1) / (np.linalg.norm(vg, axis=1) * np.linalg.norm(v0, axis=1))
    # fp32: 240 sub-steps of float32 rounding in the damping products (~1e-7 each)
    assert turn.max() < (1e-5 if precision == "fp32" else 1e-12), turn.max()
    np.testing.assert_allclose(vg, v, rtol=TOL[precision], atol=TOL[precision])
    np.testing.assert_allclose(field(f, n, "pos_", "xyz"), p, rtol=TOL[precision], atol=TOL[precision])
    d.close()
