"""The fp64 fast transcendentals the fp64 step kernels inline (csrc/adrp_device.h namespace f64:
refined v_rcp_f64 / v_rsq_f64 / Goldschmidt sqrt, range-reduced polynomials fitted by
tools/fit_f64_poly.py) against numpy longdouble references (64-bit mantissa), through
adrp_math_probe.  Bar: 4 ulp relative (2^-50 ~ 8.9e-16) on the ranges the kernels use, 4e-16
absolute near zero crossings of atan2 / asin.  Needs an MI355X: -m gpu."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from gym_pybullet_adrp_amd import _lib  # noqa: E402
from gym_pybullet_adrp_amd.utils import abi  # noqa: E402

L = np.longdouble
ULP4 = 2.0 ** -50


def probe(fn, x, x2=None):
    lib = _lib.load()
    inp = np.ascontiguousarray(x, np.float64) if x2 is None else np.concatenate([x, x2]).astype(np.float64)
    n = len(x)
    d_in = torch.from_numpy(inp).cuda()
    d_out = torch.empty(n, dtype=torch.float64, device="cuda")
    rc = lib.adrp_math_probe(fn, ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(d_out.data_ptr()), n,
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def rel_err(got, ref, floor=0.0):
    ref = np.asarray(ref, L)
    return np.abs(got.astype(L) - ref) / np.maximum(np.abs(ref), L(floor))


def test_constants_mirrored():
    assert (abi.MATH_RCP, abi.MATH_EXP, abi.MATH_COS_TINY) == (0, 7, 12)


def test_rcp_rsq_sqrt():
    rng = np.random.default_rng(0)
    x = np.concatenate([10.0 ** rng.uniform(-12, 12, 200000), [1.0, 2.0, 3.0, 0.1, 1e-300, 1e300]])
    assert rel_err(probe(abi.MATH_RCP, x), 1 / x.astype(L)).max() < ULP4
    assert rel_err(probe(abi.MATH_RSQ, x), 1 / np.sqrt(x.astype(L))).max() < ULP4
    assert rel_err(probe(abi.MATH_SQRT, x), np.sqrt(x.astype(L))).max() < ULP4
    z = probe(abi.MATH_SQRT, np.array([0.0, -0.0, -1.0]))
    assert z[0] == 0.0 and np.isnan(z[2])
    assert np.isinf(probe(abi.MATH_RCP, np.array([0.0]))[0])


def test_chain_variants():
    """The Bullet-step forms: sqrt of sums of squares (0 -> 0, NaN -> NaN, bit-identical to sqrt
    above 1e-300) and rcp / rsq without the non-finite fix-up (bit-identical to the checked forms on
    finite non-zero arguments)."""
    rng = np.random.default_rng(1)
    x = np.concatenate([10.0 ** rng.uniform(-12, 12, 200000), [1.0, 2.0, 3.0, 0.1, 1e-300, 1e300]])
    np.testing.assert_array_equal(probe(abi.MATH_SQRT_NN, x), probe(abi.MATH_SQRT, x))
    np.testing.assert_array_equal(probe(abi.MATH_RCP_NC, x), probe(abi.MATH_RCP, x))
    np.testing.assert_array_equal(probe(abi.MATH_RSQ_NC, x), probe(abi.MATH_RSQ, x))
    z = probe(abi.MATH_SQRT_NN, np.array([0.0, np.nan]))
    assert z[0] == 0.0 and np.isnan(z[1])


def test_sincos_tiny():
    """The short exp-map series on |x| <= 0.03 (taken when the whole wave is there)."""
    x = np.concatenate([np.linspace(-0.03, 0.03, 100001), [1e-300, -1e-12, 0.0]])
    xs = x[x != 0]
    assert rel_err(probe(abi.MATH_SIN_TINY, xs), np.sin(xs.astype(L))).max() < ULP4
    assert rel_err(probe(abi.MATH_COS_TINY, x), np.cos(x.astype(L))).max() < ULP4


def test_sincos_small():
    x = np.linspace(-np.pi / 8, np.pi / 8, 300001)
    x = x[x != 0]
    assert rel_err(probe(abi.MATH_SIN_SMALL, x), np.sin(x.astype(L))).max() < ULP4
    assert rel_err(probe(abi.MATH_COS_SMALL, x), np.cos(x.astype(L))).max() < ULP4


def test_atan2_asin():
    rng = np.random.default_rng(1)
    y = np.concatenate([rng.normal(size=200000) * 10.0 ** rng.uniform(-3, 3, 200000), [0.0, 1.0, -1.0, 1.0, 0.0]])
    x = np.concatenate([rng.normal(size=200000) * 10.0 ** rng.uniform(-3, 3, 200000), [1.0, 0.0, 0.0, 1.0, -1.0]])
    got = probe(abi.MATH_ATAN2, y, x)
    assert rel_err(got, np.arctan2(y.astype(L), x.astype(L)), floor=0.5).max() < ULP4
    s = np.concatenate([rng.uniform(-0.99999, 0.99999, 200000), [0.0, 0.5, -0.5]])
    assert rel_err(probe(abi.MATH_ASIN, s), np.arcsin(s.astype(L)), floor=0.5).max() < ULP4


def test_exp():
    x = np.concatenate([-np.linspace(0, 40, 200001), [-700.0, -745.5, -1e4]])
    got = probe(abi.MATH_EXP, x)
    ref = np.exp(x.astype(L))
    ok = ref > L(1e-300)
    assert rel_err(got[ok], ref[ok]).max() < ULP4
    assert got[-1] == 0.0


def test_exp_table_form():
    """the race downwash's exp (2^(j/32) table + degree-6 Taylor on |r| <= ln2/64): the same 4-ulp bar
    as exp() on x <= 0, underflow to 0 below the clamp"""
    rng = np.random.default_rng(5)
    x = np.concatenate([-np.linspace(0, 40, 200001), -rng.exponential(3.0, 200000), [-700.0, -745.5, -1e4, -0.0]])
    got = probe(abi.MATH_EXP_TAB, x)
    ref = np.exp(x.astype(L))
    ok = ref > L(1e-300)
    assert rel_err(got[ok], ref[ok]).max() < ULP4
    assert got[-2] == 0.0 and got[-1] == 1.0


def test_atan2_finite_form_matches():
    """the race Euler angles' atan2 without the non-finite fix-ups: bit-identical to atan2 on finite
    operands (zeros included)"""
    rng = np.random.default_rng(6)
    y = np.concatenate([rng.normal(size=200000) * 10.0 ** rng.uniform(-3, 3, 200000), [0.0, 1.0, -1.0, 0.0, -0.0]])
    x = np.concatenate([rng.normal(size=200000) * 10.0 ** rng.uniform(-3, 3, 200000), [1.0, 0.0, 0.0, 0.0, -1.0]])
    np.testing.assert_array_equal(probe(abi.MATH_ATAN2_NC, y, x), probe(abi.MATH_ATAN2, y, x))


def test_non_finite_inputs():
    """NaN in -> NaN out for atan2 (fmax / fmin drop a NaN), sqrt(+inf) = +inf"""
    nan, inf = np.nan, np.inf
    got = probe(abi.MATH_ATAN2, np.array([nan, 1.0, nan, 0.0]), np.array([nan, nan, 1.0, nan]))
    assert np.isnan(got).all()
    got = probe(abi.MATH_ASIN, np.array([nan]))
    assert np.isnan(got).all()
    s = probe(abi.MATH_SQRT, np.array([inf, 0.0, -0.0, 4.0, -1.0, nan]))
    assert s[0] == inf and s[1] == 0.0 and s[3] == 2.0 and np.isnan(s[4]) and np.isnan(s[5])
    assert np.signbit(s[2])


@pytest.mark.parametrize("fn", ["sinc", "cos", "norm"])
def test_exp_map_forms_are_per_lane(fn):
    """the hover fp64 exp map picks the short series (|x| <= 0.03) and the Newton norm
    (|n2 - 1| <= 1e-9) per lane.  A lane's result must not depend on its 63 wave neighbours: the same
    inputs probed in a wave of like lanes and in waves mixed with lanes that take the other form give
    bit-identical results, and each form is accurate on its own range."""
    rng = np.random.default_rng(5)
    if fn == "norm":
        fid = abi.MATH_QUAT_INV_NORM
        near = 1.0 + rng.uniform(-1e-9, 1e-9, 64 * 64)
        far = 1.0 + rng.uniform(-1e-3, 1e-3, 64 * 64)
        far = far[np.abs(far - 1) > 1e-9]
        ref = lambda v: 1 / np.sqrt(v.astype(L))
        tol = ULP4
    else:
        fid = abi.MATH_EXPMAP_SINC if fn == "sinc" else abi.MATH_EXPMAP_COS
        near = rng.uniform(-0.03, 0.03, 64 * 64)
        far = rng.uniform(0.031, np.pi / 8, 64 * 64) * rng.choice([-1, 1], 64 * 64)
        ref = (lambda v: np.sin(v.astype(L)) / v.astype(L)) if fn == "sinc" else (lambda v: np.cos(v.astype(L)))
        tol = ULP4
    alone_near, alone_far = probe(fid, near), probe(fid, far[:len(near)])
    mixed = np.empty(2 * len(near))
    mixed[0::2], mixed[1::2] = near, far[:len(near)]      # every wave holds both forms
    got = probe(fid, mixed)
    np.testing.assert_array_equal(got[0::2], alone_near)
    np.testing.assert_array_equal(got[1::2], alone_far)
    assert rel_err(alone_near, ref(near)).max() < tol
    assert rel_err(alone_far, ref(far[:len(near)])).max() < tol


def test_race_noise_box_muller_matches_oracle():
    """the fp64 race kernels' action noise (normal_pair_f, IEEE float operations only) is the
    oracle's (oracle/race.c normal_pair_f) bit for bit on the same Philox words; both are within 2
    float ulp of the float64 libm Box-Muller"""
    from oracle import oracle as O
    rng = np.random.default_rng(11)
    w = rng.integers(0, 2 ** 32, (4096, 2), dtype=np.uint64)
    w = np.concatenate([w, np.array([[0xFFFFFFFF, 0], [0, 0xFFFFFFFF], [0, 0x80000000], [0x100, 0x1234567]], np.uint64)])
    bits = (w[:, 1] << np.uint64(32)) | w[:, 0]
    x = bits.view(np.float64)
    z0, z1 = probe(abi.MATH_NORMAL_Z0, x), probe(abi.MATH_NORMAL_Z1, x)
    ref = np.array([O.normal_pair(a, b) for a, b in w], np.float64)
    np.testing.assert_array_equal(z0, ref[:, 0])
    np.testing.assert_array_equal(z1, ref[:, 1])
    u1 = ((w[:, 0] >> np.uint64(8)).astype(np.float64) + 1) / 2 ** 24
    u2 = (w[:, 1] >> np.uint64(8)).astype(np.float64) / 2 ** 24
    r = np.sqrt(-2 * np.log(u1))
    assert (np.abs(z0 - r * np.cos(2 * np.pi * u2)) <= 2.5e-7 * np.maximum(r, 1e-30) + 1e-30).all()
    assert (np.abs(z1 - r * np.sin(2 * np.pi * u2)) <= 2.5e-7 * np.maximum(r, 1e-30) + 1e-30).all()


@pytest.mark.parametrize("c", [0.002, 9.8, 65535.0, 3.0, 3.16e-10, 0.2685])
def test_constant_divisor_division_is_ieee(c):
    """f64::div_c (the fp64 kernels' x / c for the wrapper's constant divisors: numpy's rates / 0.002,
    acc / 0.002 / 9.8, _compute_pwms / 65535 / 3, _thr2pwm / 3.16e-10 / 0.2685) equals the IEEE
    quotient bit for bit, signed zeros included, over 10^6 random x across 2^-60 .. 2^60"""
    rng = np.random.default_rng(int(c * 1000) % 2 ** 31)
    x = np.ldexp(1 + rng.random(1_000_000), rng.integers(-60, 61, 1_000_000)) * rng.choice([-1.0, 1.0], 1_000_000)
    x = np.concatenate([x, [0.0, -0.0, 1.0, -1.0, c, 3 * c]])
    got = probe(abi.MATH_DIVC, x, np.full_like(x, c))
    want = x / c
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


def test_sincos_fast():
    """f64::sincos_fast (gate / part yaws and reset attitudes of the fp64 race kernels): within 2 ulp
    of the correctly rounded sin / cos on |x| <= 100 (relative; absolute 2^-52 near zero crossings),
    octant boundaries and signed zeros included"""
    rng = np.random.default_rng(19)
    x = np.concatenate([rng.uniform(-100, 100, 400000), rng.uniform(-4, 4, 200000),
                        np.arange(-40, 41) * np.pi / 8, [0.0, -0.0, 1e-300, np.pi, -np.pi, 0.5 * np.pi]])
    s, c = probe(abi.MATH_SIN_FAST, x), probe(abi.MATH_COS_FAST, x)
    xl = x.astype(L)
    for got, ref in ((s, np.sin(xl)), (c, np.cos(xl))):
        err = np.abs(got.astype(L) - ref)
        assert (err <= np.maximum(np.abs(ref) * L(2.0 ** -51), L(2.0 ** -52))).all(), float(err.max())
    assert s[-6] == 0.0 and c[-6] == 1.0


def test_fdiv_rcp_is_ieee_float_division():
    """f64::fdiv_rcp (the fp64 race firmware's float divisions, race_kernel.h mellinger_fw): rounding
    x * rcp(y) to float is the IEEE float x / y bit for bit.  4M quotients: random bit patterns over
    the whole normal range (both signs), quotients near float rounding boundaries (y a float just off
    a power of two, x with all-ones / alternating significands), the firmware's own scales (norms of
    target / y_des vectors, D terms by dt = 0.002f)"""
    rng = np.random.default_rng(23)
    n = 1 << 20

    def rand_f32(k, lo_exp=-60, hi_exp=60):
        m = rng.integers(0, 1 << 23, k, dtype=np.uint32)
        e = rng.integers(127 + lo_exp, 127 + hi_exp, k).astype(np.uint32)
        s = rng.integers(0, 2, k, dtype=np.uint32) << 31
        return (s | (e << 23) | m).view(np.float32)
    xs = [rand_f32(n), rand_f32(n, -3, 3), rng.uniform(-3, 3, n).astype(np.float32)]
    ys = [rand_f32(n), rand_f32(n, -3, 3), rng.uniform(0.05, 3, n).astype(np.float32)]
    # adversarial: y = 2^k (1 + j ulp) with small j, x with long runs of ones in the significand
    j = rng.integers(1, 64, n).astype(np.uint32)
    y_adv = ((np.uint32(127) << 23) + j).view(np.float32) * np.float32(2.0) ** rng.integers(-4, 4, n).astype(np.float32)
    x_adv = ((np.uint32(127) << 23) | (np.uint32((1 << 23) - 1) ^ rng.integers(0, 8, n, dtype=np.uint32))).view(np.float32)
    xs.append(x_adv)
    ys.append(y_adv)
    xs.append(rng.uniform(-50, 50, n).astype(np.float32))
    ys.append(np.full(n, np.float32(1.0) / np.float32(500), np.float32))
    for x, y in zip(xs, ys):
        got = probe(abi.MATH_FDIV_RCP, x.astype(np.float64), y.astype(np.float64)).astype(np.float32)
        ref = x / y
        bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
        assert len(bad) == 0, f"{len(bad)} quotients differ, e.g. {x[bad[:4]]} / {y[bad[:4]]}: {got[bad[:4]]} vs {ref[bad[:4]]}"
