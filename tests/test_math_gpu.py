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
