"""salp_math.h / salp_philox.h: accuracy, NumPy float32 trig restatement, Philox KAT.

CPU only (through the oracle library, which includes the same headers as the
device code); the device build is compared with these bit for bit in
tests/test_gpu_parity.py."""
import math

import mpmath
import numpy as np
import pytest

from oracle import oracle

mpmath.mp.prec = 120


def ulp_err(got, exact):
    exact = np.asarray(exact, np.float64)
    return np.abs(got - exact) / np.spacing(np.abs(exact).astype(np.float64))


@pytest.fixture(scope="module")
def sample():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-4, 4, 3000), rng.uniform(-0.8, 0.8, 2000),
                        rng.uniform(-1e-3, 1e-3, 500), rng.uniform(-60, 60, 500),
                        [0.0, 1.0, -1.0, 0.5, math.pi / 4, math.pi / 2]])
    y = rng.uniform(-3, 3, len(x))
    return x, y, oracle.math_selftest(x, y)


def test_sin_cos_tan_within_one_ulp(sample):
    x, _, out = sample
    for row, f in ((0, mpmath.sin), (1, mpmath.cos)):
        exact = np.array([float(f(mpmath.mpf(v))) for v in x])
        e = ulp_err(out[row], exact)
        assert np.max(e[np.abs(exact) > 1e-300]) <= 1.0
        # and it agrees with glibc (which NumPy uses for float64 sin/cos) nearly always
        glibc = np.array([math.sin(v) if row == 0 else math.cos(v) for v in x])
        assert np.mean(out[row] == glibc) > 0.95
    t = x[np.abs(x) < 1.2]
    exact = np.array([float(mpmath.tan(mpmath.mpf(v))) for v in t])
    got = oracle.math_selftest(t, t)[2]
    assert np.max(ulp_err(got, exact)) <= 2.0


def test_inverse_trig_within_two_ulp(sample):
    x, y, out = sample
    m = np.abs(x) <= 1
    ex = np.array([float(mpmath.asin(mpmath.mpf(v))) for v in x[m]])
    assert np.max(ulp_err(out[4][m], ex)) <= 2.0
    ex = np.array([float(mpmath.acos(mpmath.mpf(v))) for v in x[m]])
    assert np.max(ulp_err(out[5][m], ex)) <= 2.0
    ex = np.array([float(mpmath.atan2(mpmath.mpf(a), mpmath.mpf(b))) for a, b in zip(x, y)])
    assert np.max(ulp_err(out[3], ex)) <= 2.0
    # exact values the nozzle IK depends on (src/robot.py:79-93)
    z = oracle.math_selftest(np.array([1.0, -1.0]), np.array([1.0, 1.0]))
    assert z[5][0] == 0.0 and z[5][1] == math.pi and z[4][0] == math.pi / 2


def test_cube_correctly_rounded(sample):
    x, _, out = sample
    ex = np.array([float(mpmath.mpf(v) ** 3) for v in x])
    assert np.array_equal(out[6], ex)


def test_numpy_float32_sincos_restated_bit_for_bit():
    """NumPy's SIMD float32 cos/sin (used on the yaw, src/robot.py:76) is
    restated exactly, over the whole action range and beyond."""
    rng = np.random.default_rng(1)
    a2 = rng.uniform(-1, 1, 200000).astype(np.float32)
    yaw = (a2 * np.float32(np.pi / 2)).astype(np.float32)
    extra = rng.uniform(-40, 40, 20000).astype(np.float32)
    xs = np.concatenate([yaw, extra, np.float32([0, np.pi / 2, -np.pi / 2, 1e-8])])
    out = oracle.math_selftest(xs.astype(np.float64), np.zeros(len(xs)))
    assert np.array_equal(out[7].astype(np.float32), np.cos(xs))
    assert np.array_equal(out[8].astype(np.float32), np.sin(xs))


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors."""
    assert oracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert oracle.philox([0xffffffff] * 4, [0xffffffff] * 2) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6,
                                                                 0x6d5451fd]
    assert oracle.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_branch_free_sincos_equals_sincos():
    """sm_sincos_nb_p (every lane reduced, variant picked per lane) is
    bit-identical to sm_sincos, around the pi/4 switch, the quadrant edges,
    signed zeros and non-finite inputs included."""
    rng = np.random.default_rng(5)
    q = np.pi / 4
    edges = np.concatenate([[np.nextafter(q, 0), q, np.nextafter(q, 4)], np.arange(-8, 9) * (np.pi / 4)])
    x = np.concatenate([rng.uniform(-np.pi, np.pi, 200000), rng.uniform(-1e3, 1e3, 20000),
                        rng.uniform(-1e-6, 1e-6, 2000), edges, -edges,
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1e-300]])
    out = oracle.math_selftest(x, np.zeros(len(x)))
    for r_nb, r in ((9, 0), (10, 1)):
        assert np.array_equal(out[r_nb], out[r], equal_nan=True)
        assert np.array_equal(np.signbit(out[r_nb]), np.signbit(out[r]))
