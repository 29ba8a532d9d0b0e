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


def _ulps(got, f, xs):
    exact = np.array([float(f(mpmath.mpf(v))) for v in xs])
    return ulp_err(got, exact), exact


def test_tick_yaw_sincos_within_one_ulp():
    """sm_sincos_yaw_p (the tick's yaw, product mode): one Cody-Waite stage and
    the kernels' tail forms; within one ulp over several turns, near every
    multiple of pi/4 and at the small angles where fdlibm skips the reduction."""
    rng = np.random.default_rng(3)
    k = rng.integers(-40, 40, 4000)
    x = np.concatenate([rng.uniform(-60, 60, 6000), rng.uniform(-0.8, 0.8, 2000), rng.uniform(-1e-3, 1e-3, 500),
                        k * (math.pi / 4) + rng.uniform(-1e-6, 1e-6, len(k)), [0.0, 1.0, -1.0, math.pi / 2]])
    out = oracle.math_selftest(x, np.zeros_like(x))
    # one Cody-Waite stage: within 1e-26 |fn| absolute, so one ulp unless the
    # result is within 1e-10 |fn| of zero (x = pi/2 itself: cos 6.1e-17)
    fn = np.maximum(np.abs(np.rint(x * 2 / math.pi)), 1.0)
    for row, f in ((12, mpmath.sin), (13, mpmath.cos)):
        e, exact = _ulps(out[row], f, x)
        assert np.max(np.abs(out[row] - exact) / fn) <= 1e-26 + 0.5 * np.spacing(1.0), row
        ok = np.abs(exact) > 1e-10 * fn
        assert np.max(e[ok]) <= 1.0, (row, float(np.max(e[ok])))
    # fdlibm's sincos agrees bit for bit nearly always
    assert np.mean(out[12] == out[0]) > 0.9 and np.mean(out[13] == out[1]) > 0.9
    nan = oracle.math_selftest(np.array([np.nan, np.inf, -np.inf]), np.zeros(3))
    assert np.isnan(nan[12]).all() and np.isnan(nan[13]).all()


def test_tick_yaw_sincos_large_angles():
    """sm_sincos_yaw_p past a few turns — the range tumbling envs' roll and
    pitch reach (up to 1e5 rad in the bench's steady state, a finite 3.9e11
    during one blow-up: profiles/r5am_angle_census.json).  What it
    guarantees, against mpmath at 300 bits:

    * |x| <= 2^20 pi/2 (fdlibm's medium range, |fn| < 2^20): within one ulp,
      except where the result is within 1e-10 |fn| of zero (the single
      Cody-Waite stage, as above);
    * |x| < 2^51 pi/2 (~3.5e15; the magic-add quadrant is exact for
      |fn| < 2^51): absolute error <= 1.5e-26 |fn| + one ulp of 1 (the fused
      first stage keeps fn * pio2_1 exact; what is left is pio2_1t's own
      truncation, |fn| * 2^-87);
    * beyond: unspecified — not sin / cos at all (|values| up to 1e176, NaN
      from ~1e100 rad), reached only by envs whose state is already
      diverging; device == oracle there still holds bit for bit (shared code,
      the GPU math self-test).  The reference's own pin up to 1e11 rad is
      tests/test_oracle_tumble.py."""
    rng = np.random.default_rng(11)
    med = 2.0 ** 20 * math.pi / 2
    big = 2.0 ** 51 * math.pi / 2
    k = rng.integers(1, 2 ** 20, 1500) * rng.choice([-1, 1], 1500)
    x1 = np.concatenate([10.0 ** rng.uniform(1.5, math.log10(med), 3000) * rng.choice([-1, 1], 3000),
                         k * (math.pi / 2) + rng.uniform(-1e-4, 1e-4, len(k))])
    x1 = x1[np.abs(x1) <= med]
    x2 = 10.0 ** rng.uniform(math.log10(med), math.log10(big) - 0.01, 3000) * rng.choice([-1, 1], 3000)
    with mpmath.workprec(300):
        for x, bound in ((x1, "ulp"), (x2, "abs")):
            out = oracle.math_selftest(x, np.zeros_like(x))
            fn = np.abs(np.rint(x * 2 / math.pi))
            for row, f in ((12, mpmath.sin), (13, mpmath.cos)):
                exact = np.array([float(f(mpmath.mpf(float(v)))) for v in x])
                err = np.abs(out[row] - exact)
                assert np.all(err <= 1.5e-26 * fn + np.spacing(1.0)), (row, bound, float(np.max(err)))
                if bound == "ulp":
                    ok = np.abs(exact) > 1e-10 * fn
                    e = ulp_err(out[row][ok], exact[ok])
                    assert np.max(e) <= 1.0, (row, float(np.max(e)))


def test_tick_roll_pitch_pair():
    """sm_sincos_rp2 (round 6): the yaw's one-stage function for roll and
    pitch at every size (rows 14-17 equal the yaw rows 12 / 13 of the same
    angle bit for bit), within one ulp of mpmath on the small angles that most
    ticks see; NaN in one angle leaves the other's sin / cos alone."""
    rng = np.random.default_rng(4)
    x = np.concatenate([rng.uniform(-0.0625, 0.0625, 4000), rng.uniform(-1e-6, 1e-6, 500), [0.0625, -0.0625, 0.0]])
    y = rng.uniform(-0.0625, 0.0625, len(x))
    out = oracle.math_selftest(x, y)
    for row, f, a in ((14, mpmath.sin, x), (15, mpmath.cos, x), (16, mpmath.sin, y), (17, mpmath.cos, y)):
        e, exact = _ulps(out[row], f, a)
        ok = np.abs(exact) > 1e-300
        assert np.max(e[ok]) <= 1.0, (row, float(np.max(e[ok])))
    # every size, tumbling angles of thousands of radians included: the yaw function for both
    xb = np.concatenate([x, rng.uniform(0.07, 2.0, 300), rng.uniform(-5e3, 5e3, 300)])
    yb = np.concatenate([y, rng.uniform(-0.05, 0.05, 300), rng.uniform(-0.05, 0.05, 300)])
    ob = oracle.math_selftest(xb, yb)
    assert np.array_equal(ob[14], ob[12]) and np.array_equal(ob[15], ob[13])
    oy = oracle.math_selftest(yb, xb)
    assert np.array_equal(ob[16], oy[12]) and np.array_equal(ob[17], oy[13])
    on = oracle.math_selftest(np.array([np.nan, 0.01]), np.array([0.01, np.nan]))
    ref = oracle.math_selftest(np.array([0.01]), np.array([0.0]))
    assert np.isnan(on[14][0]) and np.isnan(on[15][0]) and np.isnan(on[16][1]) and np.isnan(on[17][1])
    assert on[16][0] == ref[14][0] and on[17][0] == ref[15][0] and on[14][1] == ref[14][0]


def test_tick_world_frame_rotation():
    """sm_world_frame: Rz(psi) Ry(theta) Rx(phi) v applied as three plane
    rotations equals the matrix product to a few ulp of |v|."""
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.06, 0.06, 400)
    y = rng.uniform(-0.06, 0.06, 400)
    out = oracle.math_selftest(x, y)
    for j in range(0, 400, 7):
        phi, th, psi = (mpmath.mpf(float(x[j])), mpmath.mpf(float(y[j])), mpmath.mpf(float(x[j] + y[j])))
        Rx = mpmath.matrix([[1, 0, 0], [0, mpmath.cos(phi), -mpmath.sin(phi)], [0, mpmath.sin(phi), mpmath.cos(phi)]])
        Ry = mpmath.matrix([[mpmath.cos(th), 0, mpmath.sin(th)], [0, 1, 0], [-mpmath.sin(th), 0, mpmath.cos(th)]])
        Rz = mpmath.matrix([[mpmath.cos(psi), -mpmath.sin(psi), 0], [mpmath.sin(psi), mpmath.cos(psi), 0], [0, 0, 1]])
        v = mpmath.matrix([float(y[j]), float(x[j]), 1.0])
        want = Rz * Ry * Rx * v
        norm = float(mpmath.norm(v))
        for r in range(3):
            assert abs(out[18 + r][j] - float(want[r])) <= 4 * np.spacing(norm), (j, r)


def test_select_form_atan_equals_fdlibm_branches():
    """sm_atan (every range by selects, one division) equals fdlibm's branchy
    sm_atan_ref bit for bit: every range, its boundaries, tiny, huge, signed
    zeros, infinities and NaN."""
    rng = np.random.default_rng(6)
    edges = np.array([0.4375, 0.6875, 1.1875, 2.4375, 2.0 ** -27, 2.0 ** 66])
    near = np.concatenate([np.nextafter(edges, 0), edges, np.nextafter(edges, np.inf)])
    x = np.concatenate([rng.uniform(-4, 4, 20000), 10.0 ** rng.uniform(-320, 300, 20000),
                        -(10.0 ** rng.uniform(-320, 300, 5000)), near, -near,
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0]])
    out = oracle.math_selftest(x, np.ones_like(x))
    a, b = out[21], out[22]
    same = (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), x[~same][:5]
