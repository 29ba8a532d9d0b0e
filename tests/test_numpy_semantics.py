"""Pin the NumPy 2.2 / OpenBLAS arithmetic the reference's hot path goes
through, as probed in this image.  The oracle and the device kernel restate
exactly these evaluation orders (grasp_lab_salp_amd/csrc/salp_math.h); if an
image update changes them, these tests say so before the golden comparison
degrades."""
import math
from fractions import Fraction

import numpy as np
import pytest


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(7)


def test_norm_is_forward_fma_chain(rng):
    """np.linalg.norm (src/dynamics.py:113,122; src/salp_robot_env.py:242,352)."""
    for v in rng.normal(size=(400, 3)) * rng.uniform(1e-6, 10, (400, 1)):
        assert np.linalg.norm(v) == math.sqrt(fma(v[2], v[2], fma(v[1], v[1], v[0] * v[0])))
        assert np.linalg.norm(v[:2]) == math.sqrt(fma(v[1], v[1], v[0] * v[0]))


def test_matmul_orders(rng):
    """3x3 @ 3x3 (rotation / mass products), contiguous and transposed mat-vec."""
    for _ in range(200):
        A, B, v = rng.normal(size=(3, 3)), rng.normal(size=(3, 3)), rng.normal(size=3)
        C = A @ B
        for i in range(3):
            for j in range(3):
                assert C[i, j] == fma(A[i, 2], B[2, j], fma(A[i, 1], B[1, j], A[i, 0] * B[0, j]))
        r = A @ v
        t = A.T @ v
        for i in range(3):
            assert r[i] == fma(A[i, 2], v[2], fma(A[i, 0], v[0], A[i, 1] * v[1]))
            assert t[i] == fma(A[2, i], v[2], fma(A[1, i], v[1], A[0, i] * v[0]))


def test_solve_diag_is_division(rng):
    """np.linalg.solve with the diagonal mass / inertia (src/dynamics.py:10,17)."""
    for _ in range(300):
        d, b = rng.uniform(0.01, 5, 3), rng.normal(size=3)
        assert np.array_equal(np.linalg.solve(np.diag(d), b), b / d)


def test_cross_is_plain(rng):
    for _ in range(300):
        a, b = rng.normal(size=3), rng.normal(size=3)
        c = np.cross(a, b)
        assert c[0] == a[1] * b[2] - a[2] * b[1]
        assert c[1] == a[2] * b[0] - a[0] * b[2]
        assert c[2] == a[0] * b[1] - a[1] * b[0]


def test_nep50_float32_promotion():
    """NumPy 2 (NEP 50): the float32 contraction makes `init_length - contraction`
    float32 (src/geometry.py:46,53,60), float32 ** 2 float32, and float32 with a
    float64 NumPy scalar float64 — the dtype flow the oracle/kernel restate."""
    c = np.float32(0.0417)
    assert isinstance(0.3 - c, np.float32)
    assert (0.3 - c) == np.float32(np.float32(0.3) - c)
    assert isinstance(c ** 2, np.float32)
    assert isinstance(np.float64(2.0) * c, np.float64)
    assert isinstance(c / np.float64(2.3), np.float64)
    assert np.array([np.float32(1), 0.0]).dtype == np.float64
    assert np.array([np.float32(1), np.float32(2)]).dtype == np.float32
    a = np.float32(0.25)
    r = np.zeros_like(np.float32([1, 1, 1]))
    r[0] = a * 0.06
    assert r[0] == np.float32(a * np.float32(0.06))


def test_polyfit_coefficients():
    """src/geometry.py:6-25 fits, exactly as the kernel's constants."""
    c = np.polyfit(np.array([0.01, 0.02, 0.03, 0.04]), np.array([0.4, 1.0, 1.8, 2.2]), 2)
    assert [x.hex() for x in c] == ['-0x1.f3ffffffffffcp+8', '0x1.5bffffffffffcp+6', '-0x1.ccccccccccccbp-2']
    c = np.polyfit(np.array([0.01, 0.02, 0.03, 0.04]), np.array([0.1, 0.3, 0.4, 0.5]), 2)
    assert [x.hex() for x in c] == ['-0x1.f400000000001p+7', '0x1.97ffffffffffep+4', '-0x1.0000000000003p-3']
    assert math.cos(math.pi / 4).hex() == '0x1.6a09e667f3bcdp-1'
    assert math.sin(math.pi / 4).hex() == '0x1.6a09e667f3bccp-1'
