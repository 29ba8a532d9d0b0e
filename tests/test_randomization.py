"""Randomisation features against samples of the
reference itself (tests/golden/randomization.npz, made by
make_randomization_golden.py).

The reference draws from NumPy's global MT19937, the oracle and the device
from Philox (grasp_lab_salp_amd/csrc/salp_random.h), so parity here is
distributional: two-sample Kolmogorov-Smirnov tests (p > 1e-3) plus the exact
properties the reference's arithmetic implies (bounds, the deterministic
(1 + u) scaling of negative observation entries, the doubled cycle counter
under latency).  Device == oracle bit for bit is tested in
tests/test_gpu_randomization.py.
"""
import os

import numpy as np
import pytest
from scipy.stats import ks_2samp

from grasp_lab_salp_amd._abi import FIELD, default_params
from oracle.oracle import Oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "randomization.npz")
P_MIN = 1e-3


@pytest.fixture(scope="module")
def ref():
    return np.load(GOLD)


def _oracle(n, seed=7, **flags):
    o = Oracle(default_params(), n, seed=seed)
    o.set_randomization(**flags)
    o.reset()
    return o


def _f(o, name):
    return o.state[FIELD[name]]


def test_coefficients_match_reference_distribution(ref):
    n = 4000
    o = _oracle(n, dynamics=True)
    ctl = np.tile([0.03, 2.0, 0.0, 0.0], (n, 1))
    o.robot_set_control(ctl, contraction_f32=False)
    assert np.all(_f(o, "rng_ctl") == 1)
    pairs = [("cd", ref["coef_cd"]), ("dfr", ref["coef_dfr"]), ("dtr", ref["coef_dtr"])]
    for j in range(3):
        for k in ("amf", "amrf", "amt", "amrt"):
            pairs.append((f"{k}{j}", ref["coef_" + k][:, j]))
    for name, r in pairs:
        got = _f(o, name)
        assert got.min() >= r.min() - 0.02 * abs(r.mean()) and got.max() <= r.max() + 0.02 * abs(r.mean()), name
        assert ks_2samp(got, r).pvalue > P_MIN, name
    # a second set_control draws fresh values
    before = _f(o, "cd").copy()
    o.robot_set_control(ctl, contraction_f32=False)
    assert np.mean(_f(o, "cd") == before) < 0.01
    # switched off: the means of src/robot.py:300-306
    o.set_randomization()
    o.robot_set_control(ctl, contraction_f32=False)
    assert np.all(_f(o, "cd") == 0.3) and np.all(_f(o, "amf0") == 0.5) and np.all(_f(o, "amt1") == 0.6)


def test_ou_disturbance_stationary_distribution(ref):
    n = 2000
    o = _oracle(n, disturbances=True)
    o.robot_set_control(np.tile([0.03, 5.0, 0.0, 0.0], (n, 1)), contraction_f32=False)
    ticks, _, _ = o.robot_cycle()
    assert ticks.min() >= int(ref["ou_steps"])
    assert np.all(_f(o, "rng_tick") == ticks)
    for name, r in (("ouf0", ref["ou_force"][:, 0]), ("ouf1", ref["ou_force"][:, 1]),
                    ("out2", ref["ou_torque"][:, 2])):
        got = _f(o, name)
        assert ks_2samp(got, r).pvalue > P_MIN, name
    # the zeroed components (force z, torque x/y) stay zero, as in the reference
    assert np.all(_f(o, "ouf2") == 0) and np.all(_f(o, "out0") == 0) and np.all(_f(o, "out1") == 0)
    assert np.all(ref["ou_force"][:, 2] == 0) and np.all(ref["ou_torque"][:, :2] == 0)
    # robot.reset() calms both processes (src/robot.py:454-455)
    o.robot_reset()
    assert np.all(_f(o, "ouf0") == 0) and np.all(_f(o, "out2") == 0)


@pytest.mark.parametrize("k", [0, 1])
def test_action_randomization_matches_reference(ref, k):
    n = 4000
    r_in = ref["act_in"][k].astype(np.float32)
    a = np.array([r_in[0] / np.float32(0.06), r_in[1] / np.float32(10.0), r_in[2] / np.float32(np.pi / 2)],
                 np.float32)
    o = _oracle(n, actions=True)
    o.step(np.tile(a, (n, 1)))
    resc = np.array([a[0] * np.float32(0.06), a[1] * np.float32(10.0), a[2] * np.float32(np.pi / 2)], np.float32)
    got = np.stack([_f(o, "contraction"), _f(o, "coast_time"), _f(o, "yaw")], 1)
    want = ref["act_out"][k]
    for j in range(3):
        rg, rw = got[:, j] / resc[j], want[:, j] / r_in[j]
        assert rg.min() >= 0.9 - 1e-6 and rg.max() <= 1.1 + 1e-6
        assert ks_2samp(rg, rw).pvalue > P_MIN, j
    # randomised actions are Python floats: float64 geometry from here on
    assert np.all(_f(o, "contr32") == 0)


def test_observation_randomization_matches_reference(ref):
    n = 4000
    a = np.tile(np.float32([0.6, 0.2, 0.4]), (n, 1))
    clean = _oracle(n).step(a)["obs"]
    noisy = _oracle(n, observations=True).step(a)["obs"]
    unc = np.array([0.05, 0.05, 0.2, 0.2, 0.02, 0.1])
    r_in, r_out = ref["obs_in"], ref["obs_out"]
    # entries 6.. untouched
    assert np.array_equal(noisy[:, 6:], clean[:, 6:])
    assert np.all(r_out[:, 6:] == r_in[6:])
    for j in range(6):
        pos = clean[:, j] > 0
        neg = clean[:, j] < 0
        # negative entries: always v * (1 + u) (the clip bounds are the sample
        # bounds in reverse order), in the reference too
        hi = clean[neg, j] * np.float32(1 + unc[j])
        assert np.array_equal(noisy[neg, j], hi)
        if r_in[j] < 0:
            assert np.all(r_out[:, j] == np.float32(r_in[j]) * np.float32(1 + unc[j]))
        if pos.sum() > 100 and r_in[j] > 0:
            zg = (noisy[pos, j].astype(np.float64) / clean[pos, j] - 1) / unc[j]
            zr = (r_out[:, j] / np.float64(r_in[j]) - 1) / unc[j]
            assert zg.min() >= -1 - 1e-5 and zg.max() <= 1 + 1e-5
            assert ks_2samp(zg, zr).pvalue > P_MIN, j


def test_latency_matches_reference(ref):
    n = 4000
    o = _oracle(n, latency=True)
    a = np.tile(np.float32([0.6, 0.2, 0.4]), (n, 1))
    o.step(a)
    assert np.all(_f(o, "cycle") == 2)            # the latency set_control counts a cycle
    assert np.all(_f(o, "contraction") == 0)
    lat = _f(o, "coast_time")
    assert lat.min() >= 0 and lat.max() <= 0.1
    assert ks_2samp(lat, ref["latency"]).pvalue > P_MIN
    o.step(a)
    assert np.all(_f(o, "cycle") == 4)


def test_all_switches_together_stay_finite():
    n = 256
    o = _oracle(n, dynamics=True, disturbances=True, actions=True, observations=True, latency=True)
    rng = np.random.default_rng(3)
    for _ in range(3):
        a = np.stack([rng.uniform(0.3, 1, n), rng.uniform(0, 1, n), rng.uniform(-1, 1, n)], 1).astype(np.float32)
        out = o.step(a, auto_reset=True)
    assert np.isfinite(out["obs"]).mean() > 0.95
