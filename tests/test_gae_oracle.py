"""The GAE oracle (oracle/gae.py) against an independent scalar restatement
and hand-computed cases.  SB3 is not installed, so these pin the restatement
to SB3's published algorithm, not to SB3 itself ("parity unpinned")."""
import numpy as np

from oracle.gae import bootstrap_timeouts, compute_returns_and_advantage


def scalar_gae(rew, val, starts, last_val, dones, gamma, lam):
    """Per-env Python loop over np.float32 scalars (SB3 expression order)."""
    T, n = rew.shape
    f = np.float32
    adv = np.zeros((T, n), np.float32)
    for e in range(n):
        last = f(0.0)
        for t in reversed(range(T)):
            if t == T - 1:
                nnt = f(1.0) - f(dones[e])
                nv = f(last_val[e])
            else:
                nnt = f(1.0) - f(starts[t + 1, e])
                nv = f(val[t + 1, e])
            delta = (f(rew[t, e]) + (f(gamma) * nv) * nnt) - f(val[t, e])
            last = delta + (f(gamma * lam) * nnt) * last
            adv[t, e] = last
    return adv, adv + val


def test_oracle_equals_scalar_restatement():
    rng = np.random.default_rng(0)
    for T, n in ((1, 3), (5, 7), (33, 17)):
        rew = rng.normal(size=(T, n)).astype(np.float32) * 50
        val = rng.normal(size=(T, n)).astype(np.float32) * 10
        starts = (rng.random((T, n)) < 0.2).astype(np.float32)
        lv = rng.normal(size=n).astype(np.float32)
        dn = rng.random(n) < 0.3
        a, r = compute_returns_and_advantage(rew, val, starts, lv, dn)
        a2, r2 = scalar_gae(rew, val, starts, lv, dn, 0.99, 0.95)
        assert np.array_equal(a, a2) and np.array_equal(r, r2)


def test_hand_computed_two_steps():
    # one env, no episode boundary: A1 = r1 + g*V_last - V1 ; A0 = r0 + g*V1 - V0 + g*l*A1
    rew = np.array([[1.0], [2.0]], np.float32)
    val = np.array([[0.5], [0.25]], np.float32)
    a, r = compute_returns_and_advantage(rew, val, np.zeros((2, 1), np.float32), np.array([4.0], np.float32),
                                         np.array([False]))
    a1 = 2.0 + 0.99 * 4.0 - 0.25
    a0 = 1.0 + 0.99 * 0.25 - 0.5 + 0.99 * 0.95 * a1
    assert np.allclose(a[:, 0], [a0, a1], rtol=1e-6)
    assert np.allclose(r, a + val)
    # episode start at step 1 cuts the bootstrap from step 0; done cuts the last value
    a, _ = compute_returns_and_advantage(rew, val, np.array([[1.0], [1.0]], np.float32),
                                         np.array([4.0], np.float32), np.array([True]))
    assert np.allclose(a[:, 0], [1.0 - 0.5, 2.0 - 0.25])


def test_timeout_bootstrap_only_for_truncation():
    r = bootstrap_timeouts([1.0, 1.0, 1.0], truncated=[True, True, False], terminated=[False, True, False],
                           terminal_values=[10.0, 10.0, 10.0])
    assert r.dtype == np.float32
    assert np.array_equal(r, np.array([1.0 + np.float32(0.99) * np.float32(10.0), 1.0, 1.0], np.float32))
