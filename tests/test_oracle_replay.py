"""The oracle's sampled replay (oracle_replay, the checker of the bench-horizon
parity test and of bench.py's parity_sampled) against the oracle's own
step-by-step API: same env-steps (src/salp_robot_env.py:196-299), any
per-env step count, arbitrary global ids, the rollout-buffer ring, and the
in-flight cycle a chained launch leaves pending (src/robot.py:740-777)."""
import numpy as np

from grasp_lab_salp_amd._abi import FIELD, default_params
from oracle import oracle as orc
from oracle.sampled import _bits_differ, check
from test_gpu_parity import philox_action

SEED = 5


def _stepped(n, steps, offset=0):
    """Oracle(n) reset, then `steps` Philox-action env-steps with auto-reset;
    states after every step and the per-step outputs."""
    o = orc.Oracle(default_params(), n, seed=SEED, env_offset=offset)
    obs = o.reset()
    states, outs, acts, befores = [o.state.copy()], [], [], []
    for _ in range(steps):
        sc = o.state[FIELD["step_count"]]
        a = np.stack([philox_action(SEED, offset + i, int(sc[i])) for i in range(n)])
        befores.append(obs)
        r = o.step(a, auto_reset=True)
        obs = r["obs"]
        outs.append(r)
        acts.append(a)
        states.append(o.state.copy())
    return states, outs, acts, befores


def test_replay_equals_step_random_with_uniform_steps():
    n, k = 48, 9
    o = orc.Oracle(default_params(), n, seed=SEED, env_offset=1000)
    o.reset()
    o.step_random(k, threads=2)
    st, _ = orc.replay(np.arange(n) + 1000, np.full(n, k), seed=SEED, threads=2)
    assert not _bits_differ(st, o.state).any()


def test_replay_per_env_steps_and_buffer_ring():
    n, steps, cap = 24, 11, 4
    states, outs, acts, befores = _stepped(n, steps)
    ks = np.arange(n) % (steps + 1)
    st, buf = orc.replay(np.arange(n), ks, seed=SEED, capacity=cap, threads=2)
    for i, k in enumerate(ks):
        assert not _bits_differ(st[:, i], states[k][:, i]).any(), (i, k)
        for t in range(max(0, k - cap), k):
            s = t % cap
            assert np.array_equal(buf["obs"][s, i], outs[t]["terminal_obs"][i], equal_nan=True)
            assert np.array_equal(buf["obs_before"][s, i], befores[t][i], equal_nan=True)
            assert np.array_equal(buf["actions"][s, i], acts[t][i])
            assert np.array_equal(buf["rewards"][s, i], np.float32(outs[t]["reward"][i]), equal_nan=True)
            assert buf["dones"][s, i] == (outs[t]["terminated"][i] | (outs[t]["truncated"][i] << 1))


def test_replay_in_flight_cycle():
    """ct_stop: the next env-step is begun and its cycle ticked up to that
    cycle_time; pending is set.  ct_stop past the cycle's end runs it whole
    (kinematics then equal the finished step's when no reset follows)."""
    n, k = 32, 3
    full, _ = orc.replay(np.arange(n), np.full(n, k + 1), seed=SEED)
    st, _ = orc.replay(np.arange(n), np.full(n, k), ct_stop=np.full(n, 1e9), seed=SEED)
    assert (st[FIELD["pending"]] == 1.0).all()
    kin = slice(FIELD["v0"], FIELD["ang2"] + 1)
    no_reset = full[FIELD["episode"]] == st[FIELD["episode"]]
    assert no_reset.sum() > n // 2
    assert not _bits_differ(st[kin][:, no_reset], full[kin][:, no_reset]).any()
    part, _ = orc.replay(np.arange(n), np.full(n, k), ct_stop=np.full(n, 0.5), seed=SEED)
    ct = part[FIELD["cycle_time"]]
    total = st[FIELD["cycle_time"]]
    assert ((ct >= 0.5) | (ct == total)).all() and (ct < 0.5 + 0.0100001).all()
    zero, _ = orc.replay(np.arange(n), np.full(n, k), ct_stop=np.zeros(n), seed=SEED)
    assert (zero[FIELD["cycle_time"]] == 0.0).all() and (zero[FIELD["pending"]] == 1.0).all()


def test_check_flags_a_mismatch():
    """The checker itself: a replayed state passes, a one-ulp change fails."""
    n = 40
    ks = np.arange(n) % 5
    st, _ = orc.replay(np.arange(n), ks, seed=SEED)
    res = check(st, ks, None, default_params(), SEED, ids=np.arange(n), threads=2)
    assert res["ok"] and res["envs_checked"] == n
    st2 = st.copy()
    st2[FIELD["v0"], 7] = np.nextafter(st2[FIELD["v0"], 7], 1.0)
    res = check(st2, ks, None, default_params(), SEED, ids=np.arange(n), threads=2)
    assert not res["ok"] and res["state_mismatch_envs"] == 1
