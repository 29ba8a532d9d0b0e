"""Randomised kernels (RAND instantiations) against the oracle, bit for bit.

Device and oracle draw from the same Philox streams (salp_random.h), so with
every switch on — dynamics randomisation, OU disturbances, action and
observation noise, latency — their states, observations and rewards must be
identical.  Distributional parity with the reference is tests/test_randomization.py.
"""
import numpy as np
import pytest
import torch

from grasp_lab_salp_amd._abi import FIELD, default_params
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
from oracle import oracle as orc
from test_gpu_parity import _cpu, assert_state_equal, random_actions

pytestmark = pytest.mark.gpu

ALL = dict(dynamics=True, disturbances=True, actions=True, observations=True, latency=True)


def make_pair(n, seed, **flags):
    p = default_params()
    env = BatchedSalpEnv(n, params=p, seed=seed)
    env.set_randomization(**flags)
    o = orc.Oracle(p, n, seed=seed)
    o.set_randomization(**flags)
    o.reset()
    return env, o


@pytest.mark.parametrize("flags", [ALL, dict(disturbances=True), dict(dynamics=True, latency=True),
                                   dict(actions=True, observations=True)])
def test_env_steps_with_randomization_equal_oracle(flags):
    n = 1024
    rng = np.random.default_rng(4)
    env, o = make_pair(n, 13, **flags)
    for t in range(5):
        a = random_actions(rng, n)
        r = env.step(torch.tensor(a), auto_reset=True)
        ro = o.step(a, auto_reset=True)
        assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True), t
        assert np.array_equal(_cpu(r.terminal_obs), ro["terminal_obs"], equal_nan=True), t
        assert np.array_equal(_cpu(r.reward), ro["reward"], equal_nan=True), t
        assert np.array_equal(_cpu(r.info), ro["info"], equal_nan=True), t
        assert_state_equal(env.get_state(), o.state, f"{flags} step {t}")
    g = _cpu(env.get_state())
    if flags.get("disturbances"):
        assert np.all(g[FIELD["rng_tick"]] > 0) and np.any(g[FIELD["ouf0"]] != 0)
    if flags.get("dynamics"):
        assert np.unique(g[FIELD["cd"]]).size > n // 2


def test_step_random_and_rollout_with_randomization_equal_oracle():
    n, steps = 512, 4
    env, o = make_pair(n, 17, **ALL)
    rs = env.step_random(steps)
    rs_o, _ = o.step_random(steps)
    assert np.array_equal(_cpu(rs), rs_o, equal_nan=True)
    assert_state_equal(env.get_state(), o.state, "step_random RAND")
    # chained rollout cut into small launches == the same work in one launch
    a = BatchedSalpEnv(n, params=default_params(), seed=23)
    b = BatchedSalpEnv(n, params=default_params(), seed=23)
    for e in (a, b):
        e.set_randomization(**ALL)
    sa = torch.zeros(n, dtype=torch.int64, device="cuda")
    sb = torch.zeros(n, dtype=torch.int64, device="cuda")
    a.rollout(10**7, steps_done=sa, max_steps=steps)
    for _ in range(200):
        b.rollout(61, steps_done=sb, max_steps=steps, chunk=16)
        if int(sb.min()) >= steps:
            break
    assert int(sa.min()) == steps and int(sb.min()) == steps
    assert np.array_equal(_cpu(a.get_state()), _cpu(b.get_state()), equal_nan=True)
    # and equal to the lock-step oracle driven with the same Philox actions
    from test_gpu_parity import philox_action
    oo = orc.Oracle(default_params(), n, seed=23)
    oo.set_randomization(**ALL)
    oo.reset()
    for t in range(steps):
        act = np.stack([philox_action(23, i, int(oo.state[FIELD["step_count"], i])) for i in range(n)])
        oo.step(act, auto_reset=True)
    assert_state_equal(a.get_state(), oo.state, "rollout RAND vs oracle")


def test_robot_api_with_disturbances_and_dynamics_equal_oracle():
    n = 256
    env, o = make_pair(n, 29, dynamics=True, disturbances=True)
    rng = np.random.default_rng(8)
    for _ in range(3):
        yaw = rng.uniform(-1.5, 1.5, n)
        env.nozzle_solve(yaw)
        o.nozzle_solve(yaw, False)
        g = _cpu(env.get_state())
        ctl = np.stack([rng.uniform(0.01, 0.06, n), rng.uniform(0, 3, n), g[FIELD["angle1"]],
                        g[FIELD["angle2"]]], 1)
        env.robot_set_control(ctl)
        o.robot_set_control(ctl, False)
        env.robot_step_through_cycle()
        o.robot_cycle()
        assert_state_equal(env.get_state(), o.state, "robot API RAND")


def test_switching_randomization_off_restores_reference_behaviour():
    n = 256
    rng = np.random.default_rng(2)
    env, o = make_pair(n, 31, **ALL)
    a = random_actions(rng, n)
    env.step(torch.tensor(a), auto_reset=True)
    o.step(a, auto_reset=True)
    env.set_randomization()
    o.set_randomization()
    for _ in range(2):
        a = random_actions(rng, n)
        r = env.step(torch.tensor(a), auto_reset=True)
        ro = o.step(a, auto_reset=True)
        assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True)
    g = _cpu(env.get_state())
    assert np.all(g[FIELD["cd"]] == 0.3)
    assert_state_equal(g, o.state, "after switching off")


def test_randomized_sorted_lockstep_and_rollout_at_scale():
    """Every switch on, 70 000 envs (more than one wave per SIMD: the lock-step
    call runs in sorted order, and the RAND kernels carry the randomisation
    fields in rows beside the env-major cold block): sorted == env order bit
    for bit, both == the oracle on a block; then a chained rollout on top."""
    n = 70_000
    p = default_params()
    a = BatchedSalpEnv(n, params=p, seed=21)
    b = BatchedSalpEnv(n, params=p, seed=21)
    for e in (a, b):
        e.set_randomization(**ALL)
    a.set_lockstep_order(1)
    b.set_lockstep_order(0)
    ra, rb = a.step_random(2), b.step_random(2)
    assert torch.equal(ra.view(torch.int64), rb.view(torch.int64))
    ga = a.get_state()
    assert torch.equal(ga.view(torch.int64), b.get_state().view(torch.int64))
    lo = 40_000
    o = orc.Oracle(p, 256, seed=21, env_offset=lo)
    o.set_randomization(**ALL)
    o.reset()
    rs_o, _ = o.step_random(2)
    assert np.array_equal(_cpu(ra)[lo:lo + 256], rs_o, equal_nan=True)
    assert_state_equal(_cpu(ga)[:, lo:lo + 256], o.state, "RAND sorted lock-step")
    done = torch.zeros(n, dtype=torch.int64, device="cuda")
    a.rollout(3000, steps_done=done, max_steps=2)
    o.step_random(2)
    assert int(done.min()) == 2
    assert_state_equal(_cpu(a.get_state())[:, lo:lo + 256], o.state, "RAND rollout after lock-step")
