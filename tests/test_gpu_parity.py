"""Device (libsalp.so, gfx950) against the CPU oracle — bit for bit.

The oracle is pinned to the reference by tests/test_oracle_golden.py; here the
HIP path must reproduce the oracle EXACTLY (np.array_equal on fp64 state,
float32 observations, fp64 rewards, flags).  Everything goes through the C ABI
via grasp_lab_salp_amd.batched_env.
"""
import numpy as np
import pytest
import torch

from golden_util import COMPARED, load_episodes, snapshot_to_state
from grasp_lab_salp_amd._abi import FIELD, FIELDS, INFO, MATH_SELFTEST_ROWS, NUM_FIELDS, default_params
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _cpu(t):
    return t.detach().cpu().numpy()


def assert_state_equal(gpu_state, cpu_state, what=""):
    g = _cpu(gpu_state) if torch.is_tensor(gpu_state) else gpu_state
    bad = [(FIELDS[f], int(np.sum(~((g[f] == cpu_state[f]) | (np.isnan(g[f]) & np.isnan(cpu_state[f]))))))
           for f in range(NUM_FIELDS) if not np.array_equal(g[f], cpu_state[f], equal_nan=True)]
    assert not bad, f"{what}: state fields differ from the oracle: {bad[:8]}"


def assert_bits_equal(x, y, what="", nan_payloads=False):
    """Two device states [NUM_FIELDS, n] equal bit for bit (nan_payloads:
    except that where both hold a NaN its payload may differ: two different
    kernels carry a diverged env's NaN through different instruction
    sequences); on failure the message names the fields and whether the
    differences are NaN payloads, signed zeros or values."""
    a, b = _cpu(x), _cpu(y)
    d = a.view(np.int64) != b.view(np.int64)
    if nan_payloads:
        d &= ~(np.isnan(a) & np.isnan(b))
    if not d.any():
        return
    nan = d & np.isnan(a) & np.isnan(b)
    zero = d & (a == 0) & (b == 0)
    val = d & ~nan & ~zero
    rows = [(FIELDS[f], int(val[f].sum()), int(nan[f].sum()), int(zero[f].sum()))
            for f in np.nonzero(d.any(1))[0]]
    envs = np.nonzero(val.any(0))[0][:8].tolist()
    raise AssertionError(f"{what}: (field, values, nan payloads, signed zeros) {rows[:10]}; value envs {envs}")


def make_pair(n, seed=3, step_kernel=-1, **kw):
    p = default_params(**kw)
    env = BatchedSalpEnv(n, params=p, seed=seed)
    env.set_step_kernel(step_kernel)
    o = orc.Oracle(p, n, seed=seed)
    return env, o


def random_actions(rng, n):
    return np.stack([rng.uniform(0, 1, n), rng.uniform(0, 1, n), rng.uniform(-1, 1, n)],
                    1).astype(np.float32)


def test_device_math_equals_oracle_math():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-4, 4, 20000), rng.uniform(-1, 1, 20000),
                        rng.uniform(-1e-4, 1e-4, 2000), rng.uniform(-80, 80, 2000),
                        [0.0, 1.0, -1.0, 0.5, np.pi / 4, np.pi / 2]])
    y = rng.uniform(-3, 3, len(x))
    # the tick's roll / pitch pair: both short, one short, either NaN / inf
    xs = np.concatenate([rng.uniform(-0.07, 0.07, 8000), [0.0, -0.0, 0.0625, -0.0625, np.nan, 0.01, np.inf, 0.01]])
    ys = np.concatenate([rng.uniform(-0.07, 0.07, 8000), [0.0, 0.0, 0.0625, 0.07, 0.01, np.nan, 0.01, -np.inf]])
    x, y = np.concatenate([x, xs]), np.concatenate([y, ys])
    g, ref = _device_math(x, y), orc.math_selftest(x, y)
    for r in range(MATH_SELFTEST_ROWS):
        assert np.array_equal(g[r], ref[r], equal_nan=True), f"math row {r}: {np.sum(g[r] != ref[r])} mismatches"
    # tumbling and diverging angles: the medium range, up to 2^51 pi/2, and
    # beyond it where sm_sincos_yaw_p is unspecified (tests/test_math.py) but
    # the device must still equal the oracle: the float64 sin / cos rows (fdlibm,
    # branch-free, the tick's yaw and roll / pitch pair; the float32 rows take
    # the yaw of an action, |x| <= pi/2, only)
    big = 10.0 ** rng.uniform(1, 308, 4000) * rng.choice([-1.0, 1.0], 4000)
    big = np.concatenate([big, 10.0 ** rng.uniform(-1.2, 11, 4000) * rng.choice([-1.0, 1.0], 4000)])
    g, ref = _device_math(big, big[::-1].copy()), orc.math_selftest(big, big[::-1].copy())
    for r in (0, 1, 9, 10, 12, 13, 14, 15, 16, 17):   # bit for bit; NaN payloads aside (x86's default NaN is negative)
        same = (g[r].view(np.int64) == ref[r].view(np.int64)) | (np.isnan(g[r]) & np.isnan(ref[r]))
        assert same.all(), f"large angles, row {r}: {int((~same).sum())} mismatches"


def _device_math(x, y):
    from grasp_lab_salp_amd import _lib
    import ctypes
    L = _lib.load()
    xd = torch.tensor(x, device="cuda")
    yd = torch.tensor(y, device="cuda")
    out = torch.empty((MATH_SELFTEST_ROWS, len(x)), dtype=torch.float64, device="cuda")
    _lib.check(L.salp_math_selftest(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(yd.data_ptr()),
                                    len(x), ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    return _cpu(out)



def test_shared_reciprocal_division_equals_ieee_division():
    """qdiv(x, rcp_of(y)) (the tick's divisions by mass, inertia, cos(pitch),
    width, ...) against the oracle's C `x / y` over 200 decades of magnitude,
    both signs, and the zero / inf operands v_div_fixup handles."""
    rng = np.random.default_rng(5)
    n = 200000
    x = 10.0 ** rng.uniform(-100, 100, n) * rng.choice([-1.0, 1.0], n)
    y = 10.0 ** rng.uniform(-100, 100, n) * rng.choice([-1.0, 1.0], n)
    sx = np.array([0.0, -0.0, 5.0, -5.0, np.inf, 2.0, 0.0, 3.0, 1.0, 7.0])
    sy = np.array([5.0, 5.0, 0.0, -0.0, 2.0, np.inf, 0.0, 3.0, 3.0, 0.1])
    x, y = np.concatenate([x, sx]), np.concatenate([y, sy])
    from grasp_lab_salp_amd import _lib
    import ctypes
    L = _lib.load()
    xd = torch.tensor(x, device="cuda")
    yd = torch.tensor(y, device="cuda")
    out = torch.empty((MATH_SELFTEST_ROWS, len(x)), dtype=torch.float64, device="cuda")
    _lib.check(L.salp_math_selftest(ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(yd.data_ptr()),
                                    len(x), ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    got = _cpu(out)[11]
    want = x / y
    both_nan = np.isnan(got) & np.isnan(want)   # 0/0: NaN payloads differ by platform
    bad = (got.view(np.uint64) != want.view(np.uint64)) & ~both_nan
    assert not bad.any(), f"{bad.sum()} quotients differ, e.g. {x[bad][:3]} / {y[bad][:3]}"

def test_fresh_envs_equal_oracle():
    env, o = make_pair(1000)
    o.reset()  # SalpRobotEnv.__init__ -> reset()
    assert_state_equal(env.get_state(), o.state, "after create")
    ob = env.reset()
    ob_o = o.reset()
    assert np.array_equal(_cpu(ob), ob_o)
    assert_state_equal(env.get_state(), o.state, "after reset")


@pytest.mark.parametrize("K", [0, 2, 4])
def test_teacher_forced_golden_rows(K):
    """Restart from every reference pre-step state of the golden fixture."""
    d = load_episodes()
    rows = np.where(d["num_obstacles_cfg"] == K)[0]
    p = default_params(num_obstacles=K)
    st = snapshot_to_state(d, "b_", rows)
    env = BatchedSalpEnv(len(rows), params=p)
    env.set_state(torch.tensor(st))
    o = orc.Oracle(p, len(rows))
    o.state[:] = st
    r = env.step(torch.tensor(d["action"][rows]), auto_reset=False)
    ro = o.step(d["action"][rows])
    assert_state_equal(env.get_state(), o.state, f"golden K={K}")
    assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True)
    assert np.array_equal(_cpu(r.reward), ro["reward"], equal_nan=True)
    assert np.array_equal(_cpu(r.terminated).astype(np.uint8), ro["terminated"])
    assert np.array_equal(_cpu(r.truncated).astype(np.uint8), ro["truncated"])
    assert np.array_equal(_cpu(r.info), ro["info"], equal_nan=True)
    # and directly against the reference itself (same tolerances as the oracle tests)
    after = snapshot_to_state(d, "a_", rows)
    g = _cpu(env.get_state())
    for name in ("pw0", "pw1", "v0", "v1", "eta2", "w2", "length", "cycle_time", "phase"):
        i = FIELD[name]
        floor = 1e-6 * np.max(np.abs(after[i])) + 1e-300
        assert np.max(np.abs(g[i] - after[i]) / np.maximum(np.abs(after[i]), floor)) <= 2e-6, name
    assert np.array_equal(_cpu(r.terminated), d["terminated"][rows].astype(bool))
    assert np.array_equal(_cpu(r.truncated), d["truncated"][rows].astype(bool))


def test_random_batch_free_running_with_auto_reset():
    """4096 envs, injected targets/obstacles, 6 env-steps of random float32
    actions, SB3-style auto-reset (Philox draws on both sides)."""
    n = 4096
    rng = np.random.default_rng(11)
    env, o = make_pair(n, seed=5)
    o.reset()
    tg = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n)], 1).astype(np.float32)
    ob = rng.uniform(-2, 2, (n, 2, 2)).astype(np.float32)
    nob = rng.integers(0, 3, n).astype(np.int32)
    obs_g = env.reset_to(torch.tensor(tg), torch.tensor(ob), torch.tensor(nob))
    obs_o = o.reset_to(tg, ob, nob)
    assert np.array_equal(_cpu(obs_g), obs_o)
    for t in range(6):
        a = random_actions(rng, n)
        if t == 2:
            a[:64] = 0.0          # zero-tick cycles
            a[64:128, 1] = 1.0    # longest coasts
        r = env.step(torch.tensor(a), auto_reset=True)
        ro = o.step(a, auto_reset=True)
        assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True), t
        assert np.array_equal(_cpu(r.terminal_obs), ro["terminal_obs"], equal_nan=True), t
        assert np.array_equal(_cpu(r.reward), ro["reward"], equal_nan=True), t
        assert np.array_equal(_cpu(r.info), ro["info"], equal_nan=True), t
        assert np.array_equal(_cpu(r.terminated).astype(np.uint8), ro["terminated"]), t
        assert np.array_equal(_cpu(r.truncated).astype(np.uint8), ro["truncated"]), t
        assert_state_equal(env.get_state(), o.state, f"step {t}")


def test_step_random_matches_oracle():
    n = 2048
    env, o = make_pair(n, seed=9)
    o.reset()
    rs = env.step_random(12)
    rs_o, _ = o.step_random(12)
    assert np.array_equal(_cpu(rs), rs_o, equal_nan=True)
    assert_state_equal(env.get_state(), o.state, "step_random")


@pytest.mark.parametrize("n", [1, 64, 300])
def test_steady_first_tick_after_reset(n):
    """Contraction exactly 0 (a clipped policy action): refill and jet times
    are negative, so the cycle's very first tick is already COAST.  Right
    after a reset the state's geometry is Robot.reset's, whose centre of mass
    differs from update_properties' in the last bits: the steady-body loop
    must not keep it (found by tests/test_gpu_collect.py, env 79 of a
    300-env collection).  One env per wave included (n = 1: the lane alone
    decides the steady switch).  Lock-step step and the chained rollout
    path, bit for bit against the oracle."""
    env, o = make_pair(n, seed=5)
    o.reset()
    env.set_state(torch.tensor(o.state))
    rng = np.random.default_rng(7)
    a = random_actions(rng, n)
    a[:, 0] = 0.0
    for t in range(3):
        r = env.step(torch.tensor(a), auto_reset=True)
        ro = o.step(a, auto_reset=True)
        assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True), t
        assert_state_equal(env.get_state(), o.state, f"contraction 0, step {t}")
        env.reset()
        o.reset()
        env.set_state(torch.tensor(o.state))


@pytest.mark.parametrize("n,k", [(300, 32), (2048, 33)])
def test_chained_step_random_equals_lockstep_steps(n, k):
    """salp_step_random(k >= 32) runs on the chained kernel (each env does its k
    env-steps back to back); k calls of salp_step_random(1) run the lock-step
    kernel.  Same state and reward sums bit for bit, also when the handle
    holds cycles cut in flight by a tick-budget rollout (both drop them and
    start a new env-step, as SalpRobotEnv.step would)."""
    p = default_params()
    a = BatchedSalpEnv(n, params=p, seed=41)
    b = BatchedSalpEnv(n, params=p, seed=41)
    for e in (a, b):
        e.rollout(333)   # leaves most envs mid-cycle (pending)
    pend = _cpu(a.field("pending"))
    assert pend.mean() > 0.5
    ra = a.step_random(k)
    rb = torch.zeros_like(ra)
    for _ in range(k):
        rb = rb + b.step_random(1)
    assert np.array_equal(_cpu(ra), _cpu(rb), equal_nan=True)
    assert_bits_equal(a.get_state(), b.get_state(), "chained vs lock-step", nan_payloads=True)
    assert np.all(_cpu(a.field("pending")) == 0)


def test_rollout_is_split_invariant_and_matches_oracle():
    """Tick-budget rollouts: cutting the same work into different launches gives
    identical bits, equal to the lock-step oracle at env-step boundaries, and
    the rollout buffer holds the per-step outputs."""
    n, steps = 1024, 6
    p = default_params()
    a = BatchedSalpEnv(n, params=p, seed=21)
    b = BatchedSalpEnv(n, params=p, seed=21)
    cap = steps
    bufs = {"obs": torch.zeros((cap, n, 10), device="cuda"),
            "obs_before": torch.zeros((cap, n, 10), device="cuda"),
            "actions": torch.zeros((cap, n, 3), device="cuda"),
            "rewards": torch.zeros((cap, n), device="cuda"),
            "dones": torch.zeros((cap, n), dtype=torch.uint8, device="cuda")}
    sa = torch.zeros(n, dtype=torch.int64, device="cuda")
    sb = torch.zeros(n, dtype=torch.int64, device="cuda")
    a.rollout(10**7, buffers=bufs, steps_done=sa, max_steps=steps)
    for _ in range(400):
        b.rollout(97, steps_done=sb, max_steps=steps)
        if int(sb.min()) >= steps:
            break
    assert int(sa.min()) == steps and int(sa.max()) == steps
    assert int(sb.min()) == steps
    ga, gb = _cpu(a.get_state()), _cpu(b.get_state())
    assert np.array_equal(ga, gb, equal_nan=True)
    o = orc.Oracle(p, n, seed=21)
    obs0 = o.reset()
    # oracle step-by-step with the same Philox actions
    from grasp_lab_salp_amd._abi import FIELD as FF
    acts = []
    outs = []
    for t in range(steps):
        act = np.zeros((n, 3), np.float32)
        for i in range(n):
            act[i] = philox_action(21, i, int(o.state[FF["step_count"], i]))
        ro = o.step(act, auto_reset=True)
        acts.append(act)
        outs.append(ro)
    assert_state_equal(ga, o.state, "rollout vs oracle")
    for t in range(steps):
        assert np.array_equal(_cpu(bufs["actions"][t]), acts[t])
        assert np.array_equal(_cpu(bufs["obs"][t]), outs[t]["terminal_obs"], equal_nan=True)
        # the observation the action was taken on: reset obs, then each step's
        # returned obs (the reset obs where the previous step ended an episode)
        before = obs0 if t == 0 else outs[t - 1]["obs"]
        assert np.array_equal(_cpu(bufs["obs_before"][t]), before, equal_nan=True), t
        assert np.array_equal(_cpu(bufs["rewards"][t]), outs[t]["reward"].astype(np.float32), equal_nan=True)
        dn = outs[t]["terminated"] | (outs[t]["truncated"] << 1)
        assert np.array_equal(_cpu(bufs["dones"][t]), dn)


@pytest.mark.parametrize("n,chunk", [(1, 128), (63, 16), (300, 128), (700, 7), (1024, 300)])
def test_rollout_reseating_in_ragged_batches_equals_lockstep(n, chunk):
    """k_rollout re-seats the envs of a workgroup onto its lanes at every chunk
    boundary (steady-body envs together).  Ragged batches (empty slots in the
    last workgroup), tiny and long chunks: the rollout with max_steps k must
    equal k lock-step env-steps bit for bit, and so the oracle."""
    p = default_params()
    k = 5
    a = BatchedSalpEnv(n, params=p, seed=31)
    b = BatchedSalpEnv(n, params=p, seed=31)
    sa = torch.zeros(n, dtype=torch.int64, device="cuda")
    for _ in range(2000):
        a.rollout(977, steps_done=sa, max_steps=k, chunk=chunk)
        if int(sa.min()) >= k:
            break
    assert int(sa.min()) == k and int(sa.max()) == k
    b.step_random(k)
    ga = _cpu(a.get_state())
    assert np.array_equal(ga, _cpu(b.get_state()), equal_nan=True)
    o = orc.Oracle(p, n, seed=31)
    o.reset()
    o.step_random(k)
    assert_state_equal(ga, o.state, f"rollout n={n} chunk={chunk}")


def philox_action(seed, env_id, step):
    """sp_action() of salp_philox.h restated in Python for the test."""
    out = orc.philox([step & 0xFFFFFFFF, step >> 32, env_id & 0xFFFFFFFF, 0 | ((env_id >> 32) << 1)],
                     [seed & 0xFFFFFFFF, seed >> 32])
    u = [np.float32(x >> 8) * np.float32(2.0 ** -24) for x in out[:3]]
    return np.array([u[0], u[1], np.float32(2.0) * u[2] - np.float32(1.0)], np.float32)


def test_sharding_by_env_id_offset():
    """An env's trajectory depends only on its global id (multi-GPU sharding)."""
    p = default_params()
    full = BatchedSalpEnv(256, params=p, seed=4)
    part = BatchedSalpEnv(64, params=p, seed=4, env_id_offset=128)
    full.step_random(5)
    part.step_random(5)
    assert np.array_equal(_cpu(full.get_state())[:, 128:192], _cpu(part.get_state()), equal_nan=True)


def test_reference_blowup_is_reproduced():
    """The reference's explicit integrator diverges when jet_time < dt (e.g. the
    action below: refill 0.0074 s, jet 0.0060 s): velocities overflow and turn
    NaN at tick 100 of the cycle (checked against the Python reference, see
    DESIGN.md).  The device reproduces it exactly as the oracle does."""
    env, o = make_pair(4, seed=0)
    o.reset()
    env.set_state(torch.tensor(o.state))
    a = np.tile(np.float32([0.0904393, 0.06936062, -0.76570743]), (4, 1))
    r = env.step(torch.tensor(a))
    ro = o.step(a)
    assert ro["ticks"][0] == 151
    assert np.all(np.isnan(ro["obs"][:, :6]))
    assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True)
    assert_state_equal(env.get_state(), o.state, "blow-up")


def test_timeout_and_zero_tick_cycles():
    """500 zero-tick cycles (action [0,0,0]) truncate with the timeout penalty."""
    n = 8
    env, o = make_pair(n, seed=2)
    o.reset()
    a = np.zeros((n, 3), np.float32)
    for t in range(500):
        r = env.step(torch.tensor(a), auto_reset=False)
    for t in range(500):
        ro = o.step(a)
    assert np.all(_cpu(r.truncated))
    assert np.array_equal(_cpu(r.reward), ro["reward"], equal_nan=True)
    assert_state_equal(env.get_state(), o.state, "timeout")
    assert np.all(_cpu(env.field("cycle")) == 500)
    assert np.all(_cpu(env.field("time")) == 0)


def test_float32_shape_carried_across_cycles():
    """A cycle that ends while REFILL still holds the float32 contracted body
    (contraction ~0, no coast: jet + coast < 0) followed by a cycle that starts
    in a different float32 shape: the first tick has both volumes float32 but
    V != prev V, the one case where jet_rates' float32 arm differs from its
    float64 arm (r2 experiment log).  Mixed with ordinary lanes in every wave;
    device == oracle bit for bit."""
    n = 256
    env, o = make_pair(n, seed=8)
    o.reset()
    rng = np.random.default_rng(3)
    a1 = random_actions(rng, n)
    a2 = random_actions(rng, n)
    sel = np.arange(n) % 2 == 0
    a1[sel, 0] = 0.0
    a1[sel, 1] = 0.0
    a1[sel, 2] = np.linspace(-1, 1, sel.sum())
    a2[sel, 0] = 0.05
    a2[sel, 1] = 0.0
    a2[sel, 2] = -np.linspace(-1, 1, sel.sum())
    for t, a in enumerate((a1, a2, random_actions(rng, n))):
        r = env.step(torch.tensor(a), auto_reset=True)
        ro = o.step(a, auto_reset=True)
        assert np.array_equal(_cpu(r.obs), ro["obs"], equal_nan=True), t
        assert np.array_equal(_cpu(r.reward), ro["reward"], equal_nan=True), t
        assert_state_equal(env.get_state(), o.state, f"step {t}")
        if t == 0:   # (almost all) even lanes end the cycle in the float32 REFILL shape
            in32 = (o.state[FIELD["geom32"], sel] == 1) & (o.state[FIELD["phase"], sel] == 0)
            assert in32.mean() > 0.9


@pytest.mark.parametrize("n", [3000, 200_000])
def test_sorted_lockstep_order_changes_nothing_but_time(n):
    """salp_set_lockstep_order: the lock-step kernels run envs sorted by their
    predicted cycle length (auto above one wave per SIMD, i.e. at 200 000
    envs).  Per-env results are bit-identical to env order, and to the oracle
    on a block of envs."""
    p = default_params()
    a = BatchedSalpEnv(n, params=p, seed=12)
    b = BatchedSalpEnv(n, params=p, seed=12)
    a.set_lockstep_order(1)
    b.set_lockstep_order(0)
    ra, rb = a.step_random(2), b.step_random(2)
    rng = np.random.default_rng(4)
    act = torch.tensor(random_actions(rng, n), device="cuda")
    sa, sb = a.step(act, auto_reset=True), b.step(act, auto_reset=True)
    assert torch.equal(ra.view(torch.int64), rb.view(torch.int64))
    for x, y in ((sa.obs, sb.obs), (sa.reward, sb.reward), (sa.info, sb.info), (sa.terminal_obs, sb.terminal_obs)):
        assert torch.equal(x.contiguous().view(torch.int32 if x.dtype == torch.float32 else torch.int64),
                           y.contiguous().view(torch.int32 if y.dtype == torch.float32 else torch.int64))
    assert torch.equal(sa.terminated, sb.terminated) and torch.equal(sa.truncated, sb.truncated)
    ga = a.get_state()
    assert torch.equal(ga.view(torch.int64), b.get_state().view(torch.int64))
    # and the envs are the reference's: oracle on a block of global ids
    lo = n // 2
    o = orc.Oracle(p, 512, seed=12, env_offset=lo)
    o.reset()
    o.step_random(2)
    o.step(_cpu(act)[lo:lo + 512], auto_reset=True)
    assert_state_equal(_cpu(ga)[:, lo:lo + 512], o.state, "sorted lock-step block")


@pytest.mark.parametrize("n", [1, 255, 4099])
def test_state_round_trip_through_the_hbm_layout(n):
    """salp_set_state / salp_get_state convert between the ABI's field-major
    view and the handle's layout (rows + env-major cold block): any bit
    pattern, NaNs and signed zeros included, comes back unchanged; ragged
    sizes exercise the padded cold-block offset."""
    env = BatchedSalpEnv(n, params=default_params(), seed=1)
    g = torch.Generator().manual_seed(n)
    bits = torch.randint(-2**62, 2**62, (NUM_FIELDS, n), generator=g, dtype=torch.int64)
    st = bits.view(torch.float64).clone()
    st[0, 0] = float("nan")
    st[1, 0] = -0.0
    env.set_state(st)
    back = env.get_state().cpu()
    assert torch.equal(back.view(torch.int64), st.view(torch.int64))


@pytest.mark.parametrize("step_kernel", [0, 1])
@pytest.mark.parametrize("n", [1, 128])
def test_steady_body_with_negative_phase_times(n, step_kernel):
    """The lock-step kernels run a cycle's COAST/REST ticks without the
    geometry once every lane of the wave is there (salp_device.h
    next_tick_steady).  Small contractions give negative refill and jet times
    (the reference's polynomial), so mx + jet < mx: the first ticks are still
    REFILL with a contracted body although cycle_time > mx + jet.  Every env
    of the batch gets such an action (the whole wave votes), 4 env-steps,
    bit for bit against the oracle; then ordinary actions.  Both salp_step
    kernels (one env per lane, one env per two-wave workgroup)."""
    env, o = make_pair(n, seed=21, step_kernel=step_kernel)
    o.reset()
    rng = np.random.default_rng(8)
    for k in range(6):
        act = random_actions(rng, n)
        if k < 4:
            act[:, 0] = rng.uniform(0.0, 0.05, n).astype(np.float32)
        env.step(torch.tensor(act, device="cuda"), auto_reset=True)
        o.step(act, auto_reset=True)
        assert_state_equal(env.get_state(), o.state, f"env-step {k}")
        if k < 4:   # the case is exercised
            assert (o.state[FIELD["jet_time"]] < 0).all()


@pytest.mark.parametrize("step_kernel", [0, 1])
@pytest.mark.parametrize("job", [0, 3, 17, 21, 22])
def test_fixture_episode_actions_on_one_env_bit_exact(job, step_kernel):
    """The actions of a reference episode (tests/golden/episodes.npz) on a
    single env, HIP lock-step kernel vs oracle, bit for bit after every
    env-step.  A one-env wave votes alone on the steady-body switch, so this
    is where a wrong switch shows (job 3, env-step 24: contraction 0.0022,
    jet time -0.07 s, turn time 0.016 s, i.e. one REFILL tick after
    cycle_time > mx + jet).  Both salp_step kernels."""
    d = load_episodes()
    rows = np.where(d["job_index"] == job)[0]
    env, o = make_pair(1, seed=job, step_kernel=step_kernel)
    o.reset()
    o.state[:] = _cpu(env.get_state())
    for k, r in enumerate(rows):
        a = np.asarray(d["action"][r], np.float32)[None]
        env.step(torch.tensor(a, device="cuda"), auto_reset=False)
        o.step(a, auto_reset=False)
        assert_state_equal(env.get_state(), o.state, f"job {job} env-step {k}")
