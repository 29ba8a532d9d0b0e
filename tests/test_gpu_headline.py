"""The HIP path at BASELINE.json's headline sizes (configs[2] and configs[3]).

configs[2]: 65 536 envs, random-action rollout on one MI355X (the bench
workload, src/salp_robot_env.py:196-299 per env-step).  configs[3]: 524 288
envs sharded 8 ways, i.e. a 65 536-env handle whose global env ids start at
rank * 65 536 (here the last rank, 7 * 65 536).

* split invariance at full size: one launch running every env to 6 env-steps
  == the same work cut into 97-tick launches (state, steps_done and rollout
  buffers, bit for bit);
* the headline rollout against the C oracle (oracle/salp_oracle.c, pinned to
  the reference by tests/test_oracle_golden.py) on blocks of env ids spread
  over the 65 536, buffers included;
* the lock-step kernel on ALL 65 536 envs against the OpenMP oracle, and the
  chained salp_step_random(32) against 32 lock-step calls;
* the config-4 shard (global ids up to 2^19 - 1, plus a block across 2^32 for
  the Philox counter's high word) against the oracle at the same global ids.
"""
import os

import numpy as np
import pytest
import torch

from grasp_lab_salp_amd._abi import FIELD, default_params
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
from oracle import oracle as orc
from test_gpu_parity import assert_state_equal, philox_action

pytestmark = pytest.mark.gpu

N = 65536
SEED = 17


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def _cpu(t):
    return t.detach().cpu().numpy()


def _bits(t):
    t = t.contiguous()
    if t.dtype == torch.float64:
        return t.view(torch.int64)
    if t.dtype == torch.float32:
        return t.view(torch.int32)
    return t


def _bits_equal(x, y):
    """Bit for bit, except that two NaNs are equal whatever their sign and
    payload: a diverged env's NaN carries a sign that depends on which tick
    instance (full / steady / settled) its lane ran, i.e. on the wave it shared
    (profiles/r6c_split_probe_r5ao.json: every non-NaN value identical), and
    NaN signs and payloads are no part of the reference's results."""
    if x.shape != y.shape:
        return False
    same = _bits(x) == _bits(y)
    if x.dtype.is_floating_point:
        same |= torch.isnan(x) & torch.isnan(y)
    return bool(same.all())


def _buffers(cap, n, dev="cuda"):
    return {"obs": torch.full((cap, n, 10), -7.0, device=dev),
            "obs_before": torch.full((cap, n, 10), -7.0, device=dev),
            "actions": torch.full((cap, n, 3), -7.0, device=dev),
            "rewards": torch.full((cap, n), -7.0, device=dev),
            "dones": torch.full((cap, n), 255, dtype=torch.uint8, device=dev)}


def test_headline_rollout_is_split_invariant_at_65536():
    """One launch that runs every env to 6 env-steps == the same work cut into
    97-tick launches (state, steps_done and rollout buffers, bit for bit).
    How far an env gets in a launch depends on the scheduling (k_rollout
    re-seats envs onto lanes every chunk and gives all-steady waves a longer
    tick budget), what it computes does not.  DESIGN.md §4 cites this test."""
    p = default_params()
    chunk, steps = 97, 6
    a = BatchedSalpEnv(N, params=p, seed=SEED)
    b = BatchedSalpEnv(N, params=p, seed=SEED)
    ba, bb = _buffers(32, N), _buffers(32, N)
    sa = torch.zeros(N, dtype=torch.int64, device="cuda")
    sb = torch.zeros(N, dtype=torch.int64, device="cuda")
    a.rollout(20000, buffers=ba, steps_done=sa, chunk=chunk, max_steps=steps)
    launches = 0
    while int(sb.min()) < steps and launches < 400:
        b.rollout(chunk, buffers=bb, steps_done=sb, chunk=chunk, max_steps=steps)
        launches += 1
    torch.cuda.synchronize()
    assert launches > 40, "the cut run should take many launches"
    assert int(sa.min()) == steps and int(sa.max()) == steps
    assert torch.equal(sa, sb)
    assert _bits_equal(a.get_state(), b.get_state())
    for k in ba:
        assert _bits_equal(ba[k], bb[k]), k
    # slots past steps_done are untouched, slots below are written
    slot = torch.arange(32, device="cuda").unsqueeze(1)
    written = slot < sa.unsqueeze(0)
    assert bool((ba["dones"][written] != 255).all()) and bool((ba["dones"][~written] == 255).all())
    # every completed env-step was counted
    assert int(sa.sum()) == int(written.sum())


def _oracle_rollout(seed, start, n, steps, env_offset_base=0):
    """The chained rollout per env == env-steps with Philox actions keyed by
    (seed, global id, step count) and auto-reset: the oracle step by step."""
    o = orc.Oracle(default_params(), n, seed=seed, env_offset=env_offset_base + start)
    obs0 = o.reset()
    outs, acts = [], []
    for _ in range(steps):
        act = np.zeros((n, 3), np.float32)
        sc = o.state[FIELD["step_count"]]
        for i in range(n):
            act[i] = philox_action(seed, env_offset_base + start + i, int(sc[i]))
        outs.append(o.step(act, auto_reset=True))
        acts.append(act)
    return o, acts, outs, obs0


def _check_blocks(env, bufs, done, steps, blocks, seed, base=0):
    g = _cpu(env.get_state())
    assert int(done.min()) == steps and int(done.max()) == steps
    for start, n in blocks:
        o, acts, outs, obs0 = _oracle_rollout(seed, start, n, steps, base)
        sl = slice(start, start + n)
        assert_state_equal(g[:, sl], o.state, f"block {base + start}")
        for t in range(steps):
            before = obs0 if t == 0 else outs[t - 1]["obs"]
            assert np.array_equal(_cpu(bufs["obs_before"][t, sl]), before, equal_nan=True), (start, t)
            assert np.array_equal(_cpu(bufs["actions"][t, sl]), acts[t]), (start, t)
            assert np.array_equal(_cpu(bufs["obs"][t, sl]), outs[t]["terminal_obs"], equal_nan=True), (start, t)
            assert np.array_equal(_cpu(bufs["rewards"][t, sl]), outs[t]["reward"].astype(np.float32),
                                  equal_nan=True), (start, t)
            dn = outs[t]["terminated"] | (outs[t]["truncated"] << 1)
            assert np.array_equal(_cpu(bufs["dones"][t, sl]), dn), (start, t)


def test_headline_rollout_matches_oracle_on_blocks():
    """configs[2]: 65 536 envs, 3 env-steps each through k_rollout (buffers
    filled), checked against the oracle on 4 blocks of env ids."""
    steps = 3
    env = BatchedSalpEnv(N, params=default_params(), seed=SEED)
    bufs = _buffers(steps, N)
    done = torch.zeros(N, dtype=torch.int64, device="cuda")
    env.rollout(6000, buffers=bufs, steps_done=done, max_steps=steps)
    torch.cuda.synchronize()
    _check_blocks(env, bufs, done, steps, [(0, 256), (20000, 256), (45311, 256), (N - 256, 256)], SEED)


def test_headline_lockstep_all_envs_match_openmp_oracle():
    """Every one of the 65 536 envs, 2 random env-steps, against the
    whole-batch OpenMP oracle (bit for bit: state and reward sums): the
    lock-step kernel k_step_random (one env-step per call, and two per call).
    Then the chained salp_step_random(32) (k_rollout with max_steps, every env
    running its env-steps back to back) equals 32 lock-step calls bit for bit."""
    p = default_params()
    env = BatchedSalpEnv(N, params=p, seed=SEED)
    rs = env.step_random(1)
    rs = rs + env.step_random(1)
    two = BatchedSalpEnv(N, params=p, seed=SEED)
    rs2 = two.step_random(2)
    o = orc.Oracle(p, N, seed=SEED)
    o.reset()
    rs_o, ticks = o.step_random(2, threads=_threads())
    assert ticks > 0
    assert np.array_equal(_cpu(rs), rs_o, equal_nan=True)
    assert_state_equal(env.get_state(), o.state, "lock-step 65536")
    assert np.array_equal(_cpu(rs2), _cpu(rs), equal_nan=True)   # NaN payloads of a diverged env's sum may differ
    assert _bits_equal(two.get_state(), env.get_state())
    rs_c = two.step_random(32)
    rs_l = torch.zeros_like(rs_c)
    for _ in range(32):
        rs_l = rs_l + env.step_random(1)
    assert np.array_equal(_cpu(rs_c), _cpu(rs_l), equal_nan=True)
    _equal_up_to_nan_payload(two.get_state(), env.get_state())


def _equal_up_to_nan_payload(x, y):
    """Bit for bit, except that where both hold a NaN the payloads may differ
    (a diverged env's NaN state goes through different instruction sequences
    in the chained and the lock-step kernels)."""
    a, b = _cpu(x), _cpu(y)
    both_nan = np.isnan(a) & np.isnan(b)
    diff = (a.view(np.int64) != b.view(np.int64)) & ~both_nan
    assert not diff.any(), (np.nonzero(diff.any(1))[0].tolist(), int(diff.sum()))


@pytest.mark.parametrize("base", [7 * N, (1 << 32) - N // 2])
def test_config4_shard_matches_oracle_at_its_global_ids(base):
    """configs[3]: the last of 8 shards (global ids 458 752 .. 524 287), and a
    shard whose ids cross 2^32 (Philox counter high word), 2 env-steps each;
    blocks checked against the oracle keyed by the same global ids."""
    steps = 2
    env = BatchedSalpEnv(N, params=default_params(), seed=SEED, env_id_offset=base)
    bufs = _buffers(steps, N)
    done = torch.zeros(N, dtype=torch.int64, device="cuda")
    env.rollout(4000, buffers=bufs, steps_done=done, max_steps=steps)
    torch.cuda.synchronize()
    _check_blocks(env, bufs, done, steps, [(0, 128), (N // 2 - 64, 128), (N - 128, 128)], SEED, base)
    # the shard's envs are the same envs as in a smaller handle at those ids
    part = BatchedSalpEnv(256, params=default_params(), seed=SEED, env_id_offset=base + 1000)
    dp = torch.zeros(256, dtype=torch.int64, device="cuda")
    part.rollout(4000, steps_done=dp, max_steps=steps)
    assert _bits_equal(part.get_state(), env.get_state()[:, 1000:1256].contiguous())
