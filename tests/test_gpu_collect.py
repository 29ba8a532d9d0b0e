"""salp_collect: PPO's collect_rollouts with the policy evaluated inside the
chained simulation kernel (include/salp.h, ppo.PPO(collect="chained")).

The kernel's buffers are checked against an independent replay:
* policy outputs: values and log-probs against the torch ActorCritic on the
  recorded observations and actions (float32 tolerance: the kernel's MLP sums
  in a different order than hipBLASLt), the exploration noise against N(0, 1);
* environment: a twin handle started from the same state and stepped
  lock-step with salp_step on the kernel's clipped actions reproduces every
  observation, reward, episode start, guard reset, the final observations and
  the whole state bit for bit (up to NaN payloads);
* rewards: SB3's timeout bootstrap gamma * V(terminal obs) where an episode
  was truncated and not terminated, 0 where the divergence guard fired;
* a policy that makes many zero-tick cycles (a boundary then leaves lanes to
  the next chunk, SALP_COLLECT_REP_MIN) on both rollout kernels.
"""
import numpy as np
import pytest
import torch

from grasp_lab_salp_amd._abi import INFO, default_params
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
from grasp_lab_salp_amd.ppo import DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS, PPO, ActorCritic, pack_policy
from grasp_lab_salp_amd.vec_env import SalpVecEnv

pytestmark = pytest.mark.gpu


def _cpu(t):
    return t.detach().cpu().numpy()


def _policy(seed, obs_dim=10):
    torch.manual_seed(seed)
    pol = ActorCritic(obs_dim, 3).cuda()
    with torch.no_grad():
        pol.action_net.weight.mul_(60.0)   # actions spread over the box, not ~ the mean
        pol.log_std.copy_(torch.tensor([-0.7, -0.4, -0.2]))
    return pol


def _buffers(n_steps, n, obs_dim):
    z = lambda *s: torch.full(s, -7.0, dtype=torch.float32, device="cuda")  # noqa: E731
    return {"obs": z(n_steps, n, obs_dim), "actions": z(n_steps, n, 3), "rewards": z(n_steps, n),
            "episode_starts": z(n_steps, n), "values": z(n_steps, n), "log_probs": z(n_steps, n)}


def _equal_up_to_nan_payload(a, b):
    a, b = np.asarray(a), np.asarray(b)
    both = np.isnan(a) & np.isnan(b)
    same = (a.view(np.int64 if a.dtype == np.float64 else np.int32)
            == b.view(np.int64 if b.dtype == np.float64 else np.int32))
    return bool(np.all(same | both))


ALL_RAND = dict(dynamics=True, disturbances=True, actions=True, observations=True, latency=True)


@pytest.mark.parametrize("n,n_steps,gamma,rand,zero_tick,kernel", [
    (300, 7, 0.99, False, False, -1), (1024, 5, 0.9, False, False, -1), (500, 6, 0.99, True, False, -1),
    (700, 12, 0.99, False, True, 1), (700, 12, 0.99, False, True, 0), (700, 12, 0.99, False, True, 2)])
def test_collect_replays_on_the_lockstep_path(n, n_steps, gamma, rand, zero_tick, kernel):
    """rand: every randomisation switch on (k_rollout<RAND, POL>; the twin's
    salp_step draws from the same Philox streams)."""
    p = default_params()
    p.max_cycles = 3        # timeouts inside the collection: the bootstrap path runs
    env = BatchedSalpEnv(n, params=p, seed=23)
    twin = BatchedSalpEnv(n, params=p, seed=23)
    if rand:
        env.set_randomization(**ALL_RAND)
        twin.set_randomization(**ALL_RAND)
    obs0 = env.reset()
    twin.set_state(env.get_state())
    env.set_rollout_kernel(kernel)
    pol = _policy(1)
    if zero_tick:
        # contraction and coast clipped to 0 for about half the draws, the yaw
        # near 0: many cycles of zero ticks, a few lanes at a time, so the
        # boundary leaves most of them to the next chunk (SALP_COLLECT_REP_MIN)
        with torch.no_grad():
            pol.action_net.weight.mul_(0.01)
            pol.action_net.bias.copy_(torch.tensor([0.0, 0.0, 0.0]))
            pol.log_std.copy_(torch.tensor([-1.0, -1.0, -3.0]))
    w = pack_policy(pol)
    bufs = _buffers(n_steps, n, env.obs_dim)
    ep_start = torch.ones(n, dtype=torch.float32, device="cuda")
    last_obs = obs0.clone()   # in/out: the observation the first step is taken on
    ep_stats = torch.zeros(4, dtype=torch.float64, device="cuda")
    diverged = torch.zeros(1, dtype=torch.int64, device="cuda")
    env.collect(w, n_steps, bufs, ep_start, last_obs, ep_stats, diverged, noise_seed=99, gamma=gamma,
                diverged_obs_abs=DIVERGED_OBS_ABS, diverged_reward_abs=DIVERGED_REWARD_ABS)
    torch.cuda.synchronize()

    # policy outputs against torch on the recorded rows
    flat_obs = bufs["obs"].reshape(-1, env.obs_dim)
    flat_act = bufs["actions"].reshape(-1, 3)
    with torch.no_grad():
        v_ref, lp_ref, _ = pol.evaluate(flat_obs, flat_act)
        mean = pol.dist(flat_obs).mean
    assert torch.allclose(bufs["values"].reshape(-1), v_ref, rtol=1e-5, atol=1e-5)
    assert torch.allclose(bufs["log_probs"].reshape(-1), lp_ref, rtol=1e-5, atol=1e-4)
    z = _cpu((flat_act - mean) / pol.log_std.exp())
    assert abs(z.mean()) < 0.05 and abs(z.std() - 1.0) < 0.05
    clipped = torch.clamp(bufs["actions"], torch.tensor([0.0, 0.0, -1.0], device="cuda"),
                          torch.tensor([1.0, 1.0, 1.0], device="cuda"))
    assert float((clipped != bufs["actions"]).float().mean()) > 0.05   # the clip matters

    # the environment side, replayed lock-step on the twin
    obs = obs0
    starts = torch.ones(n, dtype=torch.float32, device="cuda")
    stats = np.zeros(4)
    n_bad = n_trunc = 0
    for t in range(n_steps):
        assert _equal_up_to_nan_payload(_cpu(bufs["obs"][t]), _cpu(obs)), t
        assert torch.equal(bufs["episode_starts"][t], starts), t
        r = twin.step(clipped[t].contiguous(), auto_reset=True, want_terminal_obs=True)
        rew32 = r.reward.float()
        tob = r.terminal_obs
        bad = (~torch.isfinite(tob).all(1) | (tob.abs() > DIVERGED_OBS_ABS).any(1)
               | ~(r.reward.abs() <= DIVERGED_REWARD_ABS))
        done = r.terminated.bool() | r.truncated.bool()
        boot = r.truncated.bool() & ~r.terminated.bool() & ~bad
        with torch.no_grad():
            tv = pol.value(tob)
        want = torch.where(bad, torch.zeros_like(rew32), rew32)
        got = bufs["rewards"][t]
        nb = ~boot
        assert _equal_up_to_nan_payload(_cpu(got[nb]), _cpu(want[nb])), t
        assert torch.allclose(got[boot], rew32[boot] + np.float32(gamma) * tv[boot], rtol=1e-6, atol=1e-5), t
        ended = done & ~bad
        stats += [float(r.info[ended, INFO["ep_return"]].sum()), float(ended.sum()),
                  float((ended & r.terminated.bool()).sum()), float(r.info[ended, INFO["ep_len"]].sum())]
        fresh = twin.reset(mask=bad & ~done)
        obs = torch.where((bad & ~done).unsqueeze(1), fresh, r.obs)
        starts = (done | bad).float()
        n_bad += int(bad.sum())
        n_trunc += int(boot.sum())
    assert n_trunc > 0
    assert _equal_up_to_nan_payload(_cpu(last_obs), _cpu(obs))
    assert torch.equal(ep_start, starts)
    assert int(diverged) == n_bad
    assert np.allclose(_cpu(ep_stats), stats, rtol=1e-12, atol=1e-9)
    assert _equal_up_to_nan_payload(_cpu(env.get_state()), _cpu(twin.get_state()))


def test_collect_rejects_bad_buffers():
    env = BatchedSalpEnv(64, seed=1)
    pol = _policy(0)
    w = pack_policy(pol)
    bufs = _buffers(4, 64, env.obs_dim)
    args = (torch.ones(64, device="cuda"), torch.zeros((64, env.obs_dim), device="cuda"),
            torch.zeros(4, dtype=torch.float64, device="cuda"), torch.zeros(1, dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):
        env.collect(w[:-1], 4, bufs, *args)
    bad = dict(bufs, values=torch.zeros((4, 63), device="cuda"))
    with pytest.raises(ValueError):
        env.collect(w, 4, bad, *args)


def test_ppo_with_chained_collection_learns_finite():
    """PPO(collect='chained'): a few updates at 2 048 envs, finite losses,
    the buffer's episode starts and the bootstrap path exercised."""
    venv = SalpVecEnv(2048, seed=5)
    model = PPO("MlpPolicy", venv, n_steps=16, batch_size=4096, n_epochs=2, seed=3, collect="chained")
    model.learn(3 * 16 * 2048)
    assert len(model.history) == 3
    for row in model.history:
        for k, v in row.items():
            if isinstance(v, float):
                assert np.isfinite(v), (k, v)
    assert torch.isfinite(model.buf.advantages).all()


def test_ppo_collect_auto_choice():
    """collect='auto': the in-kernel collection from n_steps 256 on (the
    reference's n_steps is 2048), lock-step below."""
    venv = SalpVecEnv(256, seed=1)
    assert PPO("MlpPolicy", venv, n_steps=256, batch_size=256, seed=0).collect == "chained"
    assert PPO("MlpPolicy", venv, n_steps=32, batch_size=256, seed=0).collect == "lockstep"
