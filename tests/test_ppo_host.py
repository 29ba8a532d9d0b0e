"""Host-side PPO pieces on the CPU: SB3's timeout bootstrap, the learner's
divergence guard and the per-rank exploration-noise generator."""
import torch

from grasp_lab_salp_amd.ppo import (DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS, ActorCritic, diverged_mask,
                                    sampling_generator, timeout_bootstrap)


def test_timeout_bootstrap_only_for_truncated_not_terminated():
    rew = torch.tensor([1.0, 2.0, 3.0, 4.0])
    term = torch.tensor([False, True, True, False])
    trunc = torch.tensor([True, True, False, False])
    tv = torch.tensor([10.0, 20.0, 30.0, 40.0])
    out = timeout_bootstrap(rew, term, trunc, tv, 0.99)
    # env 0: cut by the time limit -> r + gamma V(terminal obs); env 1: a real
    # end that also hit the limit -> no bootstrap (SB3 checks not terminated)
    assert torch.equal(out, torch.tensor([1.0 + 0.99 * 10.0, 2.0, 3.0, 4.0]))


def test_diverged_mask_catches_huge_finite_values():
    obs = torch.zeros(6, 10)
    rew = torch.zeros(6)
    obs[1, 2] = float("nan")
    rew[2] = float("inf")
    obs[3, 4] = 2 * DIVERGED_OBS_ABS           # finite but diverging velocity
    rew[4] = -2 * DIVERGED_REWARD_ABS          # finite but diverging sideslip penalty
    rew[5] = 1500.0                            # success bonus + progress: legitimate
    assert diverged_mask(obs, rew).tolist() == [False, True, True, True, True, False]


def test_sampling_generator_single_process_is_seed_stream():
    g = sampling_generator(5, "cpu")
    h = torch.Generator().manual_seed(5)
    assert torch.equal(torch.randn(8, generator=g), torch.randn(8, generator=h))


def test_act_with_generator_is_mean_plus_std_noise():
    torch.manual_seed(0)
    pol = ActorCritic(10, 3)
    obs = torch.randn(4, 10)
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    a, v, lp = pol.act(obs, generator=g1)
    d = pol.dist(obs)
    eps = torch.randn(4, 3, generator=g2)
    assert torch.allclose(a, d.mean + d.stddev * eps)
    assert torch.allclose(lp, d.log_prob(a).sum(-1))


def test_pack_policy_layout():
    """ppo.pack_policy writes the ActorCritic into salp_collect's layout
    (include/salp.h SALP_POLICY_*): first-layer columns zero-padded to
    OBS_DIM_MAX, every other tensor flattened [out][in] at its offset."""
    import torch

    from grasp_lab_salp_amd._abi import OBS_DIM_MAX, POLICY_OFFSETS, POLICY_SIZE
    from grasp_lab_salp_amd.ppo import ActorCritic, pack_policy
    torch.manual_seed(0)
    pol = ActorCritic(10, 3)
    with torch.no_grad():
        pol.log_std.copy_(torch.tensor([0.1, -0.2, 0.3]))
    w = pack_policy(pol)
    assert w.shape == (POLICY_SIZE,) and w.dtype == torch.float32

    def part(name):
        off, size = POLICY_OFFSETS[name]
        return w[off:off + size]

    w1 = part("pi_w1").view(64, OBS_DIM_MAX)
    assert torch.equal(w1[:, :10], pol.pi_net[0].weight) and not w1[:, 10:].any()
    assert torch.equal(part("vf_w1").view(64, OBS_DIM_MAX)[:, :10], pol.vf_net[0].weight)
    assert torch.equal(part("pi_w2").view(64, 64), pol.pi_net[2].weight)
    assert torch.equal(part("vf_b2"), pol.vf_net[2].bias)
    assert torch.equal(part("act_w").view(3, 64), pol.action_net.weight)
    assert torch.equal(part("act_b"), pol.action_net.bias)
    assert torch.equal(part("log_std"), pol.log_std.detach())
    assert torch.equal(part("val_w"), pol.value_net.weight.view(-1))
    assert torch.equal(part("val_b"), pol.value_net.bias)
