"""Fused PPO loss head (salp_ppo_loss) against the torch expression of SB3's
PPO loss (ppo.torch_ppo_loss): loss terms and gradients, float32 tolerance."""
import pytest
import torch

from grasp_lab_salp_amd.ppo import ppo_loss, torch_ppo_loss

pytestmark = pytest.mark.gpu


def _case(B, seed, ratio_spread):
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    mu = r(B, 3) * 0.5
    log_std = r(3) * 0.3
    value = r(B) * 10
    actions = mu + r(B, 3) * log_std.exp()
    d = torch.distributions.Normal(mu, log_std.exp().expand_as(mu))
    old = d.log_prob(actions).sum(-1) + r(B) * ratio_spread   # ratios around 1, some clipped
    adv = r(B) * 100 + 3
    ret = value + r(B) * 5
    return mu, log_std, value, actions, old, adv, ret


@pytest.mark.parametrize("B,normalize", [(32768, True), (32768, False), (1000, True), (1, True)])
def test_fused_loss_matches_torch(B, normalize):
    args = _case(B, 7, 0.3)
    leaves = [t.clone().requires_grad_(True) for t in args[:3]]
    leaves2 = [t.clone().requires_grad_(True) for t in args[:3]]
    kw = dict(clip_range=0.2, ent_coef=0.01, vf_coef=0.5, normalize_advantage=normalize)
    loss, st = ppo_loss(*leaves, *args[3:], **kw)
    loss.backward()
    loss_t, st_t = torch_ppo_loss(*leaves2, *args[3:], **kw)
    loss_t.backward()
    assert torch.allclose(st, st_t, rtol=1e-4, atol=1e-5), (st, st_t)
    assert torch.allclose(loss, loss_t, rtol=1e-4, atol=1e-5)
    for a, b in zip(leaves, leaves2):
        scale = b.grad.abs().max().item() + 1e-30
        assert (a.grad - b.grad).abs().max().item() <= 1e-4 * scale + 1e-7, (a.grad, b.grad)


def test_fused_loss_rejects_bad_shapes():
    args = _case(64, 1, 0.1)
    with pytest.raises(ValueError):
        ppo_loss(args[0][:, :2], *args[1:], clip_range=0.2, ent_coef=0.0, vf_coef=0.5, normalize_advantage=True)
