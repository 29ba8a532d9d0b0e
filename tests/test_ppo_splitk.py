"""SplitKLinear (ppo.py): forward values and gradients of nn.Linear, with the
weight gradient reduced over K slices (CPU; the GPU path is the same torch ops)."""
import torch
from torch import nn

from grasp_lab_salp_amd.ppo import ActorCritic, SplitKLinear


def _grads(layer, x, gy):
    for p in layer.parameters():
        p.grad = None
    xi = x.clone().requires_grad_(True)
    y = layer(xi)
    y.backward(gy)
    return y.detach(), xi.grad, layer.weight.grad.clone(), layer.bias.grad.clone()


def test_splitk_linear_matches_linear():
    torch.manual_seed(0)
    for dtype, tol in ((torch.float64, 1e-12), (torch.float32, 2e-5)):
        ref = nn.Linear(10, 64).to(dtype)
        sk = SplitKLinear(10, 64).to(dtype)
        sk.load_state_dict(ref.state_dict())
        x = torch.randn(8192, 10, dtype=dtype)
        gy = torch.randn(8192, 64, dtype=dtype)
        a, b = _grads(ref, x, gy), _grads(sk, x, gy)
        assert torch.equal(a[0], b[0])             # forward: the same addmm
        for u, v in zip(a[1:], b[1:]):
            assert torch.allclose(u, v, rtol=tol, atol=tol * 10)


def test_splitk_linear_small_and_ragged_batches_take_linear_path():
    sk = SplitKLinear(10, 4)
    for rows in (1, 64, 513, 8191):
        x = torch.randn(rows, 10, requires_grad=True)
        sk(x).sum().backward()
        assert x.grad.shape == (rows, 10)


def test_actor_critic_uses_splitk_layers():
    pol = ActorCritic(10, 3)
    kinds = {type(m) for m in pol.modules() if isinstance(m, nn.Linear)}
    assert kinds == {SplitKLinear}
