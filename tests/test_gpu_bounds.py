"""Every lock-step C-ABI call writes only inside the buffers it is given: the
outputs sit in the middle of larger device buffers whose margins hold a
canary pattern, and the canaries must survive many steps with auto-reset,
masked resets, divergence and the sorted launch order."""
import ctypes

import numpy as np
import pytest
import torch

from grasp_lab_salp_amd import _lib
from grasp_lab_salp_amd._abi import INFO_DIM
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv

pytestmark = pytest.mark.gpu

MARGIN = 1 << 16   # bytes of canary on either side of every buffer


class Guarded:
    """A [shape] dtype tensor inside a byte buffer with canary margins."""

    def __init__(self, shape, dtype, fill=0):
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        self.raw = torch.full((MARGIN + n + MARGIN,), 0xA5, dtype=torch.uint8, device="cuda")
        self.t = self.raw[MARGIN:MARGIN + n].view(dtype).view(shape)
        self.t.fill_(fill)

    def ptr(self):
        return ctypes.c_void_p(self.t.data_ptr())

    def intact(self):
        return bool((self.raw[:MARGIN] == 0xA5).all()) and bool((self.raw[-MARGIN:] == 0xA5).all())


@pytest.mark.parametrize("n", [300, 4096])
def test_step_and_reset_write_inside_their_buffers(n):
    env = BatchedSalpEnv(n, seed=5)
    L = _lib.load()
    od = env.obs_dim
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    obs0 = Guarded((n, od), torch.float32)
    _lib.check(L.salp_reset(env._h, None, obs0.ptr(), st), env._h)
    g = torch.Generator(device="cuda").manual_seed(3)
    bufs = []
    for t in range(12):
        a = Guarded((n, 3), torch.float32)
        a.t.copy_(torch.rand((n, 3), generator=g, device="cuda") * torch.tensor([1.0, 1.0, 2.0], device="cuda")
                  - torch.tensor([0.0, 0.0, 1.0], device="cuda"))
        if t == 3:   # jet_time < dt: the reference's own blow-up, so NaN flows through the outputs
            a.t[: n // 8, 0] = 1.0
            a.t[: n // 8, 1] = 0.0
        outs = {"obs": Guarded((n, od), torch.float32), "rew": Guarded((n,), torch.float64),
                "term": Guarded((n,), torch.uint8), "trunc": Guarded((n,), torch.uint8),
                "tobs": Guarded((n, od), torch.float32), "info": Guarded((n, INFO_DIM), torch.float64)}
        _lib.check(L.salp_step(env._h, a.ptr(), outs["obs"].ptr(), outs["rew"].ptr(), outs["term"].ptr(),
                               outs["trunc"].ptr(), 1, outs["tobs"].ptr(), outs["info"].ptr(), st), env._h)
        m = Guarded((n,), torch.uint8)
        m.t[::3] = 1
        ro = Guarded((n, od), torch.float32)
        _lib.check(L.salp_reset(env._h, m.ptr(), ro.ptr(), st), env._h)
        bufs += [a, m, ro, *outs.values()]
    torch.cuda.synchronize()
    bad = [i for i, b in enumerate(bufs) if not b.intact()]
    assert not bad and obs0.intact(), f"writes outside buffers {bad}"
    env.close()


def test_rollout_step_random_and_collect_write_inside_their_buffers():
    """The chained kernels (salp_rollout with every buffer, salp_step_random on
    both of its paths, salp_collect with the guard on) over several launches
    with auto-resets and diverged envs."""
    from grasp_lab_salp_amd.ppo import ActorCritic, pack_policy
    n, cap, K = 1000, 5, 12
    env = BatchedSalpEnv(n, seed=9)
    L = _lib.load()
    od = env.obs_dim
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    bufs = []
    B = _lib.SalpRolloutBuffers()
    g = {"obs": Guarded((cap, n, od), torch.float32), "obs_before": Guarded((cap, n, od), torch.float32),
         "actions": Guarded((cap, n, 3), torch.float32), "rewards": Guarded((cap, n), torch.float32),
         "dones": Guarded((cap, n), torch.uint8), "steps_done": Guarded((n,), torch.int64)}
    for k, v in g.items():
        setattr(B, k, v.t.data_ptr())
    B.capacity, B.max_steps, B.chunk = cap, 0, 97
    for _ in range(3):
        _lib.check(L.salp_rollout(env._h, 3000, ctypes.byref(B), st), env._h)
    bufs += list(g.values())
    for k in (1, 40):   # lock-step kernel, then the chained path with a step cap
        rs = Guarded((n,), torch.float64)
        _lib.check(L.salp_step_random(env._h, k, rs.ptr(), st), env._h)
        bufs.append(rs)
    pol = ActorCritic(od, 3).cuda()
    w = Guarded((pack_policy(pol).numel(),), torch.float32)
    pack_policy(pol, w.t)
    R = _lib.SalpPolicyRollout(weights=w.t.data_ptr(), noise_seed=3, gamma=0.99, diverged_obs_abs=1e3,
                               diverged_reward_abs=1e4, n_steps=K)
    c = {"obs": Guarded((K, n, od), torch.float32), "actions": Guarded((K, n, 3), torch.float32),
         "rewards": Guarded((K, n), torch.float32), "episode_starts": Guarded((K, n), torch.float32),
         "values": Guarded((K, n), torch.float32), "log_probs": Guarded((K, n), torch.float32),
         "episode_start": Guarded((n,), torch.float32, 1.0), "last_obs": Guarded((n, od), torch.float32),
         "ep_stats": Guarded((4,), torch.float64), "diverged": Guarded((1,), torch.int64)}
    _lib.check(L.salp_reset(env._h, None, c["last_obs"].ptr(), st), env._h)
    for k, v in c.items():
        setattr(R, k, v.t.data_ptr())
    for _ in range(2):
        _lib.check(L.salp_collect(env._h, ctypes.byref(R), st), env._h)
    bufs += [w, *c.values()]
    torch.cuda.synchronize()
    bad = [i for i, b in enumerate(bufs) if not b.intact()]
    assert not bad, f"writes outside buffers {bad}"
    assert int(g["steps_done"].t.min()) > 0
    env.close()
