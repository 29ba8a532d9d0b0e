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
