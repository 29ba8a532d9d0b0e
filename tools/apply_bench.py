"""k_mlp_apply alone (salp_ppo_mlp_apply: clip_grad_norm_ + Adam over the
64-64 MlpPolicy's flat gradient): microseconds per call, back to back on one
stream (HIP events over REPS calls).  SALP_LIB selects a variant build."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.ppo import ActorCritic  # noqa: E402


def main():
    L = _lib.load()
    od = 10
    pol = ActorCritic(od, 3).cuda()
    ts = [pol.pi_net[0].weight, pol.pi_net[0].bias, pol.pi_net[2].weight, pol.pi_net[2].bias,
          pol.action_net.weight, pol.action_net.bias, pol.log_std,
          pol.vf_net[0].weight, pol.vf_net[0].bias, pol.vf_net[2].weight, pol.vf_net[2].bias,
          pol.value_net.weight, pol.value_net.bias]
    P = L.salp_ppo_mlp_num_params(od)
    g = torch.randn(P, device="cuda") * 0.1
    m, v = torch.zeros(P, device="cuda"), torch.zeros(P, device="cuda")
    step, gn = torch.zeros(1, device="cuda"), torch.zeros(1, device="cuda")
    a = _lib.SalpPpoAdam(obs_dim=od, grads=g.data_ptr(), exp_avg=m.data_ptr(), exp_avg_sq=v.data_ptr(),
                         step=step.data_ptr(), grad_norm=gn.data_ptr(), lr=3e-4, beta1=0.9, beta2=0.999, eps=1e-5,
                         max_grad_norm=0.5)
    for i, t in enumerate(ts):
        a.params[i] = t.data_ptr()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    reps = int(os.environ.get("REPS", 2000))
    for _ in range(20):
        _lib.check(L.salp_ppo_mlp_apply(ctypes.byref(a), stream))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.salp_ppo_mlp_apply(ctypes.byref(a), stream)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.environ.get("SALP_LIB", "product"), "us_per_call": e0.elapsed_time(e1) * 1e3 / reps,
                      "params": P}), flush=True)


if __name__ == "__main__":
    main()
