"""Which randomisation switch makes salp_collect (k_rollout<RAND, POL>) differ
from salp_step on a twin handle and from the oracle: one short collection per
switch, the final states compared field by field (GPU; a debugging aid of
tests/test_gpu_collect.py)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from grasp_lab_salp_amd.ppo import DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS, ActorCritic, pack_policy  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def differ(a, b):
    a, b = np.asarray(a), np.asarray(b)
    d = (a.view(np.int64) != b.view(np.int64)) & ~(np.isnan(a) & np.isnan(b))
    return {FIELDS[f]: int(d[f].sum()) for f in np.nonzero(d.any(1))[0]}


def run(flags, n=500, n_steps=int(os.environ.get("NSTEPS", 2))):
    p = default_params()
    p.max_cycles = 3
    env = BatchedSalpEnv(n, params=p, seed=23)
    twin = BatchedSalpEnv(n, params=p, seed=23)
    if flags:
        env.set_randomization(**flags)
        twin.set_randomization(**flags)
    obs0 = env.reset()
    twin.set_state(env.get_state())
    o = orc.Oracle(env.params if hasattr(env, "params") else p, n, seed=23)
    if flags:
        o.set_randomization(**flags)
    o.state[:] = env.get_state().cpu().numpy()
    torch.manual_seed(1)
    pol = ActorCritic(env.obs_dim, 3).cuda()
    with torch.no_grad():
        pol.action_net.weight.mul_(60.0)
        pol.log_std.copy_(torch.tensor([-0.7, -0.4, -0.2]))
    w = pack_policy(pol)
    z = lambda *s: torch.full(s, -7.0, dtype=torch.float32, device="cuda")  # noqa: E731
    bufs = {"obs": z(n_steps, n, env.obs_dim), "actions": z(n_steps, n, 3), "rewards": z(n_steps, n),
            "episode_starts": z(n_steps, n), "values": z(n_steps, n), "log_probs": z(n_steps, n)}
    env.collect(w, n_steps, bufs, torch.ones(n, device="cuda"), obs0.clone(),
                torch.zeros(4, dtype=torch.float64, device="cuda"), torch.zeros(1, dtype=torch.int64, device="cuda"),
                noise_seed=99, gamma=0.99, diverged_obs_abs=DIVERGED_OBS_ABS, diverged_reward_abs=DIVERGED_REWARD_ABS)
    torch.cuda.synchronize()
    lo = torch.tensor([0.0, 0.0, -1.0], device="cuda")
    hi = torch.tensor([1.0, 1.0, 1.0], device="cuda")
    clipped = torch.clamp(bufs["actions"], lo, hi)
    for t in range(n_steps):
        twin.step(clipped[t].contiguous(), auto_reset=True)
        o.step(clipped[t].cpu().numpy(), auto_reset=True)
    torch.cuda.synchronize()
    se, st = env.get_state().cpu().numpy(), twin.get_state().cpu().numpy()
    from grasp_lab_salp_amd._abi import FIELD
    extra = {}
    for f in ("cd", "dfr", "amf0", "rng_ctl", "rng_tick", "ouf0", "step_count"):
        u, c = np.unique(se[FIELD[f]], return_counts=True)
        extra[f + "_collect"] = [[float(x), int(k)] for x, k in zip(u[:6], c[:6])]
        u, c = np.unique(st[FIELD[f]], return_counts=True)
        extra[f + "_twin"] = [[float(x), int(k)] for x, k in zip(u[:6], c[:6])]
    return {**extra, "collect_vs_twin": differ(se, st), "twin_vs_oracle": differ(st, o.state),
            "collect_vs_oracle": differ(se, o.state)}


def main():
    cases = {"none": {}}
    for k in ("dynamics", "disturbances", "actions", "observations", "latency"):
        cases[k] = {k: True}
    cases["all"] = {k: True for k in ("dynamics", "disturbances", "actions", "observations", "latency")}
    only = os.environ.get("CASES")
    for name, flags in cases.items():
        if only and name not in only.split(","):
            continue
        print(json.dumps({"case": name, **run(flags)}), flush=True)


if __name__ == "__main__":
    main()
