"""Where does salp_collect's replay (tests/test_gpu_collect.py) diverge?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_collect import _buffers, _cpu, _policy  # noqa: E402

from grasp_lab_salp_amd._abi import FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from grasp_lab_salp_amd.ppo import DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS, pack_policy  # noqa: E402

n, n_steps = 300, 7
p = default_params()
p.max_cycles = int(os.environ.get("MAXC", 3))
env = BatchedSalpEnv(n, params=p, seed=23)
obs0 = env.reset()
twin = BatchedSalpEnv(n, params=p, seed=23)
env_state0 = env.get_state().clone()
twin.set_state(env_state0)
snaps = []
pol = _policy(1)
w = pack_policy(pol)
bufs = _buffers(n_steps, n, env.obs_dim)
ep_start = torch.ones(n, dtype=torch.float32, device="cuda")
last_obs = torch.zeros((n, env.obs_dim), device="cuda")
ep_stats = torch.zeros(2, dtype=torch.float64, device="cuda")
diverged = torch.zeros(1, dtype=torch.int64, device="cuda")
env.collect(w, n_steps, bufs, ep_start, last_obs, ep_stats, diverged, noise_seed=99, gamma=0.99,
            diverged_obs_abs=DIVERGED_OBS_ABS, diverged_reward_abs=DIVERGED_REWARD_ABS)
torch.cuda.synchronize()
clipped = torch.clamp(bufs["actions"], torch.tensor([0.0, 0.0, -1.0], device="cuda"),
                      torch.tensor([1.0, 1.0, 1.0], device="cuda"))
obs = obs0
prev_done = np.zeros(n, bool)
for t in range(n_steps):
    a, b = _cpu(bufs["obs"][t]), _cpu(obs)
    bad_rows = np.nonzero(~(np.isclose(a, b, rtol=0, atol=0, equal_nan=True)).all(1))[0]
    print("t", t, "mismatch envs", len(bad_rows), bad_rows[:10].tolist(), "prev_done", prev_done[bad_rows[:10]].tolist())
    for i in bad_rows[:3]:
        print("   env", i, "kernel", a[i].tolist(), "\n   twin  ", b[i].tolist())
    snaps.append(twin.get_state().clone())
    r = twin.step(clipped[t].contiguous(), auto_reset=True, want_terminal_obs=True)
    tob = r.terminal_obs
    bad = (~torch.isfinite(tob).all(1) | (tob.abs() > DIVERGED_OBS_ABS).any(1) | ~(r.reward.abs() <= DIVERGED_REWARD_ABS))
    done = r.terminated.bool() | r.truncated.bool()
    fresh = twin.reset(mask=bad & ~done)
    obs = torch.where((bad & ~done).unsqueeze(1), fresh, r.obs)
    prev_done = _cpu(done | bad)
    print("   done", int(done.sum()), "bad", int(bad.sum()), "trunc", int(r.truncated.sum()))
ga, gb = _cpu(env.get_state()), _cpu(twin.get_state())
d = ~np.isclose(ga, gb, rtol=0, atol=0, equal_nan=True)
print("state fields differing:", [FIELDS[f] for f in np.nonzero(d.any(1))[0]][:30], "envs", int(d.any(0).sum()))

# replay env ENV's step T alone: oracle vs lock-step vs salp_collect on a 1-env handle
from oracle import oracle as orc  # noqa: E402
E, T = int(os.environ.get("ENV", 79)), int(os.environ.get("T", 3))
s = snaps[T][:, E:E + 1].contiguous()
act = clipped[T][E:E + 1].contiguous()
print("action", act.tolist(), "raw", bufs["actions"][T][E].tolist())
o = orc.Oracle(p, 1, seed=23, env_offset=E)
o.state[:] = _cpu(s)
ro = o.step(_cpu(act), auto_reset=True)
one = BatchedSalpEnv(1, params=p, seed=23, env_id_offset=E)
one.set_state(s)
r1 = one.step(act, auto_reset=True)
col = BatchedSalpEnv(1, params=p, seed=23, env_id_offset=E)
col.set_state(s)
b1 = _buffers(1, 1, env.obs_dim)
col.collect(w, 1, b1, torch.zeros(1, device="cuda"), torch.zeros((1, env.obs_dim), device="cuda"),
            torch.zeros(2, dtype=torch.float64, device="cuda"), torch.zeros(1, dtype=torch.int64, device="cuda"),
            noise_seed=99, gamma=0.99, diverged_obs_abs=DIVERGED_OBS_ABS, diverged_reward_abs=DIVERGED_REWARD_ABS)
print("collect action", b1["actions"][0, 0].tolist())
print("obs oracle  ", ro["obs"][0].tolist())
print("obs lockstep", _cpu(r1.obs)[0].tolist())
so, sl, sc = o.state[:, 0], _cpu(one.get_state())[:, 0], _cpu(col.get_state())[:, 0]
for f in range(len(FIELDS)):
    if not (so[f] == sl[f] == sc[f]) and not (np.isnan(so[f]) and np.isnan(sl[f]) and np.isnan(sc[f])):
        print(f"  {FIELDS[f]:12s} oracle {so[f]!r} lockstep {sl[f]!r} collect {sc[f]!r}")
print("pre-step", {k: float(s[FIELDS.index(k), 0]) for k in ("cycle", "phase", "contraction", "refill_time", "jet_time", "coast_time", "geom32", "contr32", "length", "width", "cycle_time", "pending")})
