"""Debug: PPO collection at config 5 size (32 768 envs, 32 steps) with the
lock-step order sorted (1) and env order (0): are the buffers identical before
and after one update (HIP graph path)?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402

KEYS = ("obs", "actions", "rewards", "episode_starts", "values", "log_probs", "advantages", "returns")
runs = {}
for mode in (1, 0):
    env = SalpVecEnv(32768, seed=0, infos=False)
    env.sim.set_lockstep_order(mode)
    m = PPO("MlpPolicy", env, n_steps=32, batch_size=32768, n_epochs=10, seed=0, use_graphs=True)
    snaps = []
    for it in range(2):
        m.collect_rollouts()
        torch.cuda.synchronize()
        snaps.append({k: getattr(m.buf, k).clone() for k in KEYS})
        snaps[-1]["params"] = torch.cat([p.detach().reshape(-1) for p in m.policy.parameters()])
        m.logger = m.train()
        torch.cuda.synchronize()
        print("mode", mode, "it", it, m.logger, flush=True)
    runs[mode] = snaps
    env.close()
for it in range(2):
    for k in KEYS + ("params",):
        x, y = runs[1][it][k], runs[0][it][k]
        same = torch.equal(x.view(torch.int32), y.view(torch.int32))
        if not same:
            diff = (x != y)
            first = diff.reshape(diff.shape[0], -1).any(1).nonzero()[:1].tolist() if x.dim() > 1 else None
            print("it", it, k, "DIFFERS", int(diff.sum()), "first row", first, flush=True)
        else:
            print("it", it, k, "same", flush=True)
