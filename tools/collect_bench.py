"""salp_collect vs the plain chained rollout (same per-env step cap) vs
lock-step salp_step, env-steps/s.  N="32768 65536" K=32 python tools/collect_bench.py
(KERNEL = salp_set_rollout_kernel mode, default -1: the auto choice)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from grasp_lab_salp_amd.ppo import ActorCritic, pack_policy  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3


def main():
    k = int(os.environ.get("K", 32))
    for n in [int(x) for x in os.environ.get("N", "32768 65536").split()]:
        env = BatchedSalpEnv(n, seed=0)
        env.set_rollout_kernel(int(os.environ.get("KERNEL", "-1")))
        pol = ActorCritic(env.obs_dim, 3).cuda()
        w = pack_policy(pol)
        z = lambda *s: torch.zeros(s, dtype=torch.float32, device="cuda")  # noqa: E731
        bufs = {"obs": z(k, n, env.obs_dim), "actions": z(k, n, 3), "rewards": z(k, n), "episode_starts": z(k, n),
                "values": z(k, n), "log_probs": z(k, n)}
        extra = (torch.ones(n, device="cuda"), z(n, env.obs_dim), torch.zeros(4, dtype=torch.float64, device="cuda"),
                 torch.zeros(1, dtype=torch.int64, device="cuda"))
        out = {"n_envs": n, "k": k}
        for rep in range(2):
            # salp_collect acts first on last_obs (in/out): the env's reset
            # observation, as PPO hands it over (the other legs moved the state)
            extra[1].copy_(env.reset())
            extra[0].fill_(1.0)
            out[f"collect_{rep}"] = n * k / timed(lambda: env.collect(w, k, bufs, *extra, diverged_obs_abs=1e3,
                                                                       diverged_reward_abs=1e4)) / 1e6
            sd = torch.zeros(n, dtype=torch.int64, device="cuda")
            out[f"rollout_cap_{rep}"] = n * k / timed(lambda: env.rollout(10 ** 8, steps_done=sd, max_steps=k)) / 1e6
            acts = [torch.rand((n, 3), device="cuda") for _ in range(k)]
            out[f"lockstep_step_{rep}"] = n * k / timed(lambda: [env.step(a, auto_reset=True) for a in acts]) / 1e6
            out[f"step_random_{rep}"] = n * k / timed(lambda: env.step_random(k)) / 1e6
        print(json.dumps({a: (round(b, 2) if isinstance(b, float) else b) for a, b in out.items()}), flush=True)
        env.close()


if __name__ == "__main__":
    main()
