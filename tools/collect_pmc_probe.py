"""salp_collect at BASELINE configs[4]'s size (32 768 envs, n_steps 256, the
PPO leg's defaults: the auto two-wave kernel, k_rollout_split<true> from round 6, chunk 176) with a fresh 64-64 tanh
policy (seed 0), twice (the first dispatch is the warm-up the summary drops),
for rocprofv3 --pmc passes (tools/gpu_pmc_collect.sh PROBE=1).  Prints the
env-steps and the mean ticks per env-step of the second call's sampled replay
(oracle/sampled.check_collect) so that the counts can be normalised."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from grasp_lab_salp_amd.ppo import DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS, ActorCritic, pack_policy  # noqa: E402
from oracle import sampled  # noqa: E402  (the checker, after the profiled calls)


def main():
    n, T = int(os.environ.get("N", 32768)), int(os.environ.get("T", 256))
    env = BatchedSalpEnv(n, seed=0)
    torch.manual_seed(0)
    w = pack_policy(ActorCritic(env.obs_dim, 3).cuda())
    z = lambda *s: torch.zeros(s, dtype=torch.float32, device="cuda")  # noqa: E731
    bufs = {"obs": z(T, n, env.obs_dim), "actions": z(T, n, 3), "rewards": z(T, n), "episode_starts": z(T, n),
            "values": z(T, n), "log_probs": z(T, n)}
    ep_start = torch.ones(n, device="cuda")
    last_obs = env.reset()
    stats = torch.zeros(4, dtype=torch.float64, device="cuda")
    div = torch.zeros(1, dtype=torch.int64, device="cuda")
    for call in range(2):
        if call == 1:
            state0, obs0 = env.get_state().cpu().numpy(), last_obs.cpu().numpy()
        env.collect(w, T, bufs, ep_start, last_obs, stats, div, noise_seed=1, gamma=0.99,
                    diverged_obs_abs=DIVERGED_OBS_ABS, diverged_reward_abs=DIVERGED_REWARD_ABS)
        torch.cuda.synchronize()
    # the second (profiled) call replayed on sampled blocks: its ticks per env-step
    chk = sampled.check_collect(state0, obs0, {k: bufs[k].cpu().numpy() for k in ("obs", "actions", "rewards",
                                                                                   "episode_starts")},
                                last_obs.cpu().numpy(), env.get_state().cpu().numpy(), env.params, 0,
                                guard=(DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS))
    out = {"n_envs": n, "n_steps": T, "env_steps_per_dispatch": n * T, "ticks_per_env_step": chk["ticks_per_env_step"],
           "ticks_sample_env_steps": chk["env_steps_replayed"], "parity_ok": chk["ok"],
           "policy": "fresh 64-64 tanh ActorCritic (torch seed 0), noise seed 1"}
    print(json.dumps(out))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "collect_probe.json"), "w") as f:
        json.dump(out, f)
    env.close()


if __name__ == "__main__":
    main()
