"""Lock-step env-steps/s (salp_step_random, one env-step per env per launch
unless STEPS says otherwise) in env order vs sorted by predicted cycle length.

    N="65536 262144" STEPS=1 python tools/lockstep_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def rate(env, steps, reps):
    env.step_random(steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        env.step_random(steps)
    e1.record()
    torch.cuda.synchronize()
    return env.n_envs * steps * reps / (e0.elapsed_time(e1) / 1e3)


def main():
    steps = int(os.environ.get("STEPS", 1))
    reps = int(os.environ.get("REPS", 6))
    for n in [int(x) for x in os.environ.get("N", "65536 262144").split()]:
        out = {"n_envs": n, "steps_per_launch": steps}
        for mode in (0, 1):
            env = BatchedSalpEnv(n, seed=0)
            env.set_lockstep_order(mode)
            out["sorted" if mode else "env_order"] = rate(env, steps, reps)
            env.close()
        out["speedup"] = out["sorted"] / out["env_order"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
