"""salp_step_random(k) env-steps/s for several k (one process per build mode:
SALP_STEP_RANDOM_LOCKSTEP=1 forces the lock-step kernel for every k).

    K="1 2 4 8 16 32" N=65536 python tools/step_random_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def main():
    n = int(os.environ.get("N", 65536))
    env = BatchedSalpEnv(n, seed=0)
    env.step_random(1)
    out = {"n_envs": n, "lockstep_forced": os.environ.get("SALP_STEP_RANDOM_LOCKSTEP") == "1",
           "chunk": os.environ.get("SALP_STEP_RANDOM_CHUNK", "128")}
    for k in [int(x) for x in os.environ.get("K", "1 2 4 8 16 32").split()]:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step_random(k)
        e1.record()
        torch.cuda.synchronize()
        out[f"k{k}"] = round(n * k / (e0.elapsed_time(e1) / 1e3) / 1e6, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
