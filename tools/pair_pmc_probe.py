"""One step-capped chained rollout per kernel (k_rollout, then k_rollout_pair)
at N envs, for rocprofv3 --pmc passes comparing the two (tools/gpu_pmc_pair.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def main():
    n, k = int(os.environ.get("N", 32768)), int(os.environ.get("K", 16))
    for kern in (0, 1):
        env = BatchedSalpEnv(n, seed=0)
        env.set_rollout_kernel(kern)
        sd = torch.zeros(n, dtype=torch.int64, device="cuda")
        env.rollout(10 ** 8, steps_done=sd, max_steps=k)
        torch.cuda.synchronize()
        env.close()


if __name__ == "__main__":
    main()
