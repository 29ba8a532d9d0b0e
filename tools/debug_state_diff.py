"""Debug: run the bench's rollout sequence with the in-tree library and dump
the field-major state (get_state) to gpurun_out/state_<tag>.npy."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd._abi import default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402

n = int(os.environ.get("N", 65536))
budget = int(os.environ.get("BUDGET", 8192))
launches = int(os.environ.get("LAUNCHES", 2))
env = BatchedSalpEnv(n, params=default_params(), seed=0)
cap = 16
bufs = {"obs": torch.zeros((cap, n, env.obs_dim), dtype=torch.float32, device="cuda"),
        "actions": torch.zeros((cap, n, 3), dtype=torch.float32, device="cuda"),
        "rewards": torch.zeros((cap, n), dtype=torch.float32, device="cuda"),
        "dones": torch.zeros((cap, n), dtype=torch.uint8, device="cuda")}
done = torch.zeros(n, dtype=torch.int64, device="cuda")
s0 = env.get_state().cpu().numpy()
for _ in range(launches):
    env.rollout(budget, buffers=bufs, steps_done=done, chunk=128)
torch.cuda.synchronize()
s1 = env.get_state().cpu().numpy()
tag = os.environ.get("TAG", "x")
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/state1_{tag}.npy", s1.astype(np.float64))
print(tag, "done", int(done.sum()), "n_obst", np.unique(s1[76]), flush=True)
