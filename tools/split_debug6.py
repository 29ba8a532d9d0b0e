import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
def run(kernel, budget, n=1, seed=11):
    env = BatchedSalpEnv(n, params=default_params(), seed=seed)
    env.set_rollout_kernel(kernel)
    done = torch.zeros(n, dtype=torch.int64, device="cuda")
    env.rollout(budget, steps_done=done, max_steps=3, chunk=64)
    s = env.get_state().cpu().numpy()
    env.close()
    return s
ref = run(0, 64)
print(os.environ.get("SALP_LIB", "product"), "k_rollout pw0", ref[FIELD["pw0"], 0], [run(2, 64)[FIELD["pw0"], 0] for _ in range(3)])
a, b = run(0, 10 ** 7, n=4096), run(2, 10 ** 7, n=4096)
d = (a.view(np.int64) != b.view(np.int64)) & ~(np.isnan(a) & np.isnan(b))
print("4096 envs x 3 steps: envs differing", int(d.any(0).sum()))
