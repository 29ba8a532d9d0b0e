import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
def run(kernel, budget, chunk):
    env = BatchedSalpEnv(1, params=default_params(), seed=11)
    env.set_rollout_kernel(kernel)
    done = torch.zeros(1, dtype=torch.int64, device="cuda")
    env.rollout(budget, steps_done=done, max_steps=1, chunk=chunk)
    s = env.get_state().cpu().numpy()[:, 0]
    env.close()
    return s
for chunk in (64,):
    for budget in (64, 128, 192, 320, 640):
        a, b = run(0, budget, chunk), run(2, budget, chunk)
        diff = [FIELDS[f] for f in range(len(a)) if a[f] != b[f] and not (np.isnan(a[f]) and np.isnan(b[f]))]
        print(budget, "ct", a[FIELD["cycle_time"]], b[FIELD["cycle_time"]], "diff", diff[:10])
        for f in ("eta0", "eta2", "pw0", "pw1", "w2", "v0"):
            print("    ", f, a[FIELD[f]], b[FIELD[f]])
