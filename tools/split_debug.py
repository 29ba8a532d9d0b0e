"""Debug: k_rollout vs k_rollout_split on small rollouts (state fields that
differ, per max_steps)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def run(kernel, n, steps, seed=11, budget=10 ** 7, chunk=64):
    env = BatchedSalpEnv(n, params=default_params(), seed=seed)
    env.set_rollout_kernel(kernel)
    done = torch.zeros(n, dtype=torch.int64, device="cuda")
    env.rollout(budget, steps_done=done, max_steps=steps, chunk=chunk)
    torch.cuda.synchronize()
    s = env.get_state().cpu().numpy()
    env.close()
    return s, done.cpu().numpy()


for n in (1, 64, 200):
    for steps in (1, 2, 3):
        for chunk in (64, 2000):
            a, da = run(0, n, steps, chunk=chunk)
            b, db = run(2, n, steps, chunk=chunk)
            d = (a.view(np.int64) != b.view(np.int64)) & ~(np.isnan(a) & np.isnan(b))
            fields = [FIELDS[f] for f in np.nonzero(d.any(1))[0]]
            envs = np.nonzero(d.any(0))[0]
            print(f"n={n} steps={steps} chunk={chunk} steps_equal={np.array_equal(da, db)} envs_diff={len(envs)} "
                  f"fields={fields[:12]}", flush=True)
            if len(envs):
                j = envs[0]
                for f in np.nonzero(d[:, j])[0][:6]:
                    print("   ", FIELDS[f], a[f, j], b[f, j], "ct", a[FIELDS.index('cycle_time'), j], b[FIELDS.index('cycle_time'), j])
