import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
for chunk in (64, 256):
    for budget in (chunk, 2 * chunk, 3 * chunk, 4 * chunk, 10 ** 7):
        env = BatchedSalpEnv(1, params=default_params(), seed=11)
        env.set_rollout_kernel(2)
        done = torch.zeros(1, dtype=torch.int64, device="cuda")
        env.rollout(budget, steps_done=done, max_steps=1, chunk=chunk)
        s = env.get_state().cpu().numpy()[:, 0]
        print("chunk", chunk, "budget", budget, "B integrated", s[FIELD["eta0"]], "slots", s[FIELD["eta1"]], "b2", s[FIELD["eta2"]],
              "B ct", s[FIELD["pw0"]], "c0", s[FIELD["pw2"]], "| A ct", s[FIELD["cycle_time"]], "done", int(done[0]), flush=True)
        env.close()
