import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
for kernel in (0, 1, 2):
    for chunk in (64, 2000):
        env = BatchedSalpEnv(1, params=default_params(), seed=11)
        env.set_rollout_kernel(kernel)
        env.pair_timeouts()
        done = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        t = time.time()
        env.rollout(10 ** 7, steps_done=done, max_steps=1, chunk=chunk)
        torch.cuda.synchronize()
        dt = time.time() - t
        s = env.get_state().cpu().numpy()
        print(kernel, chunk, "time %.4f" % dt, "timeouts", env.pair_timeouts(), "eta2", s[FIELD["eta2"], 0], "ang2", s[FIELD["ang2"], 0], flush=True)
        env.close()
