import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
env = BatchedSalpEnv(1, params=default_params(), seed=11)
env.set_rollout_kernel(2)
done = torch.zeros(1, dtype=torch.int64, device="cuda")
env.rollout(64, steps_done=done, max_steps=1, chunk=64)
s = env.get_state().cpu().numpy()[:, 0]
print("B: sum v0 integrated", s[FIELD["eta0"]], "sum v0 read", s[FIELD["eta1"]], "first", s[FIELD["eta2"]])
print("A: sum v0 published", s[FIELD["ang0"]], "wave-ticks", s[FIELD["ang1"]], "v0 now", s[FIELD["v0"]], "pw0", s[FIELD["pw0"]])
