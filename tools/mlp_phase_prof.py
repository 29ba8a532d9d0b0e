"""Where k_mlp_fwd_bwd spends its time, per wave and phase (phase i ends at
the kernel's i-th __syncthreads(), the last one at the kernel's end).  Needs
the instrumented build of tools/build_mlp_prof.py (SALP_LIB=
exp_build/libsalp_mlpprof.so)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402

NPH = 24   # tools/build_mlp_prof.py: phase i ends at the kernel's i-th __syncthreads()


def main():
    env = SalpVecEnv(32768, seed=0, infos=False)
    m = PPO("MlpPolicy", env, n_steps=8, batch_size=32768, n_epochs=1, seed=0, use_graphs=False)
    m.learn(8 * 32768)
    idx = torch.randperm(8 * 32768, device="cuda")[:32768]
    acc = torch.zeros(4, device="cuda")
    for _ in range(3):
        m._fused_minibatch(idx, acc)
    torch.cuda.synchronize()
    L = _lib.load()
    L.salp_debug_mlp_prof.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    n = 256 * 8
    a = np.zeros((n, NPH), dtype=np.uint64)
    assert L.salp_debug_mlp_prof(a.ctypes.data, n) == 0
    w = a.astype(np.float64)
    tot = w.sum(1)
    print(json.dumps({"frac_by_barrier": [round(float(x), 4) for x in w.sum(0) / tot.sum()],
                      "wave_cycles_mean": float(tot.mean())}))


if __name__ == "__main__":
    main()
