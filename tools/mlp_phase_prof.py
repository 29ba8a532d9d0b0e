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
    w = a[:, :NPH - 2].astype(np.float64)
    tot = w.sum(1)
    t0, t1 = a[:, NPH - 2].astype(np.int64), a[:, NPH - 1].astype(np.int64)
    base = t0.min()
    print(json.dumps({"frac_by_barrier": [round(float(x), 4) for x in w.sum(0) / tot.sum()],
                      "cycles_by_barrier_mean": [round(float(x)) for x in w.mean(0)],
                      "wave_cycles_mean": float(tot.mean()),
                      # wall_clock64: 100 MHz
                      "wave_start_us": {"p50": float(np.percentile(t0 - base, 50)) / 100,
                                        "max": float((t0 - base).max()) / 100},
                      "wave_end_us": {"p50": float(np.percentile(t1 - base, 50)) / 100,
                                      "max": float((t1 - base).max()) / 100},
                      "wave_span_us_mean": float((t1 - t0).mean()) / 100}))


if __name__ == "__main__":
    main()
