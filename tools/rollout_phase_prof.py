"""Where a k_rollout launch spends its time, per wave: boundary + re-seat
(spill, env-step epilogue/prologue, barrier, unspill), full ticks, steady
ticks, settled ticks.  Needs the instrumented variant built by
tools/build_variant.py (SALP_LIB=exp_build/libsalp_tprof.so; it records
s_memtime deltas per lane and exports salp_debug_prof).  Bench config."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def main():
    n, budget, cap = 65536, 8192, 16
    env = BatchedSalpEnv(n, seed=0)
    od = env.obs_dim
    bufs = {"obs": torch.empty((cap, n, od), device="cuda"), "obs_before": torch.empty((cap, n, od), device="cuda"),
            "actions": torch.empty((cap, n, 3), device="cuda"), "rewards": torch.empty((cap, n), device="cuda"),
            "dones": torch.empty((cap, n), dtype=torch.uint8, device="cuda")}
    sd = torch.zeros(n, dtype=torch.int64, device="cuda")
    L = _lib.load()
    L.salp_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    out = {}
    for launch in range(int(os.environ.get("LAUNCHES", 6))):
        env.rollout(budget, buffers=bufs, steps_done=sd)
        torch.cuda.synchronize()
        a = np.zeros((n, 4), dtype=np.uint64)
        assert L.salp_debug_prof(a.ctypes.data, n) == 0
        w = a[::64].astype(np.float64)          # lane 0 of every wave
        tot = w.sum(1)
        out[launch] = {"frac": [round(float(x), 4) for x in (w.sum(0) / tot.sum())],
                       "wave_total_mean": float(tot.mean()), "wave_total_max": float(tot.max())}
        print(json.dumps({"launch": launch, **out[launch]}), flush=True)
    print(json.dumps({"phases": ["boundary+reseat", "full", "steady", "settled"], "last": out[max(out)]}))


if __name__ == "__main__":
    main()
