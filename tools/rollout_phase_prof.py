"""Where a k_rollout launch goes, per wave: env-step boundary + re-seat, full
ticks, steady ticks, settled ticks, the re-seat barrier and the re-seat itself (s_memtime
cycles and loop iterations,
summed over the launch's waves).  Needs the instrumented variant

    EXTRA_FLAGS=-DSALP_ROLLOUT_PROF=1 python tools/build_variant.py rprof

run with SALP_LIB=exp_build/libsalp_rprof.so.  Bench configuration (65 536
envs, tick budget 8 192, chunk 64, 16-slot rollout buffer).  Prints, per
launch, each part's share of the wave time and its cycles per wave iteration
(per tick of that kind; the boundary per chunk)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402

PARTS = ["boundary", "full", "steady", "settled", "barrier", "reseat"]


def main():
    n, budget, cap = 65536, 8192, 16
    env = BatchedSalpEnv(n, seed=0)
    od = env.obs_dim
    bufs = {"obs": torch.empty((cap, n, od), device="cuda"), "obs_before": torch.empty((cap, n, od), device="cuda"),
            "actions": torch.empty((cap, n, 3), device="cuda"), "rewards": torch.empty((cap, n), device="cuda"),
            "dones": torch.empty((cap, n), dtype=torch.uint8, device="cuda")}
    sd = torch.zeros(n, dtype=torch.int64, device="cuda")
    L = _lib.load()
    L.salp_debug_rollout_prof.argtypes = [ctypes.c_void_p]
    a = np.zeros((2, len(PARTS)), dtype=np.uint64)
    L.salp_debug_rollout_prof(a.ctypes.data)   # clear
    rows = []
    for launch in range(int(os.environ.get("LAUNCHES", 6))):
        s0 = int(sd.sum())
        env.rollout(budget, buffers=bufs, steps_done=sd)
        torch.cuda.synchronize()
        assert L.salp_debug_rollout_prof(a.ctypes.data) == 0
        cyc, its = a[0].astype(np.float64), a[1].astype(np.float64)
        row = {"launch": launch, "env_steps": int(sd.sum()) - s0,
               "share": dict(zip(PARTS, [round(float(x), 4) for x in cyc / cyc.sum()])),
               "wave_iterations": dict(zip(PARTS[1:4], [int(x) for x in its[1:4]])),
               "cycles_per_iteration": dict(zip(PARTS[1:4], [round(float(c / max(i, 1)), 1)
                                                              for c, i in zip(cyc[1:4], its[1:4])])),
               "wave_cycles_total": float(cyc.sum())}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"parts": PARTS, "last": rows[-1]}))


if __name__ == "__main__":
    main()
