"""Time the tick body alone (salp_bench_ticks) and the rollout at several chunks."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402


def main():
    n = int(os.environ.get("N", 65536))
    ticks = int(os.environ.get("TICKS", 4096))
    env = BatchedSalpEnv(n, seed=0)
    env.step_random(2)   # realistic mid-episode states
    L = _lib.load()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.salp_bench_ticks(env.handle, 64, s), env.handle)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.check(L.salp_bench_ticks(env.handle, ticks, s), env.handle)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(json.dumps({"tick_only_ms": ms, "ticks": ticks, "n": n, "env_ticks_per_s": n * ticks / ms * 1e3,
                      "us_per_tick_per_wave": ms * 1e3 / ticks}))


if __name__ == "__main__":
    main()
