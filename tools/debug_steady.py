"""Debug: after a long tick-only run (salp_bench_ticks), which envs are not in
the steady body state (phase COAST/REST, length/width = init, float64)?"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402

n = 65536
env = BatchedSalpEnv(n, seed=0)
env.step_random(2)
L = _lib.load()
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
_lib.check(L.salp_bench_ticks(env.handle, int(os.environ.get("TICKS", 16384)), s), env.handle)
st = env.get_state().cpu()
p = default_params()
ph, Ln, Wd, g32 = (st[FIELD[k]] for k in ("phase", "length", "width", "geom32"))
print("phase counts", {int(v): int((ph == v).sum()) for v in ph.unique()})
bad = (ph < 2) | (Ln != p.init_length) | (Wd != p.init_width) | (g32 != 0)
print("not steady", int(bad.sum()), "of", n)
idx = bad.nonzero().flatten()[:10].tolist()
for i in idx:
    print(i, {k: float(st[FIELD[k], i]) for k in ("phase", "length", "width", "geom32", "cycle_time", "refill_time",
                                                "jet_time", "coast_time", "turn_time")})
print("L0", p.init_length, "W0", p.init_width)
t = st[FIELD["time"]]
print("steady-path ticks per env (time // 1e6): min", int((t // 1e6).min()), "mean", float((t // 1e6).mean()),
      "max", int((t // 1e6).max()))
