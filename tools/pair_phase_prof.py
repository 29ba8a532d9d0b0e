"""Where k_rollout_pair's waves spend their cycles (s_memtime per phase, summed
over waves): boundary + re-seat, tick compute, packet publish, waiting for the
partner, packet read, world-frame update.  Needs the variant
    EXTRA_FLAGS=-DSALP_PAIR_PROF=1 python tools/build_variant.py pprof
run with SALP_LIB=exp_build/libsalp_pprof.so.  N envs (default 32768),
random-action chained rollout with a step cap of K env-steps."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd import _lib  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402

PHASES = ["boundary", "tick", "publish", "wait", "read", "world", "barrier"]


def main():
    L = _lib.load()
    L.salp_debug_pair_prof.argtypes = [ctypes.c_void_p]
    k = int(os.environ.get("K", 16))
    collect = os.environ.get("COLLECT") == "1"
    for n in [int(x) for x in os.environ.get("N", "32768").split()]:
        env = BatchedSalpEnv(n, seed=0)
        env.set_rollout_kernel(1)
        sd = torch.zeros(n, dtype=torch.int64, device="cuda")
        if collect:
            from grasp_lab_salp_amd.ppo import ActorCritic, pack_policy
            w = pack_policy(ActorCritic(env.obs_dim, 3).cuda())
            z = lambda *s: torch.zeros(s, dtype=torch.float32, device="cuda")  # noqa: E731
            bufs = {"obs": z(k, n, env.obs_dim), "actions": z(k, n, 3), "rewards": z(k, n),
                    "episode_starts": z(k, n), "values": z(k, n), "log_probs": z(k, n)}
            extra = [torch.ones(n, device="cuda"), env.reset(), torch.zeros(4, dtype=torch.float64, device="cuda"),
                     torch.zeros(1, dtype=torch.int64, device="cuda")]
            run = lambda: env.collect(w, k, bufs, *extra, diverged_obs_abs=1e3, diverged_reward_abs=1e4)  # noqa: E731
        else:
            run = lambda: env.rollout(10 ** 8, steps_done=sd.zero_(), max_steps=k)  # noqa: E731
        run()   # warm-up
        torch.cuda.synchronize()
        a = np.zeros((2, len(PHASES)), np.uint64)
        L.salp_debug_pair_prof(a.ctypes.data)
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        assert L.salp_debug_pair_prof(a.ctypes.data) == 0
        out = {"n_envs": n, "k": k, "collect": collect, "env_steps_per_sec": n * k / el}
        for r, role in enumerate(("A", "B")):
            tot = float(a[r].sum())
            out[role] = {p: round(float(a[r, j]) / tot, 4) for j, p in enumerate(PHASES)}
            out[role]["cycles_per_wave"] = tot / (n // 64)
        print(json.dumps(out), flush=True)
        env.close()


if __name__ == "__main__":
    main()
