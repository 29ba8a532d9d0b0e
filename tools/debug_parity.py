"""Diagnose a device-vs-oracle mismatch: which envs / fields / outputs differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELDS, NUM_FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    n = 4096
    rng = np.random.default_rng(11)
    p = default_params()
    env = BatchedSalpEnv(n, params=p, seed=5)
    o = orc.Oracle(p, n, seed=5)
    o.reset()
    tg = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n)], 1).astype(np.float32)
    ob = rng.uniform(-2, 2, (n, 2, 2)).astype(np.float32)
    nob = rng.integers(0, 3, n).astype(np.int32)
    env.reset_to(torch.tensor(tg), torch.tensor(ob), torch.tensor(nob))
    o.reset_to(tg, ob, nob)
    a = np.stack([rng.uniform(0, 1, n), rng.uniform(0, 1, n), rng.uniform(-1, 1, n)], 1).astype(np.float32)
    for auto in (False, True):
        st_g, st_o = env.get_state().cpu().numpy(), o.state.copy()
        assert np.array_equal(st_g, st_o)
        r = env.step(torch.tensor(a), auto_reset=auto)
        ro = o.step(a, auto_reset=auto)
        g = env.get_state().cpu().numpy()
        done = (ro["terminated"] | ro["truncated"]).astype(bool)
        print(f"auto_reset={auto}: done envs {done.sum()}")
        bad_obs = np.where(np.any(r.obs.cpu().numpy() != ro["obs"], 1))[0]
        bad_tobs = np.where(np.any(r.terminal_obs.cpu().numpy() != ro["terminal_obs"], 1))[0]
        bad_rew = np.where(r.reward.cpu().numpy() != ro["reward"])[0]
        print(" obs mismatches", len(bad_obs), "of which done", done[bad_obs].sum(), bad_obs[:10])
        print(" terminal obs mismatches", len(bad_tobs), " reward mismatches", len(bad_rew))
        for f in range(NUM_FIELDS):
            d = np.where(g[f] != o.state[f])[0]
            if len(d):
                print(f"  field {FIELDS[f]:12s} {len(d):5d} envs, done {done[d].sum()}, e.g. env {d[0]}: "
                      f"gpu {g[f][d[0]]!r} oracle {o.state[f][d[0]]!r}")
        if len(bad_obs):
            i = bad_obs[0]
            print(" env", i, "gpu obs", r.obs.cpu().numpy()[i], "\n     oracle obs", ro["obs"][i])
        # restore identical states for the next round
        env.set_state(torch.tensor(o.state))


if __name__ == "__main__":
    main()
