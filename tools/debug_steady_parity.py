"""Debug: drop-in episode actions (tests/golden episodes.npz, JOB) stepped on
the HIP env (1 env) and the C oracle side by side; report the first env-step
whose state differs bit for bit, and the fields that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_util import load_episodes  # noqa: E402
from grasp_lab_salp_amd._abi import FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from oracle import oracle as orc  # noqa: E402

d = load_episodes()
job = int(os.environ.get("JOB", 3))
rows = np.where(d["job_index"] == job)[0]
p = default_params()
env = BatchedSalpEnv(1, params=p, seed=job)
o = orc.Oracle(p, 1, seed=job)
env.reset()
o.reset()
o.state[:] = env.get_state().cpu().numpy()
KEYS = ('length', 'width', 'geom32', 'pvol32', 'cycle_time', 'refill_time', 'turn_time', 'jet_time', 'coast_time',
        'volume', 'prev_volume', 'com', 'com_rate', 'com_acc', 'phase', 'contraction')
for k, r in enumerate(rows):
    before = {f: repr(float(o.state[FIELDS.index(f), 0])) for f in KEYS if f in FIELDS}
    a = np.asarray(d["action"][r], np.float32)[None]
    env.step(torch.tensor(a, device="cuda"), auto_reset=False)
    o.step(a, auto_reset=False)
    g = env.get_state().cpu().numpy()
    diff = [FIELDS[f] for f in range(len(FIELDS)) if not np.array_equal(g[f], o.state[f], equal_nan=True)]
    if diff:
        print("state before:", before, flush=True)
        print("first differing env-step", k, "row", r, "action", a.tolist(), "fields", diff[:12], flush=True)
        for name in diff[:6]:
            i = FIELDS.index(name)
            print("  ", name, repr(float(g[i, 0])), repr(float(o.state[i, 0])), flush=True)
        break
else:
    print("no difference over", len(rows), "env-steps", flush=True)
