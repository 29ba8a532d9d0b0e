"""Dump one salp_collect run per rollout kernel (k_rollout, k_rollout_pair) to
an .npz, to compare two builds of libsalp.so bit for bit (SALP_LIB selects the
build): python tools/collect_dump.py OUT.npz [N_ENVS] [N_STEPS]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_pair import _collect  # noqa: E402

out = {}
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
t = int(sys.argv[3]) if len(sys.argv) > 3 else 12
for kernel in (0, 1):
    res, _, _ = _collect(kernel, n, t)
    for k, v in res.items():
        out[f"k{kernel}_{k}"] = v
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1], len(out), "arrays")
