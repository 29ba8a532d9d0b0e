"""Split-invariance probe: the headline split test's two
runs, each twice, and where they differ.

    SALP_LIB=exp_build/libsalp_X.so ORACLE_LIB=exp_build/X/oracle/libsalp_oracle.so \
        python tools/split_probe.py > gpurun_out/split_probe.json

Runs test_gpu_headline.py's workload (65 536 envs, seed 17, 6 env-steps per
env): A = one launch, B = 97-tick launches; A2 / B2 repeat them (a launch
that differs from its own repeat is nondeterministic: a race, not a
scheduling dependence).  For every pair it reports the differing envs, the
fields and whether the differences are NaN payloads (both NaN), signed zeros
or values, with examples; then replays up to 32 differing env ids on the C
oracle built from the same headers (ORACLE_LIB) and says which run equals it.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grasp_lab_salp_amd._abi import FIELD, FIELDS, default_params  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from oracle import oracle as orc  # noqa: E402

if os.environ.get("ORACLE_LIB"):
    orc.LIB_PATH = os.environ["ORACLE_LIB"]
    orc.build = lambda force=False: orc.LIB_PATH

N, SEED, STEPS, CHUNK = int(os.environ.get("N", 65536)), 17, 6, 97


def run(cut, kernel=-1):
    e = BatchedSalpEnv(N, params=default_params(), seed=SEED)
    e.set_rollout_kernel(kernel)
    done = torch.zeros(N, dtype=torch.int64, device="cuda")
    launches = 0
    if not cut:
        e.rollout(20000, steps_done=done, chunk=CHUNK, max_steps=STEPS)
        launches = 1
    else:
        while int(done.min()) < STEPS and launches < 400:
            e.rollout(CHUNK, steps_done=done, chunk=CHUNK, max_steps=STEPS)
            launches += 1
    torch.cuda.synchronize()
    s = e.get_state().cpu().numpy()
    e.close()
    return s, done.cpu().numpy(), launches


def diff(a, b):
    d = a.view(np.int64) != b.view(np.int64)
    nan = d & np.isnan(a) & np.isnan(b)
    zero = d & (a == 0) & (b == 0)
    val = d & ~nan & ~zero
    envs = np.nonzero(d.any(0))[0]
    out = {"envs": int(len(envs)), "value_envs": int(val.any(0).sum()), "nan_payload_envs": int(nan.any(0).sum()),
           "signed_zero_envs": int(zero.any(0).sum()),
           "fields": {FIELDS[f]: [int(val[f].sum()), int(nan[f].sum()), int(zero[f].sum())]
                      for f in np.nonzero(d.any(1))[0]},
           "examples": []}
    for j in envs[:6]:
        for f in np.nonzero(d[:, j])[0][:4]:
            out["examples"].append({"env": int(j), "field": FIELDS[f], "a": float(a[f, j]).hex(),
                                    "b": float(b[f, j]).hex(), "a_bits": hex(int(a[f, j:j + 1].view(np.uint64)[0])),
                                    "b_bits": hex(int(b[f, j:j + 1].view(np.uint64)[0]))})
    return out, envs


def main():
    res = {"lib": os.environ.get("SALP_LIB", "product"), "oracle": orc.LIB_PATH}
    A, dA, _ = run(False)
    A2, _, _ = run(False)
    B, dB, nl = run(True)
    B2, _, _ = run(True)
    res["cut_launches"] = nl
    res["steps_done_equal"] = bool(np.array_equal(dA, dB))
    for name, (x, y) in {"A_vs_A2": (A, A2), "B_vs_B2": (B, B2), "A_vs_B": (A, B)}.items():
        res[name], envs = diff(x, y)
        if name == "A_vs_B":
            ids = envs[:32].astype(np.int64)
    if len(ids):
        pend = A[FIELD["pending"], ids] != 0.0
        ct = np.where(pend, A[FIELD["cycle_time"], ids], -1.0)
        st, _ = orc.replay(ids, dA[ids], ct, seed=SEED, params=default_params(),
                           threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
        bits = lambda x: x.view(np.int64)
        eqA = (bits(A[:, ids]) == bits(st)) | (np.isnan(A[:, ids]) & np.isnan(st))
        eqB = (bits(B[:, ids]) == bits(st)) | (np.isnan(B[:, ids]) & np.isnan(st))
        res["oracle_replay"] = {"ids": ids.tolist(), "A_equals_oracle": int(eqA.all(0).sum()),
                                "B_equals_oracle": int(eqB.all(0).sum()),
                                "A_nan_envs": int(np.isnan(A[:, ids]).any(0).sum()),
                                "A_pending": int(pend.sum())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
