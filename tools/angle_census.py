import sys, json, numpy as np, torch
sys.path.insert(0, '/root/repo')
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
from grasp_lab_salp_amd._abi import FIELD
env = BatchedSalpEnv(65536, seed=0)
env.reset()
out = []
for L in range(1, 81):
    env.rollout(8192)
    if L in (3, 10, 20, 30, 50, 80):
        st = env.get_state().cpu().numpy()
        e0, e1, e2 = st[FIELD["eta0"]], st[FIELD["eta1"]], st[FIELD["eta2"]]
        nan = np.isnan(e0) | np.isnan(e1)
        inf = np.isinf(e0) | np.isinf(e1)
        fin = np.isfinite(e0) & np.isfinite(e1)
        big = fin & ((np.abs(e0) > 1/16) | (np.abs(e1) > 1/16))
        vbig = fin & ((np.abs(e0) > np.pi/4) | (np.abs(e1) > np.pi/4))
        out.append({"launch": L, "nan": int(nan.sum()), "inf": int(inf.sum()), "finite_gt_1_16": int(big.sum()),
                    "finite_gt_pi_4": int(vbig.sum()), "waves_with_gt_1_16": int(((big | inf).reshape(-1, 64)).any(1).sum()),
                    "max_abs_finite_roll": float(np.nanmax(np.abs(np.where(fin, e0, 0)))), "max_abs_finite_pitch": float(np.nanmax(np.abs(np.where(fin, e1, 0))))})
print(json.dumps(out))
