"""Debug: PPO.learn() (4 iterations, config 5 at n_steps 32) through the HIP
graph; report whether the parameters stay finite.  Knobs (environment):
GRAPHS=1|0, ORDER=-1|0|1 (lock-step launch order), SYNC=1 (device sync
between collection and update), STREAM=1 (run on a non-default stream)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402

graphs = os.environ.get("GRAPHS", "1") == "1"
order = int(os.environ.get("ORDER", "-1"))
sync = os.environ.get("SYNC", "0") == "1"
env = SalpVecEnv(32768, seed=0, infos=False)
env.sim.set_lockstep_order(order)
m = PPO("MlpPolicy", env, n_steps=32, batch_size=32768, n_epochs=10, seed=0, use_graphs=graphs,
        fused_loss=os.environ.get("FUSED", "1") == "1")
if os.environ.get("PERM") == "host":     # permutations drawn on the host and uploaded
    orig = torch.randperm
    hg = torch.Generator().manual_seed(0)

    def rp(n, generator=None, device=None):
        return orig(n, generator=hg).to(device)
    torch.randperm = rp
if sync:
    inner = m.collect_rollouts

    def collect():
        ev = inner()
        torch.cuda.synchronize()
        return ev
    m.collect_rollouts = collect
if os.environ.get("STREAM", "0") == "1":
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.learn(4 * 32 * 32768)
    torch.cuda.synchronize()
else:
    m.learn(4 * 32 * 32768)
ok = all(bool(torch.isfinite(p).all()) for p in m.policy.parameters())
print({k: os.environ.get(k) for k in ("GRAPHS", "ORDER", "SYNC", "STREAM", "FUSED", "PERM")}, ok,
      [round(r["vf_loss"], 1) for r in m.history], flush=True)
