"""Debug: the fused PPO loss (salp_ppo_loss) captured in a HIP graph and
replayed on new inputs vs the same call made eagerly: bit-identical?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import ppo_loss  # noqa: E402

dev = torch.device("cuda")
B = 32768
g = torch.Generator(device=dev).manual_seed(0)


def fresh():
    mu = torch.randn(B, 3, device=dev, generator=g)
    return {"mu": mu, "value": torch.randn(B, device=dev, generator=g) * 100,
            "act": mu + 0.3 * torch.randn(B, 3, device=dev, generator=g),
            "old": torch.randn(B, device=dev, generator=g) - 3.0, "adv": torch.randn(B, device=dev, generator=g) * 50,
            "ret": torch.randn(B, device=dev, generator=g) * 300}


log_std = torch.zeros(3, device=dev, requires_grad=True)
static = {k: v.clone() for k, v in fresh().items()}
smu = static["mu"].clone().requires_grad_(True)
sv = static["value"].clone().requires_grad_(True)


def run(mu, v, d):
    loss, stats = ppo_loss(mu, log_std, v, d["act"], d["old"], d["adv"], d["ret"], 0.2, 0.0, 0.5, True)
    gm, gs, gv = torch.autograd.grad(loss, (mu, log_std, v))
    return torch.cat([loss.reshape(1), stats, gm.reshape(-1), gs, gv])


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(3):
        run(smu, sv, static)
torch.cuda.current_stream().wait_stream(side)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out = run(smu, sv, static)
bad = 0
for it in range(int(os.environ.get("ITERS", 200))):
    d = fresh()
    with torch.no_grad():
        smu.copy_(d["mu"])
        sv.copy_(d["value"])
    for k in ("act", "old", "adv", "ret"):
        static[k].copy_(d[k])
    graph.replay()
    ref = run(d["mu"].clone().requires_grad_(True), d["value"].clone().requires_grad_(True), d)
    if not torch.equal(out.view(torch.int32), ref.view(torch.int32)):
        bad += 1
        diff = (out != ref).nonzero().reshape(-1)
        if bad <= 5:
            print("replay", it, "differs at", diff[:8].tolist(), "n", diff.numel(), "graph", out[:5].tolist(),
                  "eager", ref[:5].tolist(), "finite", bool(torch.isfinite(out).all()), flush=True)
print("mismatching replays", bad, flush=True)
