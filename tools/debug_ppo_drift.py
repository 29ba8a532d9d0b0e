"""Debug: at chosen minibatches of PPO.learn() (HIP graph path), compare the
gradients one graph replay leaves (after clipping) with the same minibatch
computed eagerly from the same parameters: does the graph drift?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402

env = SalpVecEnv(32768, seed=0, infos=False)
m = PPO("MlpPolicy", env, n_steps=32, batch_size=32768, n_epochs=10, seed=0, use_graphs=True,
        fused_loss=os.environ.get("FUSED", "1") == "1")
CHECK = {300, 700, 1000, 1400, 1700, 2000, 2300, 2600, 2900}
state = {"mb": 0}
inner = m._graphed_minibatch
pol = m.policy


def tensors():
    out = []
    for p in pol.parameters():
        out.append(p.data)
        for v in m.opt.state.get(p, {}).values():
            if torch.is_tensor(v):
                out.append(v)
    return out


def wrapped(idx):
    mb = state["mb"]
    state["mb"] += 1
    if m._graph is None or mb not in CHECK:
        return inner(idx)
    pre = [t.clone() for t in tensors()]
    acc0 = m._g_acc.clone()
    inner(idx)
    torch.cuda.synchronize()
    g_graph = [p.grad.clone() for p in pol.parameters()]
    post = [t.clone() for t in tensors()]
    # eager from the same state
    for t, s in zip(tensors(), pre):
        t.copy_(s)
    saved = [p.grad for p in pol.parameters()]
    for p in pol.parameters():
        p.grad = None
    m._minibatch(m._g_idx, torch.zeros(4, device=m.device))
    torch.cuda.synchronize()
    g_eager = [p.grad.clone() for p in pol.parameters()]
    rel = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(g_graph, g_eager))
    fin = all(bool(torch.isfinite(g).all()) for g in g_graph)
    print("mb", mb, "graph grads finite", fin, "max rel diff graph vs eager", rel, flush=True)
    if rel > 0:
        for (n, _), a, b in zip(pol.named_parameters(), g_graph, g_eager):
            print("   ", n, "graph max", float(a.abs().max()), "eager max", float(b.abs().max()),
                  "rel", float((a - b).abs().max() / (b.abs().max() + 1e-30)), flush=True)
    # put the graph's state back (its grad buffers and the post-step values)
    for p, g in zip(pol.parameters(), saved):
        p.grad = g
    for t, s in zip(tensors(), post):
        t.copy_(s)
    m._g_acc.copy_(acc0 + (m._g_acc - m._g_acc))


m._graphed_minibatch = wrapped
m.learn(int(os.environ.get("ITERS", 4)) * 32 * 32768)
print("history", [round(r["vf_loss"], 1) for r in m.history], flush=True)
