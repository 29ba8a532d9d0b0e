"""Debug: run PPO.learn() through the HIP graph; at the first minibatch after
which the parameters are non-finite, restore parameters and Adam state to
their values before it and replay the same minibatch twice more: does the
NaN come back (a deterministic function of the inputs) or not (a race)?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402

env = SalpVecEnv(32768, seed=0, infos=False)
m = PPO("MlpPolicy", env, n_steps=32, batch_size=32768, n_epochs=10, seed=0, use_graphs=True)
state = {"mb": 0, "done": False}
inner = m._graphed_minibatch


def tensors():
    out = []
    for p in m.policy.parameters():
        out.append(p.data)
        for v in m.opt.state.get(p, {}).values():
            if torch.is_tensor(v):
                out.append(v)
    return out


def fin():
    return all(bool(torch.isfinite(p).all()) for p in m.policy.parameters())


def wrapped(idx):
    if state["done"] or m._graph is None:
        state["mb"] += 1
        return inner(idx)
    pre = [t.clone() for t in tensors()]
    inner(idx)
    torch.cuda.synchronize()
    mb = state["mb"]
    state["mb"] += 1
    if fin():
        return
    state["done"] = True
    print("first non-finite after minibatch", mb, flush=True)
    for k in range(3):
        for t, s in zip(tensors(), pre):
            t.copy_(s)
        m._graph.replay()
        torch.cuda.synchronize()
        print(" replay again", k, "finite", fin(), "grads finite",
              all(bool(torch.isfinite(p.grad).all()) for p in m.policy.parameters()), flush=True)
    for t, s in zip(tensors(), pre):
        t.copy_(s)
    b, pol, N = m.buf, m.policy, m.n_steps * m.n_envs
    ix = m._g_idx
    obs, act = b.obs.reshape(N, -1)[ix], b.actions.reshape(N, -1)[ix]
    old, adv, ret = b.log_probs.reshape(N)[ix], b.advantages.reshape(N)[ix], b.returns.reshape(N)[ix]
    mu = pol.action_net(pol.pi_net(obs))
    v = pol.value(obs)
    var = torch.exp(2 * pol.log_std)
    lp = (-(act - mu) ** 2 / (2 * var) - pol.log_std - 0.9189385332046727).sum(-1)
    print(" log_std", pol.log_std.tolist(), "max lp-old", float((lp - old).max()), "min", float((lp - old).min()),
          "max|mu|", float(mu.abs().max()), "max|v|", float(v.abs().max()), "max|ret|", float(ret.abs().max()),
          "max|adv|", float(adv.abs().max()), "adv std", float(adv.std()), "max|obs|", float(obs.abs().max()),
          flush=True)
    from grasp_lab_salp_amd.ppo import torch_ppo_loss
    loss, _ = torch_ppo_loss(mu, pol.log_std, v, act, old, adv, ret, 0.2, 0.0, 0.5, True)[:2]
    gr = torch.autograd.grad(loss, list(pol.parameters()), allow_unused=True)
    print(" torch loss", float(loss), "grads finite", [bool(torch.isfinite(x).all()) if x is not None else None
                                                       for x in gr],
          "max|g|", [float(x.abs().max()) if x is not None else None for x in gr], flush=True)
    from grasp_lab_salp_amd.ppo import ppo_loss
    lf, sf = ppo_loss(mu, pol.log_std, v, act, old, adv, ret, 0.2, 0.0, 0.5, True)
    gf = torch.autograd.grad(lf, [mu, pol.log_std, v])
    lt, st = torch_ppo_loss(mu, pol.log_std, v, act, old, adv, ret, 0.2, 0.0, 0.5, True)[:2]
    gt = torch.autograd.grad(lt, [mu, pol.log_std, v])
    print(" fused", float(lf), sf.tolist(), "torch", float(lt), st.tolist(), flush=True)
    for name, a, c in zip(("dmu", "dlog_std", "dv"), gf, gt):
        print("  ", name, "fused finite", bool(torch.isfinite(a).all()), "max|diff|",
              float((a - c).abs().max()), "max|torch|", float(c.abs().max()), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save({k: t.detach().cpu() for k, t in dict(mu=mu, log_std=pol.log_std, v=v, act=act, old=old, adv=adv,
                                                      ret=ret).items()}, "gpurun_out/ppo_nan_inputs.pt")
    for t, s in zip(tensors(), pre):
        t.copy_(s)
    for p in pol.parameters():
        p.grad = None
    mean = pol.action_net(pol.pi_net(obs))
    lf, sf = ppo_loss(mean, pol.log_std, pol.value(obs), act, old, adv, ret, m._clip(), m.ent_coef, m.vf_coef, True)
    lf.backward()
    gfin = lambda: [bool(torch.isfinite(p.grad).all()) for p in pol.parameters()]  # noqa: E731
    print(" step by step: loss", float(lf), "grads finite", gfin(), flush=True)
    tn = torch.nn.utils.clip_grad_norm_(pol.parameters(), m.max_grad_norm)
    print(" after clip: total norm", float(tn), "grads finite", gfin(), flush=True)
    st = {k: (v.tolist() if v.numel() < 4 else float(v.abs().max())) for k, v in m.opt.state[pol.log_std].items()}
    print(" adam state of log_std", st, m.opt.defaults, flush=True)
    m.opt.step()
    print(" after adam: params finite", fin(), flush=True)


m._graphed_minibatch = wrapped
m.learn(4 * 32 * 32768)
print("history", [round(r["vf_loss"], 1) for r in m.history], flush=True)
