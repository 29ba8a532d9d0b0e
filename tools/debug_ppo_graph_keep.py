"""Experiment: why does a HIP graph of the torch PPO minibatch step (custom
policies; fused_update=False) go stale when it is kept across collections
?  Runs PPO with the graph KEPT
from the first update in several variants and, in the third update, compares
one graph replay with the same minibatch run eagerly from the same parameters
and Adam state (bitwise), and reports whether the parameters stay finite.

Variants (VARIANTS env, comma-separated):
  side      warm-up on a fresh side stream per warm-up step (the product's)
  current   warm-up on the current stream
  grads     side-stream warm-up, but gradients allocated before the capture
            (zero_grad(set_to_none=False) at capture: the graph accumulates
            into tensors from the normal pool, not its private pool)
  pool      side-stream warm-up, capture into a pool kept by the PPO object
            (torch.cuda.graph_pool_handle()) so nothing else reuses it
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grasp_lab_salp_amd.ppo import PPO  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402


class KeptGraphPPO(PPO):
    variant = "side"

    def train(self):   # the graph is NOT reset per update
        N = self.n_steps * self.n_envs
        acc = torch.zeros(4, device=self.device)
        for _ in range(self.n_epochs):
            perm = torch.randperm(N, generator=self.gen, device=self.device)
            for s in range(0, N, self.batch_size):
                self._graphed_minibatch(perm[s:s + self.batch_size])
        return {"pg_loss": 0.0}

    def _graphed_minibatch(self, idx):
        if self._graph is None:
            if self._graph_warm == 0:
                self._g_idx = torch.empty_like(idx)
                self._g_acc = torch.zeros(4, device=self.device)
                self._pool = torch.cuda.graph_pool_handle() if self.variant == "pool" else None
            self._g_idx.copy_(idx)
            if self._graph_warm < 3:
                cur = torch.cuda.current_stream(self.device)
                side = cur if self.variant == "current" else torch.cuda.Stream(self.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    self.opt.zero_grad(set_to_none=True)
                    self._minibatch(self._g_idx, self._g_acc)
                cur.wait_stream(side)
                self._graph_warm += 1
                return
            self.opt.zero_grad(set_to_none=self.variant != "grads")
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph, pool=self._pool):
                self._minibatch(self._g_idx, self._g_acc)
        else:
            self._g_idx.copy_(idx)
        self._graph.replay()


def run(variant, n_envs, n_steps, updates, collect):
    KeptGraphPPO.variant = variant
    env = SalpVecEnv(n_envs, seed=0, infos=False)
    if os.environ.get("SPLITK", "1") == "0":   # plain nn.Linear backward (no split-K bmm)
        from grasp_lab_salp_amd.ppo import SplitKLinear
        SplitKLinear.ROWS_PER_SPLIT = 1 << 40
    if os.environ.get("ACT_PATCH") == "nogemm":   # lock-step collection without policy GEMMs
        from grasp_lab_salp_amd.ppo import ActorCritic

        def act(self, obs, generator=None):
            n = obs.shape[0]
            a = 0.5 + 0.1 * torch.randn((n, 3), generator=generator, device=obs.device)
            z = torch.zeros(n, device=obs.device)
            return a, z, z.clone()
        ActorCritic.act = act
    if os.environ.get("VALUE_PATCH") == "1":   # no value GEMMs outside autograd (collection, bootstrap)
        from grasp_lab_salp_amd.ppo import ActorCritic
        real_value = ActorCritic.value

        def value(self, obs):
            if torch.is_grad_enabled():
                return real_value(self, obs)
            return torch.zeros(obs.shape[0], device=obs.device)
        ActorCritic.value = value
    m = KeptGraphPPO("MlpPolicy", env, n_steps=n_steps, batch_size=32768,
                     n_epochs=int(os.environ.get("N_EPOCHS", 2)), seed=0, use_graphs=True, collect=collect,
                     fused_update=False, fused_loss=os.environ.get("FUSED_LOSS", "1") == "1",
                     reset_nonfinite=os.environ.get("NO_GUARD") != "1")
    out = {"variant": variant, "checks": [], "env": {k: os.environ.get(k) for k in
                                                   ("N_STEPS", "N_EPOCHS", "SPLITK", "FUSED_LOSS", "COLLECT", "ACT_PATCH", "NO_GUARD", "NO_COLLECT", "SYNC_ALLOC", "VALUE_PATCH", "COLLECT_STREAM",
                                                    "TORCH_BLAS_PREFER_HIPBLASLT")}}
    inner = m._graphed_minibatch

    def tensors():
        t = []
        for p in m.policy.parameters():
            t.append(p.data)
            t += [v for v in m.opt.state.get(p, {}).values() if torch.is_tensor(v)]
        return t

    def check(idx):
        if m._graph is None or len(out["checks"]) >= updates:
            return inner(idx)
        upd = m.num_timesteps // (n_steps * n_envs)
        if upd < len(out["checks"]) + 1:
            return inner(idx)
        pre = [t.clone() for t in tensors()]
        inner(idx)
        g_graph = [p.grad.clone() for p in m.policy.parameters()]
        post = [t.clone() for t in tensors()]
        keep = [p.grad for p in m.policy.parameters()]
        for t, s in zip(tensors(), pre):
            t.copy_(s)
        for p in m.policy.parameters():
            p.grad = None
        m._minibatch(m._g_idx, torch.zeros(4, device=m.device))
        same = all(torch.equal(a, p.grad) for a, p in zip(g_graph, m.policy.parameters()))
        fin = all(bool(torch.isfinite(g).all()) for g in g_graph)
        out["checks"].append({"update": upd + 1, "graph_equals_eager": same, "graph_grads_finite": fin})
        for p, g in zip(m.policy.parameters(), keep):
            p.grad = g
        for t, s in zip(tensors(), post):
            t.copy_(s)

    m._graphed_minibatch = check
    if os.environ.get("NO_COLLECT") == "1":   # one real collection, then updates on the same buffer
        real = m.collect_rollouts
        calls = []

        def collect_once():
            if not calls:
                calls.append(1)
                return real()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            for e in ev:
                e.record()
            return ev
        m.collect_rollouts = collect_once
    if os.environ.get("COLLECT_STREAM") == "1":   # eager collection on its own stream
        real_s = m.collect_rollouts
        cs = torch.cuda.Stream()

        def collect_on_stream():
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                ev = real_s()
            torch.cuda.current_stream().wait_stream(cs)
            return ev
        m.collect_rollouts = collect_on_stream
    if os.environ.get("SYNC_ALLOC") == "1":   # empty the caching allocator between updates
        real_c = m.collect_rollouts

        def collect_then_empty():
            ev = real_c()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            return ev
        m.collect_rollouts = collect_then_empty
    m.learn((updates + 1) * n_steps * n_envs)
    out["params_finite"] = all(bool(torch.isfinite(p).all()) for p in m.policy.parameters())
    return out


if __name__ == "__main__":
    n_envs = int(os.environ.get("N_ENVS", 32768))
    n_steps = int(os.environ.get("N_STEPS", 8))
    collect = os.environ.get("COLLECT", "lockstep")
    for v in os.environ.get("VARIANTS", "side,current,grads,pool").split(","):
        print(json.dumps(run(v, n_envs, n_steps, int(os.environ.get("UPDATES", 4)), collect)), flush=True)
