"""RecurrentPPO with sb3-contrib's ``MlpLstmPolicy`` on the batched simulator:
the learner of ``/root/reference/src/train_robot_recurrent_ppo.py:85-107``
(``lstm_hidden_size=256, n_lstm_layers=1, enable_critic_lstm=True,
shared_lstm=False``; lr 3e-4, n_steps 2048, batch 64, 10 epochs, gamma 0.99,
GAE lambda 0.95, clip 0.2, ent 0, vf 0.5, max_grad_norm 0.5).

sb3-contrib (>= 2.0) is not installed here: its semantics are restated, and
parity with it is unpinned.  What is kept:

* policy: an LSTM for the actor and another for the critic on the raw
  observation, then SB3's ``net_arch`` pi=[64, 64] / vf=[64, 64] tanh MLPs, the
  action / value heads and a state-independent log-std (orthogonal init of the
  MLPs and heads as SB3; the LSTMs keep torch's default init, as sb3-contrib);
* the LSTM states are zeroed where an episode starts, before that step
  (sb3-contrib ``_process_sequence``), in collection and in training alike;
* the timeout bootstrap evaluates the terminal observation with the critic
  state after the step, episode start 0; the last value with the episode
  starts of the next step (``RecurrentPPO.collect_rollouts``);
* training re-runs the LSTMs over sequences from the states stored at their
  first step.  sb3-contrib cuts an env's rollout into sequences at episode
  starts and pads them; here every env's rollout is cut into fixed
  ``seq_len``-step sequences (the state stored every ``seq_len`` steps) and
  episode starts inside a sequence zero the state there.  Both compute the
  same forward pass per step; minibatches are ``batch_size // seq_len``
  sequences (no padding rows).

Collection is lock-step (``salp_step`` per env-step: the LSTM policy is not
evaluated inside the simulation kernel; ``salp_collect`` runs the MLP
policy), with the same divergence guard, episode statistics and HIP-event
phase timings as :class:`~grasp_lab_salp_amd.ppo.PPO`.
"""
import ctypes
import math

import torch
from torch import nn

from . import _lib
from .ppo import PPO, SplitKLinear, _ortho, allreduce_gradients, ppo_loss

__all__ = ["RecurrentActorCritic", "RecurrentPPO", "lstm_cell"]


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


class _LSTMCellFn(torch.autograd.Function):
    """The elementwise part of an LSTM step through the HIP kernels of
    salp_lstm_cell_forward / _backward (include/salp.h): one kernel each way
    instead of ~8 / ~12 torch kernels."""

    @staticmethod
    def forward(ctx, gates, c_prev, keep):
        m, h4 = gates.shape
        H = h4 // 4
        h = torch.empty((m, H), dtype=gates.dtype, device=gates.device)
        c = torch.empty_like(h)
        act = torch.empty_like(gates)
        st = ctypes.c_void_p(torch.cuda.current_stream(gates.device).cuda_stream)
        _lib.check(_lib.load().salp_lstm_cell_forward(m, H, _ptr(gates), _ptr(c_prev), _ptr(keep), _ptr(h), _ptr(c),
                                                      _ptr(act), st))
        ctx.save_for_backward(act, c_prev, keep, c)
        return h, c

    @staticmethod
    def backward(ctx, dh, dc):
        act, c_prev, keep, c = ctx.saved_tensors
        m, H = c.shape
        dh = torch.zeros_like(c) if dh is None else dh.contiguous()
        dc = None if dc is None else dc.contiguous()
        dg = torch.empty_like(act)
        dcp = torch.empty_like(c_prev)
        st = ctypes.c_void_p(torch.cuda.current_stream(c.device).cuda_stream)
        _lib.check(_lib.load().salp_lstm_cell_backward(m, H, _ptr(act), _ptr(c_prev), _ptr(keep), _ptr(c), _ptr(dh),
                                                       _ptr(dc), _ptr(dg), _ptr(dcp), st))
        return dg, dcp, None


class _SharedInputProjFn(torch.autograd.Function):
    """y[t, k] = x[t] @ w[k]: the input projection of every step t of the
    networks k, which share the input x [T, 1, n, K] (observations: no
    gradient); w [1, nets, K, N].  The weight gradient sum_t x_t^T dy[t, k] has
    K = 11 rows and T n = 32 768 reduction steps per minibatch: as one GEMM per
    network the library runs it on a handful of workgroups (~140 us); here the
    steps are the batch of one batched GEMM and the T products are summed
    (same math, another summation order)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        return torch.matmul(x, w)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return None, torch.matmul(x.transpose(-1, -2), gy).sum(0, keepdim=True)


class _LSTMPairSeqFn(torch.autograd.Function):
    """Both LSTMs (actor, critic) over a whole sequence, with the backward pass
    through time written out instead of recorded step by step (CUDA float32).

    Inputs: gx [T, 2, n, 4H] (input projection + bias), w_hh [2, H, 4H],
    h0 / c0 [2, n, H], keep [T, n] and keep2 [T, 2n] (1 - episode start).
    Outputs: h of every step [T, 2, n, H] and the last c [2, n, H].
    Per step forward: G = hk W_hh (one batched GEMM for both networks), then
    the cell kernel (salp_lstm_step_forward), which adds gx and writes the
    next step's hk = h keep; backward: the cell kernel (salp_lstm_step_backward,
    dh = d_out + d hk_next keep_next), then d hk = dG W_hh^T (one batched
    GEMM).  The recurrent weight gradient
    sum_t hk_t^T dG_t is one batched GEMM over all steps at the end, and dG
    of every step is written straight into the input projection's gradient,
    where step-by-step autograd ran 16 weight-gradient GEMMs and the
    accumulations between them."""

    @staticmethod
    def forward(ctx, gx, w_hh, h0, c0, keep, keep2):
        T, _, n, H4 = gx.shape
        H = H4 // 4
        out = gx.new_empty(T, 2, n, H)
        hk = gx.new_empty(T, 2, n, H)
        act = gx.new_empty(T, 2, n, H4)
        cs = gx.new_empty(T + 1, 2, n, H)
        cs[0].copy_(c0)
        g = gx.new_empty(2, n, H4)
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream(gx.device).cuda_stream)
        torch.mul(h0, keep[0].view(1, n, 1), out=hk[0])
        for t in range(T):
            torch.bmm(hk[t], w_hh, out=g)
            nxt = t + 1 < T
            _lib.check(lib.salp_lstm_step_forward(2 * n, H, _ptr(g), _ptr(gx[t]), _ptr(cs[t]), _ptr(keep2[t]),
                                                  _ptr(keep2[t + 1] if nxt else None), _ptr(out[t]),
                                                  _ptr(cs[t + 1]), _ptr(act[t]), _ptr(hk[t + 1] if nxt else None), st))
        ctx.save_for_backward(w_hh, hk, act, cs, keep, keep2)
        return out, cs[T]

    @staticmethod
    def backward(ctx, d_out, d_cT):
        w_hh, hk, act, cs, keep, keep2 = ctx.saved_tensors
        T, _, n, H = hk.shape
        lib = _lib.load()
        st = ctypes.c_void_p(torch.cuda.current_stream(hk.device).cuda_stream)
        dG = torch.empty_like(act)
        d_out = torch.zeros_like(hk) if d_out is None else d_out.contiguous()
        dc = None if d_cT is None else d_cT.contiguous()
        dhk = None                         # d hk[t + 1]
        w_t = w_hh.transpose(1, 2).contiguous()
        for t in range(T - 1, -1, -1):
            dcp = torch.empty_like(d_out[t])
            _lib.check(lib.salp_lstm_step_backward(2 * n, H, _ptr(act[t]), _ptr(cs[t]), _ptr(keep2[t]),
                                                   _ptr(cs[t + 1]), _ptr(d_out[t]), _ptr(dhk),
                                                   _ptr(keep2[t + 1] if dhk is not None else None), _ptr(dc),
                                                   _ptr(dG[t]), _ptr(dcp), st))
            dhk = torch.bmm(dG[t], w_t)
            dc = dcp
        d_w = torch.matmul(hk.transpose(-1, -2), dG).sum(0)
        return dG, d_w, dhk * keep[0].view(1, n, 1), dc, None, None


def lstm_cell(gates, c_prev, keep):
    """(h, c) of one LSTM step from the gate pre-activations [m, 4H] (i, f, g,
    o), the previous cell state [m, H] and keep [m] (the state is zeroed where
    keep is 0).  CUDA float32: the HIP kernels (fails if libsalp.so is
    missing); CPU: the same equations in torch ops (the tests' path)."""
    if gates.is_cuda:
        return _LSTMCellFn.apply(gates.contiguous(), c_prev.contiguous(), keep.contiguous())
    i, f, g, o = gates.chunk(4, 1)
    c = torch.sigmoid(f) * (c_prev * keep.unsqueeze(1)) + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(c), c


class RecurrentActorCritic(nn.Module):
    """sb3-contrib ``RecurrentActorCriticPolicy`` (MlpLstmPolicy) with separate
    actor and critic LSTMs.  A recurrent state is one [4, n, H] tensor:
    (h, c) of the actor LSTM, then (h, c) of the critic LSTM."""

    def __init__(self, obs_dim, act_dim, lstm_hidden_size=256, net_arch=(64, 64)):
        super().__init__()
        self.hidden = int(lstm_hidden_size)
        self.lstm_actor = nn.LSTM(obs_dim, self.hidden)
        self.lstm_critic = nn.LSTM(obs_dim, self.hidden)

        def mlp():
            layers, d = [], self.hidden
            for h in net_arch:
                layers += [_ortho(SplitKLinear(d, h), math.sqrt(2)), nn.Tanh()]
                d = h
            return nn.Sequential(*layers), d

        self.pi_net, d_pi = mlp()
        self.vf_net, d_vf = mlp()
        self.action_net = _ortho(SplitKLinear(d_pi, act_dim), 0.01)
        self.value_net = _ortho(SplitKLinear(d_vf, 1), 1.0)
        self.log_std = nn.Parameter(torch.zeros(act_dim))

    def initial_state(self, n, device=None):
        return torch.zeros(4, n, self.hidden, device=device)

    @staticmethod
    def _run(lstm, x, h, c, starts):
        """x [T, n, D] through `lstm` (torch's LSTM equations and parameter
        layout, gates i, f, g, o) from (h, c) [n, H]; the state is zeroed where
        starts[t] (an episode starts at step t), before step t.  The input
        projection of all T steps is one GEMM; each step is one GEMM plus the
        fused cell (lstm_cell: one HIP kernel each way), all capturable in a
        HIP graph (a fused RNN library call cannot reset states inside a
        sequence).
        Returns (outputs [T, n, H], h, c)."""
        T, n, D = x.shape
        # unbind, not gx[t]: the backward of T separate selects would zero-fill
        # and add T full-size [T, n, 4H] gradients; unbind's is one stack
        gx = torch.addmm(lstm.bias_ih_l0 + lstm.bias_hh_l0, x.reshape(T * n, D),
                         lstm.weight_ih_l0.t()).view(T, n, -1).unbind(0)
        w_hh = lstm.weight_hh_l0.t()
        keeps = (1.0 - starts).unbind(0)
        outs = []
        for t in range(T):
            keep = keeps[t]
            h, c = lstm_cell(torch.addmm(gx[t], h * keep.unsqueeze(1), w_hh), c, keep)
            outs.append(h)
        return torch.stack(outs), h, c

    def _run_pair(self, x, state, starts):
        """_run of the actor and the critic LSTM together (same input, same
        episode starts): every GEMM batched over the two networks (bmm), one
        cell launch per step for both.  state [4, n, H].
        Returns (actor outputs, critic outputs [T, n, H], new state)."""
        T, n, D = x.shape
        la, lc = self.lstm_actor, self.lstm_critic
        w_hh = torch.stack([la.weight_hh_l0, lc.weight_hh_l0]).transpose(1, 2)        # [2, H, 4H]
        # input projection of all T steps, the bias folded in as a ones column
        wb = torch.stack([torch.cat([la.weight_ih_l0.t(), (la.bias_ih_l0 + la.bias_hh_l0).unsqueeze(0)]),
                          torch.cat([lc.weight_ih_l0.t(), (lc.bias_ih_l0 + lc.bias_hh_l0).unsqueeze(0)])])
        xa = torch.cat([x, x.new_ones(T, n, 1)], 2).unsqueeze(1)                       # [T, 1, n, D + 1]
        if torch.is_grad_enabled():
            gx = _SharedInputProjFn.apply(xa, wb.unsqueeze(0))
        else:
            gx = torch.matmul(xa, wb.unsqueeze(0))                                     # [T, 2, n, 4H]
        keep1 = (1.0 - starts)                                                        # [T, n]
        keep2 = keep1.repeat(1, 2)                                                    # [T, 2n]: both nets
        if x.is_cuda:
            out, c = _LSTMPairSeqFn.apply(gx, w_hh, state[0::2].contiguous(), state[1::2].contiguous(), keep1,
                                          keep2)
            h = out[T - 1]
            oa, oc = out.unbind(1)
            return oa, oc, torch.stack([h[0], c[0], h[1], c[1]])
        gx = gx.unbind(0)
        keeps = keep1.unbind(0)
        keeps2 = keep2.unbind(0)
        h, c = state[0::2], state[1::2].reshape(2 * n, -1)                            # [2, n, H], [2n, H]
        outs = []
        for t in range(T):
            g = torch.baddbmm(gx[t], h * keeps[t].view(1, n, 1), w_hh)
            hf, c = lstm_cell(g.view(2 * n, -1), c, keeps2[t])
            h = hf.view(2, n, -1)
            outs.append(h)
        out = torch.stack(outs, 1)                                                    # [2, T, n, H]
        c = c.view(2, n, -1)
        return out[0], out[1], torch.stack([h[0], c[0], h[1], c[1]])

    def forward_seq(self, obs, state, starts, critic=True):
        """Latents of a sequence: obs [T, n, D], state [4, n, H], starts [T, n].
        Returns (actor latent [T, n, H], critic latent or None, new state)."""
        if critic:
            return self._run_pair(obs, state, starts)
        lp, hp, cp = self._run(self.lstm_actor, obs, state[0], state[1], starts)
        return lp, None, torch.stack([hp, cp, state[2], state[3]])

    def _dist(self, latent_pi):
        # the heads on [rows, H] (SplitKLinear's split-K weight gradient)
        mean = self.action_net(self.pi_net(latent_pi.reshape(-1, latent_pi.shape[-1])))
        mean = mean.view(*latent_pi.shape[:-1], -1)
        return torch.distributions.Normal(mean, self.log_std.exp().expand_as(mean), validate_args=False)

    def _value(self, latent_vf):
        v = self.value_net(self.vf_net(latent_vf.reshape(-1, latent_vf.shape[-1])))
        return v.view(latent_vf.shape[:-1])

    @torch.no_grad()
    def act(self, obs, state, episode_starts, generator=None):
        """One step for every env: obs [n, D] -> (action, value, log_prob,
        new state); the Gaussian noise from `generator` when given."""
        lp, lv, new = self.forward_seq(obs.unsqueeze(0), state, episode_starts.unsqueeze(0))
        d = self._dist(lp[0])
        if generator is None:
            a = d.sample()
        else:
            a = d.mean + d.stddev * torch.randn(d.mean.shape, generator=generator, device=d.mean.device,
                                                dtype=d.mean.dtype)
        return a, self._value(lv[0]), d.log_prob(a).sum(-1), new

    @torch.no_grad()
    def predict_values(self, obs, state, episode_starts):
        """V(obs) with the critic LSTM from `state` (not advanced)."""
        lv, _, _ = self._run(self.lstm_critic, obs.unsqueeze(0), state[2], state[3], episode_starts.unsqueeze(0))
        return self._value(lv[0])

    def evaluate(self, obs, actions, state, starts):
        """Training pass over sequences: obs [T, n, D], actions [T, n, A],
        state [4, n, H] at the sequences' first step, starts [T, n].
        Returns (value, log_prob, entropy), each [T, n]."""
        lp, lv, _ = self.forward_seq(obs, state, starts)
        d = self._dist(lp)
        return self._value(lv), d.log_prob(actions).sum(-1), d.entropy().sum(-1)


class RecurrentPPO(PPO):
    """sb3-contrib ``RecurrentPPO`` on a :class:`~grasp_lab_salp_amd.vec_env.SalpVecEnv`
    (see the module docstring for the semantics).  ``batch_size`` counts
    env-steps and must be a multiple of ``seq_len``."""

    def __init__(self, policy, env, learning_rate=3e-4, n_steps=2048, batch_size=64, n_epochs=10, gamma=0.99,
                 gae_lambda=0.95, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                 normalize_advantage=True, seed=0, device=None, verbose=0, reset_nonfinite=True,
                 policy_kwargs=None, seq_len=16, use_graphs=None):
        sim = getattr(env, "sim", env)
        kw = dict(policy_kwargs or {})
        for k, want in (("n_lstm_layers", 1), ("enable_critic_lstm", True), ("shared_lstm", False)):
            if kw.pop(k, want) != want:
                raise ValueError(f"policy_kwargs {k}={want} is the supported configuration")
        if policy == "MlpLstmPolicy":
            torch.manual_seed(int(seed))
            policy = RecurrentActorCritic(sim.obs_dim, 3, lstm_hidden_size=kw.pop("lstm_hidden_size", 256),
                                          net_arch=tuple(kw.pop("net_arch", (64, 64))))
        elif not isinstance(policy, RecurrentActorCritic):
            raise ValueError("policy must be 'MlpLstmPolicy' or a RecurrentActorCritic")
        if kw:
            raise ValueError(f"unsupported policy_kwargs: {sorted(kw)}")
        if n_steps % seq_len or batch_size % seq_len:
            raise ValueError("n_steps and batch_size must be multiples of seq_len")
        super().__init__(policy, env, learning_rate=learning_rate, n_steps=n_steps, batch_size=batch_size,
                         n_epochs=n_epochs, gamma=gamma, gae_lambda=gae_lambda, clip_range=clip_range,
                         ent_coef=ent_coef, vf_coef=vf_coef, max_grad_norm=max_grad_norm,
                         normalize_advantage=normalize_advantage, seed=seed, device=device, verbose=verbose,
                         reset_nonfinite=reset_nonfinite, use_graphs=use_graphs, fused_loss=False,
                         collect="lockstep", fused_update=False)
        self.seq_len = int(seq_len)
        self.n_seq = self.n_steps // self.seq_len
        self._lstm_state = self.policy.initial_state(self.n_envs, self.device)
        # recurrent state at the first step of every sequence [n_seq, 4, n, H]
        self.seq_states = torch.zeros(self.n_seq, 4, self.n_envs, self.policy.hidden, device=self.device)

    # -------------------------------------------- collection hooks (PPO)
    def _act(self, t, obs):
        if t % self.seq_len == 0:
            self.seq_states[t // self.seq_len].copy_(self._lstm_state)
        a, v, lp, self._lstm_state = self.policy.act(obs, self._lstm_state, self._episode_starts,
                                                     generator=self.sample_gen)
        return a, v, lp

    def _terminal_value(self, terminal_obs):
        # the critic state after the step, no reset (the episode ended at it)
        return self.policy.predict_values(terminal_obs, self._lstm_state, torch.zeros_like(self._episode_starts))

    def _last_values(self):
        # (a guard reset ends an episode too: the next step's episode start
        # zeroes that env's state, as for any other episode end)
        return self.policy.predict_values(self._obs, self._lstm_state, self._episode_starts)

    # ------------------------------------------------------------ update
    def _seq_minibatch(self, ids, acc):
        """One PPO gradient step on sequences `ids` (sequence k of env e is
        id k * n_envs + e)."""
        b, pol = self.buf, self.policy
        n, T = self.n_envs, self.seq_len
        k, e = ids // n, ids % n
        t = k.unsqueeze(0) * T + torch.arange(T, device=self.device).unsqueeze(1)   # [T, m]
        ee = e.unsqueeze(0).expand_as(t)
        obs, act = b.obs[t, ee], b.actions[t, ee]
        old_lp, adv, ret, starts = b.log_probs[t, ee], b.advantages[t, ee], b.returns[t, ee], b.episode_starts[t, ee]
        state = self.seq_states[k, :, e].transpose(0, 1)                             # [4, m, H]
        old_lp, adv, ret = (x.reshape(-1) for x in (old_lp, adv, ret))
        norm = self.normalize_advantage and adv.numel() > 1
        cr = self._clip()
        if obs.is_cuda:
            # the loss head as the fused HIP kernels of salp_ppo_loss (the MLP
            # PPO's, ppo.ppo_loss): one launch each way instead of ~25
            lat_pi, lat_vf, _ = pol.forward_seq(obs, state, starts)
            mean = pol.action_net(pol.pi_net(lat_pi.reshape(-1, lat_pi.shape[-1])))
            value = pol.value_net(pol.vf_net(lat_vf.reshape(-1, lat_vf.shape[-1]))).reshape(-1)
            loss, stats = ppo_loss(mean, pol.log_std, value, act.reshape(-1, act.shape[-1]), old_lp, adv, ret, cr,
                                   self.ent_coef, self.vf_coef, norm)
        else:
            v, lp, ent = pol.evaluate(obs, act, state, starts)
            v, lp, ent = (x.reshape(-1) for x in (v, lp, ent))
            if norm:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            ratio = torch.exp(lp - old_lp)
            pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - cr, 1 + cr)).mean()
            vf = torch.nn.functional.mse_loss(ret, v)
            ent_loss = -ent.mean()
            loss = pg + self.ent_coef * ent_loss + self.vf_coef * vf
            clip = ((ratio - 1).abs() > cr).float().mean()
            stats = torch.stack([pg.detach(), vf.detach(), -ent_loss.detach(), clip.detach()])
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        allreduce_gradients(list(pol.parameters()))
        nn.utils.clip_grad_norm_(pol.parameters(), self.max_grad_norm)
        self.opt.step()
        acc += stats

    def _minibatch(self, idx, acc):
        # PPO._graphed_minibatch captures / replays this with `idx` = sequence ids
        self._seq_minibatch(idx, acc)

    def train(self):
        """n_epochs passes over the rollout's sequences in random minibatches of
        batch_size // seq_len sequences.  On one GPU the minibatch step (the
        BPTT over seq_len steps: ~1 000 small kernels) runs as a HIP graph
        captured in the first update and kept (PPO._graphed_minibatch; the
        collection runs on its own stream, PPO.learn); a ragged last
        minibatch runs eagerly."""
        total = self.n_seq * self.n_envs
        per = self.batch_size // self.seq_len
        if total % per:
            self._graph, self._graph_warm = None, 0
        acc = torch.zeros(4, device=self.device)
        steps = 0
        for _ in range(self.n_epochs):
            perm = torch.randperm(total, generator=self.gen, device=self.device)
            for s in range(0, total, per):
                ids = perm[s:s + per]
                if self.use_graphs and ids.numel() == per:
                    self._graphed_minibatch(ids)
                else:
                    self._seq_minibatch(ids, acc)
                steps += 1
        if self.use_graphs and self._graph_warm > 0:
            acc = acc + self._g_acc
            self._g_acc.zero_()
        vals = (acc / max(steps, 1)).tolist()
        return dict(zip(("pg_loss", "vf_loss", "entropy", "clip_frac"), vals))
