"""On-device PPO over the batched simulator (BASELINE.json config 5).

The reference trains with Stable-Baselines3 learners (SAC, src/train_robot.py:
62-69; RecurrentPPO, src/train_robot_recurrent_ppo.py:85-107) on 4-8 envs
stepped through Python processes.  Here the envs, the rollout buffer, the GAE
scan (HIP kernel ``salp_gae``) and the policy all stay in HBM:

* collection: ``n_steps`` lock-step env-steps of every env (``salp_step`` with
  SB3 auto-reset), actions sampled from a diagonal Gaussian MLP policy and
  clipped to the action box before the step (SB3 ``collect_rollouts``);
  truncated-not-terminated episodes get ``gamma * V(terminal_obs)`` added to
  their reward (SB3's timeout bootstrap);
  or, with ``collect="chained"`` (the default from n_steps 256 on), ``salp_collect``: the policy is evaluated
  inside the chained simulation kernel at each env's own env-step boundaries
  (exploration noise from Philox keyed by env id and step), so no env waits
  for the slowest cycle of the batch between two steps;
* advantages / returns: ``salp_gae`` (bit-identical to SB3's NumPy code,
  oracle/gae.py);
* update: SB3 PPO's clipped surrogate + value MSE - entropy, advantage
  normalisation per minibatch, grad-norm clipping, Adam;
* multi-GPU: one process per GPU, each with its own env shard; gradients are
  averaged with one flat all-reduce per minibatch (torch.distributed, ``nccl``
  = RCCL over xGMI; the MLP's gradients are ~20 KB, so one bucket);
* update: for the built-in policy the whole minibatch step (forward, loss,
  backward, clipping, Adam) is four HIP kernels (``salp_ppo_mlp_grads`` /
  ``salp_ppo_mlp_apply``, csrc/salp_ppo_mlp.hip) instead of ~60 torch kernels;
  it is captured into a HIP graph once and replayed per minibatch (with
  several ranks as two graphs around the eager gradient all-reduce); other
  policies take the torch path (autograd, torch Adam, a graph per update, one
  GPU only).

The policy is SB3's ``MlpPolicy`` for PPO (separate 64-64 tanh actor and critic,
orthogonal init, state-independent log-std).  The reference's RecurrentPPO
uses an LSTM-256 policy; at 32 768 envs its per-step LSTM state buffer would
not fit, so config 5 runs the MLP policy.  SB3 itself is not
installed: its semantics are restated, not pinned by a reference test.
"""
import ctypes
import math
import os
import time

import torch
import torch.distributed as dist
from torch import nn

from . import _lib
from ._abi import INFO, OBS_DIM_MAX, POLICY_OFFSETS, POLICY_SIZE

__all__ = ["compute_gae", "ppo_loss", "torch_ppo_loss", "ActorCritic", "SplitKLinear", "RolloutBuffer", "PPO",
           "allreduce_gradients", "sampling_generator", "timeout_bootstrap", "diverged_mask"]


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def compute_gae(rewards, values, episode_starts, last_values, dones, gamma=0.99, gae_lambda=0.95,
                advantages=None, returns=None):
    """SB3 ``compute_returns_and_advantage`` on the GPU (``salp_gae``).
    All inputs float32 CUDA tensors, [n_steps, n_envs] / [n_envs]."""
    T, n = rewards.shape
    for name, t, shape in (("rewards", rewards, (T, n)), ("values", values, (T, n)),
                           ("episode_starts", episode_starts, (T, n)), ("last_values", last_values, (n,)),
                           ("dones", dones, (n,))):
        if not t.is_cuda or t.dtype != torch.float32 or tuple(t.shape) != shape or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous float32 CUDA tensor of shape {shape}")
    adv = torch.empty_like(rewards) if advantages is None else advantages
    ret = torch.empty_like(rewards) if returns is None else returns
    stream = ctypes.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    _lib.check(_lib.load().salp_gae(T, n, _ptr(rewards), _ptr(values), _ptr(episode_starts), _ptr(last_values),
                                    _ptr(dones), float(gamma), float(gae_lambda), _ptr(adv), _ptr(ret), stream))
    return adv, ret


class _SplitKLinearFn(torch.autograd.Function):
    """y = x @ W.T + b whose weight gradient is a split-K reduction.

    A minibatch of 32 768 rows makes dW = dY.T @ X a 64x64 (or 64x10) output
    with K = 32 768: the library picks one or four output tiles and no split-K,
    so 4 workgroups run a 32 768-long reduction (~120-150 us per GEMM, half of
    the whole update, profiles/r1m_ppo_kernel_stats.csv).  Here K is cut into
    `splits` slices reduced by one batched GEMM (64 and more workgroups), and
    the partial products are summed: same math, different summation order."""

    @staticmethod
    def forward(ctx, x, weight, bias, splits):
        ctx.save_for_backward(x, weight)
        ctx.splits = splits
        return torch.addmm(bias, x, weight.t())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        s = ctx.splits
        gx = gy @ weight if ctx.needs_input_grad[0] else None
        r = gy.shape[0] // s
        gw = torch.bmm(gy.reshape(s, r, -1).transpose(1, 2), x.reshape(s, r, -1)).sum(0)
        return gx, gw, gy.sum(0), None


class SplitKLinear(nn.Linear):
    """``nn.Linear`` (same parameters, init and forward values) whose weight
    gradient uses a split-K reduction for large row counts (see
    :class:`_SplitKLinearFn`); small or ragged batches take ``nn.Linear``'s
    own path."""

    ROWS_PER_SPLIT = 512

    def forward(self, x):
        rows = x.shape[0] if x.dim() == 2 else 0
        s = rows // self.ROWS_PER_SPLIT
        if torch.is_grad_enabled() and s >= 8 and rows % self.ROWS_PER_SPLIT == 0:
            return _SplitKLinearFn.apply(x, self.weight, self.bias, s)
        return super().forward(x)


class _FusedPPOLossFn(torch.autograd.Function):
    """SB3 PPO loss head through the HIP kernels of ``salp_ppo_loss``: the
    forward pass also produces d loss / d (mu, log_std, value), which the
    backward pass only scales.  Outputs (loss, stats[pg, vf, entropy,
    clip_fraction]); stats carry no gradient."""

    @staticmethod
    def forward(ctx, mu, log_std, value, actions, old_logp, adv, returns, clip, ent_coef, vf_coef, normalize):
        B = mu.shape[0]
        dev = mu.device
        out = torch.empty(8, dtype=torch.float32, device=dev)
        dmu = torch.empty_like(mu)
        dv = torch.empty_like(value)
        ws = torch.empty(_PPO_WS, dtype=torch.float64, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(_lib.load().salp_ppo_loss(B, _ptr(mu), _ptr(log_std), _ptr(value), _ptr(actions),
                                             _ptr(old_logp), _ptr(adv), _ptr(returns), float(clip),
                                             float(ent_coef), float(vf_coef), int(bool(normalize)), _ptr(ws),
                                             _ptr(out), _ptr(dmu), _ptr(dv), stream))
        ctx.save_for_backward(dmu, dv, out)
        stats = out[1:5].clone()
        ctx.mark_non_differentiable(stats)
        return out[0].clone(), stats

    @staticmethod
    def backward(ctx, g_loss, g_stats):
        dmu, dv, out = ctx.saved_tensors
        return dmu * g_loss, out[5:8] * g_loss, dv * g_loss, None, None, None, None, None, None, None, None


_PPO_WS = 2048   # include/salp.h SALP_PPO_WORKSPACE_DOUBLES
_EP_RETURN = INFO["ep_return"]
_EP_LEN = INFO["ep_len"]


def ppo_loss(mu, log_std, value, actions, old_logp, advantages, returns, clip_range, ent_coef, vf_coef,
             normalize_advantage):
    """Fused SB3 PPO loss (``salp_ppo_loss``): returns (loss, stats) with
    stats = [pg_loss, vf_loss, entropy, clip_fraction]; differentiable in mu
    [B,3], log_std [3] and value [B].  CUDA float32 tensors."""
    ts = (mu, log_std, value, actions, old_logp, advantages, returns)
    B = mu.shape[0]
    shapes = ((B, 3), (3,), (B,), (B, 3), (B,), (B,), (B,))
    for t, shp in zip(ts, shapes):
        if not t.is_cuda or t.dtype != torch.float32 or tuple(t.shape) != shp:
            raise ValueError(f"ppo_loss: expected a float32 CUDA tensor of shape {shp}, got {tuple(t.shape)}")
    return _FusedPPOLossFn.apply(*(t.contiguous() for t in ts), clip_range, ent_coef, vf_coef,
                                 normalize_advantage)


def torch_ppo_loss(mu, log_std, value, actions, old_logp, advantages, returns, clip_range, ent_coef, vf_coef,
                   normalize_advantage):
    """The same loss as torch ops (SB3 PPO.train), the reference for ppo_loss."""
    d = torch.distributions.Normal(mu, log_std.exp().expand_as(mu), validate_args=False)
    lp = d.log_prob(actions).sum(-1)
    ent = d.entropy().sum(-1)
    adv = advantages
    if normalize_advantage and adv.numel() > 1:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(lp - old_logp)
    pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip_range, 1 + clip_range)).mean()
    vf = torch.nn.functional.mse_loss(returns, value)
    ent_loss = -ent.mean()
    loss = pg + ent_coef * ent_loss + vf_coef * vf
    clip = ((ratio - 1).abs() > clip_range).float().mean()
    return loss, torch.stack([pg.detach(), vf.detach(), -ent_loss.detach(), clip.detach()])


def _ortho(layer, gain):
    nn.init.orthogonal_(layer.weight, gain=gain)
    nn.init.zeros_(layer.bias)
    return layer


class ActorCritic(nn.Module):
    """SB3 ``ActorCriticPolicy`` with ``net_arch=dict(pi=[64, 64], vf=[64, 64])``,
    tanh, orthogonal init (sqrt(2) hidden, 0.01 action head, 1 value head) and
    ``log_std_init=0``."""

    def __init__(self, obs_dim, act_dim, hidden=(64, 64)):
        super().__init__()

        def mlp():
            layers, d = [], obs_dim
            for h in hidden:
                layers += [_ortho(SplitKLinear(d, h), math.sqrt(2)), nn.Tanh()]
                d = h
            return nn.Sequential(*layers), d

        self.pi_net, d_pi = mlp()
        self.vf_net, d_vf = mlp()
        self.action_net = _ortho(SplitKLinear(d_pi, act_dim), 0.01)
        self.value_net = _ortho(SplitKLinear(d_vf, 1), 1.0)
        self.log_std = nn.Parameter(torch.zeros(act_dim))

    def value(self, obs):
        return self.value_net(self.vf_net(obs)).squeeze(-1)

    def dist(self, obs):
        mean = self.action_net(self.pi_net(obs))
        return torch.distributions.Normal(mean, self.log_std.exp().expand_as(mean), validate_args=False)

    @torch.no_grad()
    def act(self, obs, generator=None):
        """(action, value, log_prob); the Gaussian noise comes from `generator`
        when given (Normal.sample draws mean + std * N(0, 1) the same way)."""
        d = self.dist(obs)
        if generator is None:
            a = d.sample()
        else:
            a = d.mean + d.stddev * torch.randn(d.mean.shape, generator=generator, device=d.mean.device,
                                                dtype=d.mean.dtype)
        return a, self.value(obs), d.log_prob(a).sum(-1)

    def evaluate(self, obs, actions):
        d = self.dist(obs)
        return self.value(obs), d.log_prob(actions).sum(-1), d.entropy().sum(-1)


def pack_policy(pol, out=None):
    """The ActorCritic's parameters in salp_collect's packed float32 layout
    (include/salp.h SALP_POLICY_*; first-layer inputs zero-padded to
    OBS_DIM_MAX columns).  ``out``: a preallocated [POLICY_SIZE] tensor."""
    lin = [m for m in pol.pi_net if isinstance(m, nn.Linear)] + [m for m in pol.vf_net if isinstance(m, nn.Linear)]
    if len(lin) != 4 or lin[1].in_features != 64 or lin[0].out_features != 64 or lin[0].in_features > OBS_DIM_MAX:
        raise ValueError("salp_collect runs the 64-64 tanh MlpPolicy only")
    p = lin[0].weight
    w = out if out is not None else torch.empty(POLICY_SIZE, dtype=torch.float32, device=p.device)
    w.zero_()

    def put(name, t):
        off, size = POLICY_OFFSETS[name]
        if name.endswith("w1"):
            w[off:off + size].view(64, OBS_DIM_MAX)[:, :t.shape[1]].copy_(t)
        else:
            w[off:off + size].copy_(t.reshape(-1))

    with torch.no_grad():
        for pre, (l1, l2) in (("pi", lin[:2]), ("vf", lin[2:])):
            put(pre + "_w1", l1.weight)
            put(pre + "_b1", l1.bias)
            put(pre + "_w2", l2.weight)
            put(pre + "_b2", l2.bias)
        put("act_w", pol.action_net.weight)
        put("act_b", pol.action_net.bias)
        put("log_std", pol.log_std)
        put("val_w", pol.value_net.weight)
        put("val_b", pol.value_net.bias)
    return w


def sampling_generator(seed, device):
    """The exploration-noise generator of one rank: seeded with (seed, rank),
    so ranks that share initial weights still draw independent actions for
    their own envs (a shared seed would correlate the noise of env i on every
    rank).  Rank 0 of a run keeps the single-process stream."""
    rank = dist.get_rank() if (dist.is_available() and dist.is_initialized()) else 0
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) + 1_000_003 * int(rank))
    return g


def timeout_bootstrap(reward, terminated, truncated, terminal_value, gamma):
    """SB3 ``collect_rollouts``' handling of time limits: an episode cut by
    truncation (not termination) gets ``gamma * V(terminal_obs)`` added to its
    last reward, so GAE does not treat the time limit as a real end.
    Branch-free over the batch (no host sync)."""
    trunc_only = truncated & ~terminated
    return torch.where(trunc_only, reward + gamma * terminal_value, reward)


# Learner-side divergence guard.  The reference integrator diverges for some
# actions (jet_time < dt; tests/test_gpu_parity.py::test_reference_blowup_is_
# reproduced): velocities grow by orders of magnitude for many ticks before
# they overflow to inf/NaN, so an env on its way there first returns huge
# FINITE rewards (100 * (prev_dist - dist), -100 * |avg v_y|) and observations.
# A legitimate step stays far inside these bounds: |reward| <= ~1.5e3 (success
# +500, progress and penalties of a body moving < 1 m/s within 5 m of the
# target), |obs| < 1e2 (metres, m/s, rad).
# HIP-graph capture checks only this thread's calls: with RCCL, the process
# group's watchdog thread keeps querying events while a rank captures
_CAPTURE_MODE = "thread_local"

DIVERGED_OBS_ABS = 1e3
DIVERGED_REWARD_ABS = 1e4


def diverged_mask(obs, reward):
    """Envs whose step shows divergence: non-finite, or beyond the bounds above."""
    return (~torch.isfinite(obs).all(1) | ~torch.isfinite(reward) | (obs.abs() > DIVERGED_OBS_ABS).any(1)
            | (reward.abs() > DIVERGED_REWARD_ABS))


class RolloutBuffer:
    """Device rollout buffer, SB3 layout [n_steps, n_envs, ...] float32."""

    def __init__(self, n_steps, n_envs, obs_dim, act_dim, device):
        z = lambda *s: torch.zeros(s, dtype=torch.float32, device=device)  # noqa: E731
        self.obs = z(n_steps, n_envs, obs_dim)
        self.actions = z(n_steps, n_envs, act_dim)
        self.rewards = z(n_steps, n_envs)
        self.episode_starts = z(n_steps, n_envs)
        self.values = z(n_steps, n_envs)
        self.log_probs = z(n_steps, n_envs)
        self.advantages = z(n_steps, n_envs)
        self.returns = z(n_steps, n_envs)
        self.n_steps, self.n_envs = n_steps, n_envs


def allreduce_gradients(params, group=None):
    """Average gradients over all ranks with ONE flat all-reduce (a single
    bucket: the policy is small, so the all-reduce is latency-bound and one
    message is the cheapest shape for the ring).  No-op without a group."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    flat /= world
    off = 0
    for g in grads:
        k = g.numel()
        g.copy_(flat[off:off + k].view_as(g))
        off += k


class PPO:
    """SB3-style PPO on a :class:`~grasp_lab_salp_amd.vec_env.SalpVecEnv`
    (or anything exposing ``.sim`` = :class:`BatchedSalpEnv`).  Constructor
    arguments and defaults follow SB3's ``PPO`` (and the reference's
    RecurrentPPO values where it sets them)."""

    def __init__(self, policy, env, learning_rate=3e-4, n_steps=2048, batch_size=64, n_epochs=10, gamma=0.99,
                 gae_lambda=0.95, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                 normalize_advantage=True, seed=0, device=None, verbose=0, reset_nonfinite=True,
                 use_graphs=None, fused_loss=None, collect="auto", fused_update=None, max_graph_minibatches=1024):
        if policy not in ("MlpPolicy", None) and not isinstance(policy, nn.Module):
            raise ValueError("policy must be 'MlpPolicy' or an nn.Module")
        if fused_loss and isinstance(policy, nn.Module) and not all(
                hasattr(policy, k) for k in ("action_net", "pi_net", "log_std", "value")):
            raise ValueError("fused_loss=True needs an ActorCritic-shaped policy (action_net, pi_net, log_std, "
                             "value); pass fused_loss=False for a custom policy")
        if collect not in ("auto", "lockstep", "chained"):
            raise ValueError("collect must be 'auto', 'lockstep' or 'chained'")
        self.env = env
        self.sim = getattr(env, "sim", env)
        self.device = self.sim.device if device is None else torch.device(device)
        self.n_envs = self.sim.n_envs
        self.obs_dim = self.sim.obs_dim
        self.act_dim = 3
        torch.manual_seed(int(seed))
        self.policy = (policy if isinstance(policy, nn.Module) else ActorCritic(self.obs_dim, self.act_dim)).to(
            self.device)
        if dist.is_available() and dist.is_initialized():   # identical initial weights on every rank
            for p in self.policy.parameters():
                dist.broadcast(p.data, 0)
        # ... but independent exploration noise per rank (its own env shard)
        self.sample_gen = sampling_generator(seed, self.device)
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._multi = multi
        # the whole minibatch step (forward, loss, backward, clipping, Adam) as
        # the HIP kernels of salp_ppo_mlp_grads / salp_ppo_mlp_apply for the
        # built-in policy on a GPU; torch ops + torch Adam otherwise
        if fused_update and not isinstance(self.policy, ActorCritic):
            raise ValueError("fused_update=True runs the built-in ActorCritic (64-64 tanh MlpPolicy) only")
        if fused_update and self.device.type != "cuda":
            raise ValueError("fused_update=True runs HIP kernels: it needs a ROCm GPU device")
        self.fused_update = (self.device.type == "cuda" and isinstance(self.policy, ActorCritic)
                             and self.policy.pi_net[0].out_features == 64 if fused_update is None
                             else bool(fused_update))
        # HIP graphs: on one rank always; with several ranks for the fused step
        # only, as two graphs (gradient, then clip + Adam) with the RCCL
        # all-reduce of the flat gradient between them, outside any capture
        graphs_ok = self.device.type == "cuda" and (not multi or self.fused_update)
        self.use_graphs = graphs_ok if use_graphs is None else bool(use_graphs) and graphs_ok
        # fused Adam on the GPU: one kernel for all parameters instead of ~4
        # elementwise kernels per parameter tensor (capturable either way)
        fused = self.device.type == "cuda"
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=learning_rate, eps=1e-5,
                                    capturable=self.use_graphs, fused=fused or None)
        self._graph = None
        self._graph_warm = 0
        self._epoch_graph = None   # fused step, one GPU: one graph per chunk of minibatches
        self._rem_graph = None     # and one for the epoch's last m % chunk minibatches
        self.max_graph_minibatches = max(1, int(max_graph_minibatches))
        self._g_clip = None
        self._collect_stream = None
        self._train_stream = None
        self.n_steps, self.batch_size, self.n_epochs = int(n_steps), int(batch_size), int(n_epochs)
        # clip_range may be an SB3-style schedule: f(progress_remaining) -> value
        self.gamma, self.gae_lambda, self.clip_range = gamma, gae_lambda, clip_range
        self._progress = 1.0
        self.ent_coef, self.vf_coef, self.max_grad_norm = ent_coef, vf_coef, max_grad_norm
        self.normalize_advantage = normalize_advantage
        # the loss head runs as the fused HIP kernels of salp_ppo_loss for the
        # built-in policy on a GPU; torch ops otherwise (custom policies)
        self.fused_loss = (self.device.type == "cuda" and isinstance(self.policy, ActorCritic)
                           if fused_loss is None else bool(fused_loss))
        if self.fused_update:
            self._init_fused(learning_rate)
        self.verbose = verbose
        self.reset_nonfinite = reset_nonfinite
        self._nonfinite = torch.zeros((), dtype=torch.int64, device=self.device)
        # finished-episode statistics of the current collection (device, sync-free):
        # return sum, episodes, successes (target reached: terminated), length sum
        self._ep_stats = torch.zeros(4, dtype=torch.float64, device=self.device)
        # minibatch permutations are drawn on the device: SB3 permutes on the
        # host (np.random.permutation), which at n_steps 2048 x 32 768 envs is
        # a 537 MB index array per epoch to build and upload
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.buf = RolloutBuffer(self.n_steps, self.n_envs, self.obs_dim, self.act_dim, self.device)
        self.low = torch.tensor([0.0, 0.0, -1.0], device=self.device)
        self.high = torch.tensor([1.0, 1.0, 1.0], device=self.device)
        self._obs = None
        self._episode_starts = torch.ones(self.n_envs, dtype=torch.float32, device=self.device)
        # auto: the in-kernel collection for the built-in policy on a GPU from
        # 256 env-steps per collection on (config 5 at n_steps 2048: collection
        # 5.76 -> 4.21 s; at n_steps 32 the two take the same time)
        if collect == "auto":
            collect = ("chained" if self.device.type == "cuda" and isinstance(self.policy, ActorCritic)
                       and self.n_steps >= 256 else "lockstep")
        self.collect = collect
        if collect == "chained":
            if not isinstance(self.policy, ActorCritic):
                raise ValueError("collect='chained' evaluates the built-in ActorCritic inside the kernel")
            self._packed = torch.empty(POLICY_SIZE, dtype=torch.float32, device=self.device)
            self._last_obs = torch.empty((self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
            self._noise_seed = int(seed) + 1_000_003 * (dist.get_rank() if multi else 0)
        self.num_timesteps = 0
        self.logger = {}
        self.timing = {"collect_s": 0.0, "gae_s": 0.0, "train_s": 0.0}
        self.history = []   # per iteration: losses, finished-episode mean return, diverged envs

    # --------------------------------------------- fused minibatch step
    def _init_fused(self, lr):
        """Flat gradient and Adam state of salp_ppo_mlp (include/salp.h
        SalpMlpTensor order), the kernels' workspace."""
        L = _lib.load()
        pol = self.policy
        lin = [pol.pi_net[0], pol.pi_net[2], pol.vf_net[0], pol.vf_net[2]]
        if any(m.out_features != 64 for m in lin) or lin[1].in_features != 64 or lin[0].in_features != self.obs_dim:
            raise ValueError("salp_ppo_mlp runs the 64-64 tanh MlpPolicy only")
        self._mlp_tensors = [pol.pi_net[0].weight, pol.pi_net[0].bias, pol.pi_net[2].weight, pol.pi_net[2].bias,
                             pol.action_net.weight, pol.action_net.bias, pol.log_std,
                             pol.vf_net[0].weight, pol.vf_net[0].bias, pol.vf_net[2].weight, pol.vf_net[2].bias,
                             pol.value_net.weight, pol.value_net.bias]
        for t in self._mlp_tensors:
            if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device):
                raise ValueError("policy tensors must be contiguous float32 on the PPO device")
        P = L.salp_ppo_mlp_num_params(self.obs_dim)
        z = lambda n: torch.zeros(n, dtype=torch.float32, device=self.device)  # noqa: E731
        self._f_grads, self._f_m, self._f_v = z(P), z(P), z(P)
        self._f_step, self._f_gnorm = z(1), z(1)
        self._f_ws = torch.empty(L.salp_ppo_mlp_workspace_doubles(self.batch_size, self.obs_dim),
                                 dtype=torch.float64, device=self.device)
        self._f_lr = float(lr)
        self._f_adam = _lib.SalpPpoAdam(obs_dim=self.obs_dim, grads=self._f_grads.data_ptr(),
                                        exp_avg=self._f_m.data_ptr(), exp_avg_sq=self._f_v.data_ptr(),
                                        step=self._f_step.data_ptr(), grad_norm=self._f_gnorm.data_ptr(),
                                        lr=self._f_lr, beta1=0.9, beta2=0.999, eps=1e-5,
                                        max_grad_norm=float(self.max_grad_norm if self.max_grad_norm else 0.0))
        for i, t in enumerate(self._mlp_tensors):
            self._f_adam.params[i] = t.data_ptr()
        # clip + Adam over many blocks (k_mlp_adam, ABI 13), the squared norm's partials written by the
        # gradient reduction itself on one rank (after the all-reduce, by k_mlp_norm, on several);
        # SALP_PPO_APPLY=one keeps the one-block kernel (k_mlp_apply), for A / B runs
        self._f_apply_ws = torch.zeros(_lib.APPLY_WORKSPACE_DOUBLES, dtype=torch.float64, device=self.device)
        self._f_norm_part = None
        if os.environ.get("SALP_PPO_APPLY", "blocks") != "one":
            self._f_adam.workspace = self._f_apply_ws.data_ptr()
            if not self._multi:
                self._f_adam.norm_ready = 1
                self._f_norm_part = self._f_apply_ws.data_ptr()

    def _fused_minibatch(self, idx, acc, part="all", adv_part=None):
        """One SB3 PPO minibatch step through salp_ppo_mlp: gradient of the
        loss over rows `idx` (stats added to `acc`), the gradient all-reduce
        when there are several ranks, then clip_grad_norm_ and Adam.  `part`
        "grads" / "apply" runs only the part before / after the all-reduce
        (the two graphs of a multi-rank learner).  `adv_part`: this minibatch's
        advantage partials from salp_ppo_mlp_adv_partials (an epoch's in one
        launch), else the gradient call computes them."""
        L = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if part == "apply":
            _lib.check(L.salp_ppo_mlp_apply(ctypes.byref(self._f_adam), stream))
            return
        b = self.buf
        m = _lib.SalpPpoMinibatch(batch=idx.numel(), obs_dim=self.obs_dim,
                                  normalize_advantage=int(bool(self.normalize_advantage) and idx.numel() > 1),
                                  idx=idx.data_ptr(), obs=b.obs.data_ptr(), actions=b.actions.data_ptr(),
                                  old_log_prob=b.log_probs.data_ptr(), advantages=b.advantages.data_ptr(),
                                  returns=b.returns.data_ptr(), grads=self._f_grads.data_ptr(),
                                  clip_range=self._clip(), ent_coef=float(self.ent_coef), vf_coef=float(self.vf_coef),
                                  workspace=self._f_ws.data_ptr(), stats=acc.data_ptr(),
                                  adv_part=adv_part.data_ptr() if adv_part is not None else None,
                                  norm_part=self._f_norm_part)
        for i, t in enumerate(self._mlp_tensors):
            m.params[i] = t.data_ptr()
        _lib.check(L.salp_ppo_mlp_grads(ctypes.byref(m), stream))
        if part == "grads":
            return
        self._allreduce_flat_grads()
        _lib.check(L.salp_ppo_mlp_apply(ctypes.byref(self._f_adam), stream))

    def _allreduce_flat_grads(self):
        """Mean of the flat gradient over the ranks (one RCCL message, ~42 KB)."""
        if self._multi:
            dist.all_reduce(self._f_grads)
            self._f_grads /= dist.get_world_size()

    # ---------------------------------------------------------- rollout
    def collect_rollouts(self):
        """n_steps lock-step env-steps into the buffer, then GAE.  Returns the
        HIP events (start, before GAE, after GAE) on the current stream, so
        the split of the GPU timeline is attributed to the right phase."""
        b, sim = self.buf, self.sim
        stream = torch.cuda.current_stream(self.device)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        if self._obs is None:
            self._obs = sim.reset()
        self._ep_stats.zero_()
        if self.collect == "chained":
            return self._collect_chained(ev, stream)
        for t in range(self.n_steps):
            obs = self._obs
            a, v, lp = self._act(t, obs)
            r = sim.step(torch.clamp(a, self.low, self.high), auto_reset=True, want_terminal_obs=True)
            rew = r.reward.float()
            reached = r.terminated.clone()   # the task's own termination: target reached
            bad = None
            if self.reset_nonfinite:
                rew, bad = self._reset_diverged(r, rew)
            # no host sync in the loop: the bootstrap value is computed for every
            # env and selected where the episode was truncated, not terminated
            with torch.no_grad():
                tv = self._terminal_value(r.terminal_obs)
            rew = timeout_bootstrap(rew, r.terminated, r.truncated, tv, self.gamma)
            done = (r.terminated | r.truncated)
            ended = done if bad is None else done & ~bad    # episodes that ended by the task's rules
            ep_ret, ep_len = r.info[:, _EP_RETURN], r.info[:, _EP_LEN]
            zero = torch.zeros_like(ep_ret)
            self._ep_stats += torch.stack([torch.where(ended, ep_ret, zero).sum(), ended.sum().double(),
                                           (ended & reached).sum().double(), torch.where(ended, ep_len, zero).sum()])
            b.obs[t].copy_(obs)
            b.actions[t].copy_(a)
            b.rewards[t].copy_(rew)
            b.episode_starts[t].copy_(self._episode_starts)
            b.values[t].copy_(v)
            b.log_probs[t].copy_(lp)
            self._obs = r.obs
            self._episode_starts = done.float()
        with torch.no_grad():
            last_values = self._last_values().contiguous()
        ev[1].record(stream)
        compute_gae(b.rewards, b.values, b.episode_starts, last_values, self._episode_starts.contiguous(),
                    self.gamma, self.gae_lambda, b.advantages, b.returns)
        ev[2].record(stream)
        return ev

    # hooks of the lock-step collection (RecurrentPPO carries LSTM states through them)
    def _act(self, t, obs):
        """(action, value, log_prob) of step t's observations."""
        return self.policy.act(obs, generator=self.sample_gen)

    def _terminal_value(self, terminal_obs):
        """V(terminal observation) for the timeout bootstrap."""
        return self.policy.value(terminal_obs)

    def _last_values(self):
        """V(observation after the last step) for GAE."""
        return self.policy.value(self._obs)

    def _collect_chained(self, ev, stream):
        """collect_rollouts on salp_collect: the same buffers, bootstrap and
        divergence guard, evaluated per env at its own env-step boundaries
        inside the simulation kernel (include/salp.h)."""
        b = self.buf
        w = pack_policy(self.policy, self._packed)
        if self._obs is not self._last_obs:   # salp_collect takes the first observation from last_obs
            self._last_obs.copy_(self._obs)
        guard = self.reset_nonfinite
        self.sim.collect(w, self.n_steps, {"obs": b.obs, "actions": b.actions, "rewards": b.rewards,
                                           "episode_starts": b.episode_starts, "values": b.values,
                                           "log_probs": b.log_probs},
                         self._episode_starts, self._last_obs, self._ep_stats, self._nonfinite.view(1),
                         noise_seed=self._noise_seed, gamma=self.gamma,
                         diverged_obs_abs=DIVERGED_OBS_ABS if guard else 0.0,
                         diverged_reward_abs=DIVERGED_REWARD_ABS if guard else 0.0)
        self._obs = self._last_obs
        with torch.no_grad():
            last_values = self.policy.value(self._obs).contiguous()
        ev[1].record(stream)
        compute_gae(b.rewards, b.values, b.episode_starts, last_values, self._episode_starts.contiguous(),
                    self.gamma, self.gae_lambda, b.advantages, b.returns)
        ev[2].record(stream)
        return ev

    def _reset_diverged(self, r, rew):
        """The reference integrator diverges for some actions (jet_time < dt,
        tests/test_gpu_parity.py::test_reference_blowup_is_reproduced) and its
        env then returns huge, later NaN, observations and rewards until the
        500-cycle timeout.  A learner cannot consume those: envs flagged by
        :func:`diverged_mask` are reset on the spot and the step is recorded as
        a termination with reward 0 (no bootstrap from a diverged state).
        Sync-free: the masked reset is a no-op where the mask is all zero.
        The guard looks at the step's own observation: the terminal one where
        the episode ended (r.obs is already the auto-reset observation there),
        as salp_collect does; an env that ended its episode is not reset a
        second time.  Returns (reward, diverged mask)."""
        done = r.terminated | r.truncated
        seen = torch.where(done.unsqueeze(1), r.terminal_obs, r.obs)
        bad = diverged_mask(seen, rew)
        self._nonfinite = self._nonfinite + bad.sum()
        again = bad & ~done
        fresh = self.sim.reset(mask=again)
        col = again.unsqueeze(1)
        r.obs.copy_(torch.where(col, fresh, r.obs))
        r.truncated |= bad
        r.terminated |= bad     # terminal: no gamma * V(terminal_obs) bootstrap
        return torch.where(bad, torch.zeros_like(rew), rew), bad

    @property
    def nonfinite_resets(self):
        """Envs reset because their state diverged (host int; syncs)."""
        return int(self._nonfinite)

    def _clip(self):
        c = self.clip_range
        return float(c(self._progress)) if callable(c) else float(c)

    # ----------------------------------------------------------- update
    def _minibatch(self, idx, acc):
        """One SB3 PPO gradient step on rollout rows `idx`; adds
        (pg_loss, vf_loss, entropy, clip_fraction) to `acc`."""
        if self.fused_update:
            return self._fused_minibatch(idx, acc)
        b, pol = self.buf, self.policy
        N = self.n_steps * self.n_envs
        obs, act = b.obs.reshape(N, -1)[idx], b.actions.reshape(N, -1)[idx]
        rows = (b.log_probs.reshape(N)[idx], b.advantages.reshape(N)[idx], b.returns.reshape(N)[idx])
        norm = self.normalize_advantage and idx.numel() > 1
        if self.fused_loss:
            mean = pol.action_net(pol.pi_net(obs))
            loss, stats = ppo_loss(mean, pol.log_std, pol.value(obs), act, *rows, self._clip(), self.ent_coef,
                                   self.vf_coef, norm)
        else:   # any policy exposing evaluate(obs, actions) -> (value, log_prob, entropy)
            v, lp, ent = pol.evaluate(obs, act)
            old_lp, adv, ret = rows
            if norm:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            ratio = torch.exp(lp - old_lp)
            cr = self._clip()
            pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - cr, 1 + cr)).mean()
            vf = torch.nn.functional.mse_loss(ret, v)
            ent_loss = -ent.mean()
            loss = pg + self.ent_coef * ent_loss + self.vf_coef * vf
            clip = ((ratio - 1).abs() > cr).float().mean()
            stats = torch.stack([pg.detach(), vf.detach(), -ent_loss.detach(), clip.detach()])
        loss.backward()
        allreduce_gradients(list(pol.parameters()))
        nn.utils.clip_grad_norm_(pol.parameters(), self.max_grad_norm)
        self.opt.step()
        acc += stats

    def _graphed_minibatch(self, idx):
        """The same step through a HIP graph: three eager warm-up steps on a
        side stream, then one capture, then replays (static index / stats
        buffers; Adam is capturable).  The fused step allocates nothing and
        reads only persistent buffers: it is captured on its first call and
        the graph is kept across updates."""
        if self._graph is not None and self._g_clip != self._clip():
            # a clip_range schedule moved: the value captured in the graph is
            # stale (fused and torch steps alike; the torch step's warm-up is
            # done, so it recaptures at once)
            self._graph = None
        if self._graph is None and self.fused_update:
            if self._graph_warm == 0:
                self._g_idx = torch.empty_like(idx)
                self._g_acc = torch.zeros(4, device=self.device)
            self._g_idx.copy_(idx)
            self._g_clip = self._clip()
            self._graph = torch.cuda.CUDAGraph()
            if self._multi:   # gradient graph | all-reduce (eager) | clip + Adam graph
                with torch.cuda.graph(self._graph, capture_error_mode=_CAPTURE_MODE):
                    self._fused_minibatch(self._g_idx, self._g_acc, part="grads")
                self._graph_apply = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._graph_apply, capture_error_mode=_CAPTURE_MODE):
                    self._fused_minibatch(self._g_idx, self._g_acc, part="apply")
            else:
                with torch.cuda.graph(self._graph, capture_error_mode=_CAPTURE_MODE):
                    self._minibatch(self._g_idx, self._g_acc)
            self._graph_warm = 1
        elif self._graph is None:
            if self._graph_warm == 0:
                self._g_idx = torch.empty_like(idx)
                self._g_acc = torch.zeros(4, device=self.device)
            self._g_idx.copy_(idx)
            if self._graph_warm < 3:
                side = torch.cuda.Stream(self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    self.opt.zero_grad(set_to_none=True)
                    self._minibatch(self._g_idx, self._g_acc)
                torch.cuda.current_stream(self.device).wait_stream(side)
                self._graph_warm += 1
                return
            self.opt.zero_grad(set_to_none=True)
            self._g_clip = self._clip()
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph, capture_error_mode=_CAPTURE_MODE):
                self._minibatch(self._g_idx, self._g_acc)
        else:
            self._g_idx.copy_(idx)
        self._graph.replay()
        if self.fused_update and self._multi:
            self._allreduce_flat_grads()
            self._graph_apply.replay()

    def train(self):
        """n_epochs passes of minibatch updates over the rollout buffer.  The
        minibatch graph is captured once and replayed for every update.  A
        torch-step graph (custom policies) kept across updates went stale when
        eager GEMMs ran on the stream it replays on between updates (the
        lock-step collection's policy forwards: the captured GEMMs then read a
        BLAS workspace the eager ones had reused), so learn()
        runs the collection on a stream of its own; a torch-step graph is
        still captured afresh per update when the buffer leaves an eager tail
        minibatch (its GEMMs run on the replay stream)."""
        N = self.n_steps * self.n_envs
        if self.fused_update and self.use_graphs and not self._multi and N % self.batch_size == 0:
            return self._train_epoch_graphs()
        if not self.fused_update and N % self.batch_size:
            self._graph, self._graph_warm = None, 0   # eager tail minibatch: recapture (see docstring)
        acc = torch.zeros(4, device=self.device)
        steps = 0
        for _ in range(self.n_epochs):
            perm = torch.randperm(N, generator=self.gen, device=self.device)
            for s in range(0, N, self.batch_size):
                idx = perm[s:s + self.batch_size]
                if self.use_graphs and idx.numel() == self.batch_size:
                    self._graphed_minibatch(idx)
                else:
                    if not self.fused_update:
                        self.opt.zero_grad(set_to_none=False)
                    self._minibatch(idx, acc)
                steps += 1
        if self.use_graphs and self._graph_warm > 0:
            acc = acc + self._g_acc
            self._g_acc.zero_()
        vals = (acc / max(steps, 1)).tolist()
        return dict(zip(("pg_loss", "vf_loss", "entropy", "clip_frac"), vals))

    def _graph_chunk(self, m):
        """Minibatches per captured graph: the epoch's `m` minibatches, at most
        max_graph_minibatches (a graph's node count and its capture loop stay
        bounded whatever n_steps x n_envs / batch_size is: SB3's default
        batch_size 64 at 32 768 envs x 2 048 steps would otherwise be a million
        minibatches in one graph).  m % chunk minibatches are left for a second,
        shorter graph (_train_epoch_graphs)."""
        return min(m, self.max_graph_minibatches)

    def _train_epoch_graphs(self):
        """train() for the fused step on one GPU: every minibatch reads its rows
        from a slice of one persistent index buffer, so a chunk of C
        minibatches (4 kernels each) is one HIP graph, captured once and
        replayed M // C times per epoch (M minibatches per epoch; C = M, one
        graph per epoch, unless M exceeds max_graph_minibatches), each time
        after the next C x batch_size indices of the epoch's permutation are
        copied into it; the last M % C minibatches are a second graph, captured
        once too.  A graph opens with one launch of the advantage partials of
        all its minibatches (salp_ppo_mlp_adv_partials, the sums each
        minibatch's gradient call would otherwise launch for itself).  The same
        results as minibatch by minibatch (no per-minibatch launch from
        Python)."""
        N = self.n_steps * self.n_envs
        bs = self.batch_size
        m = N // bs
        c = self._graph_chunk(m)
        rem = m % c
        fresh = False
        if self._epoch_graph is None or self._g_clip != self._clip():
            if self._epoch_graph is None:
                self._perm = torch.empty(N, dtype=torch.int64, device=self.device)
                # the graph's index buffer: the permutation itself when one
                # graph covers the epoch, else a chunk-sized copy target
                self._gperm = self._perm if c == m else torch.empty(c * bs, dtype=torch.int64, device=self.device)
                self._g_acc = torch.zeros(4, device=self.device)
            torch.randperm(N, generator=self.gen, device=self.device, out=self._perm)
            if c != m:
                self._gperm.copy_(self._perm[:c * bs])
            self._g_clip = self._clip()
            # the chunk's advantage partials in one launch (salp_ppo_mlp_adv_partials), then its minibatches
            self._g_advp = torch.empty(c * _lib.ADV_PARTIAL_DOUBLES, dtype=torch.float64, device=self.device)

            epoch_adv = os.environ.get("SALP_PPO_EPOCH_ADV", "1") != "0"   # 0: per minibatch (A/B runs)

            def chunk(k_mb):
                if epoch_adv:
                    L = _lib.load()
                    stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
                    _lib.check(L.salp_ppo_mlp_adv_partials(bs, k_mb, self._gperm.data_ptr(),
                                                           self.buf.advantages.data_ptr(), self._g_advp.data_ptr(),
                                                           stream))
                for k in range(k_mb):
                    self._fused_minibatch(self._gperm[k * bs:(k + 1) * bs], self._g_acc,
                                          adv_part=self._g_advp[k * _lib.ADV_PARTIAL_DOUBLES:] if epoch_adv else None)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                chunk(c)
            self._epoch_graph = g
            self._rem_graph = None
            if rem:   # the ragged tail: a graph of its own over the head of the same buffers
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, capture_error_mode=_CAPTURE_MODE):
                    chunk(rem)
                self._rem_graph = gr
            fresh = True
        for e in range(self.n_epochs):
            if not (fresh and e == 0):   # the capture's permutation serves the first epoch
                torch.randperm(N, generator=self.gen, device=self.device, out=self._perm)
            for k in range(m // c):
                if c != m and not (fresh and e == 0 and k == 0):
                    self._gperm.copy_(self._perm[k * c * bs:(k + 1) * c * bs])
                self._epoch_graph.replay()
            if rem:
                self._gperm[:rem * bs].copy_(self._perm[(m - rem) * bs:m * bs])
                self._rem_graph.replay()
        vals = (self._g_acc / (self.n_epochs * m)).tolist()
        self._g_acc.zero_()
        return dict(zip(("pg_loss", "vf_loss", "entropy", "clip_frac"), vals))

    def learn(self, total_timesteps, log_interval=1):
        """Collect + GAE + update until ``total_timesteps`` env-steps.  The
        phase timings come from HIP events on the stream (collection, GAE and
        update are attributed where the GPU ran them); ``history`` gets one
        row per iteration."""
        it = 0
        start_steps = self.num_timesteps
        stream = torch.cuda.current_stream(self.device)
        if self._collect_stream is None and self.device.type == "cuda":
            self._collect_stream = torch.cuda.Stream(self.device)
            self._train_stream = torch.cuda.Stream(self.device)
        while self.num_timesteps < total_timesteps:
            done_frac = (self.num_timesteps - start_steps) / max(total_timesteps - start_steps, 1)
            self._progress = 1.0 - done_frac
            div0 = self._nonfinite.clone()
            if self._collect_stream is not None:
                # eager collection (policy GEMMs) off the stream the update
                # graph replays on (train() docstring); ordered both ways
                cs = self._collect_stream
                cs.wait_stream(stream)
                with torch.cuda.stream(cs):
                    ev = self.collect_rollouts()
                stream.wait_stream(cs)
            else:
                ev = self.collect_rollouts()
            if self._train_stream is not None:
                # the update (warm-up, captures and replays) on a stream the
                # learner owns: eager work a caller issues between learn()
                # calls (predict, an evaluation loop) never lands on the
                # stream the kept graphs replay on
                ts = self._train_stream
                ts.wait_stream(stream)
                with torch.cuda.stream(ts):
                    self.logger = self.train()
                stream.wait_stream(ts)
            else:
                self.logger = self.train()
            end = torch.cuda.Event(enable_timing=True)
            end.record(stream)
            end.synchronize()
            self.timing["collect_s"] += ev[0].elapsed_time(ev[1]) / 1e3
            self.timing["gae_s"] += ev[1].elapsed_time(ev[2]) / 1e3
            self.timing["train_s"] += ev[2].elapsed_time(end) / 1e3
            self.num_timesteps += self.n_steps * self.n_envs
            it += 1
            if self.collect == "chained":
                # the two-wave collection kernel never hangs the GPU: a wave that
                # waits for its partner in vain gives up, and its envs' buffers
                # are invalid (include/salp.h salp_pair_timeouts)
                self.sim.check_pair()
            ret_sum, n_ep, n_succ, len_sum = self._ep_stats.tolist()
            row = {"iteration": len(self.history) + 1, "timesteps": self.num_timesteps, **self.logger,
                   "episodes": int(n_ep), "ep_return_mean": ret_sum / n_ep if n_ep else None,
                   "success_rate": n_succ / n_ep if n_ep else None,
                   "ep_len_mean": len_sum / n_ep if n_ep else None,
                   "diverged_envs": int(self._nonfinite - div0)}
            self.history.append(row)
            if self.verbose and it % log_interval == 0:
                print(row, flush=True)
        return self
