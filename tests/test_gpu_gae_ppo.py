"""GAE kernel (salp_gae) bit-identical to the SB3 restatement (oracle/gae.py),
and the on-device PPO loop (grasp_lab_salp_amd.ppo) running end to end."""
import numpy as np
import pytest
import torch

from oracle.gae import compute_returns_and_advantage

pytestmark = pytest.mark.gpu


def _case(rng, T, n, p_start=0.05):
    rew = (rng.normal(size=(T, n)) * 30).astype(np.float32)
    rew[rng.random((T, n)) < 0.01] += 500.0     # terminal bonuses / penalties
    val = (rng.normal(size=(T, n)) * 10).astype(np.float32)
    st = (rng.random((T, n)) < p_start).astype(np.float32)
    lv = (rng.normal(size=n) * 10).astype(np.float32)
    dn = rng.random(n) < 0.1
    return rew, val, st, lv, dn


@pytest.mark.parametrize("T,n", [(1, 1), (1, 300), (5, 257), (16, 64), (37, 1000), (64, 4096)])
def test_gae_bit_identical_to_oracle(T, n):
    from grasp_lab_salp_amd.ppo import compute_gae
    rng = np.random.default_rng(T * 1000 + n)
    rew, val, st, lv, dn = _case(rng, T, n)
    cu = lambda x: torch.tensor(x, dtype=torch.float32, device="cuda").contiguous()  # noqa: E731
    adv, ret = compute_gae(cu(rew), cu(val), cu(st), cu(lv), cu(dn.astype(np.float32)), 0.99, 0.95)
    a_ref, r_ref = compute_returns_and_advantage(rew, val, st, lv, dn, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), a_ref)
    assert np.array_equal(ret.cpu().numpy(), r_ref)


def test_gae_full_size_sampled_envs():
    """Config-5 size (32 768 envs x 256 steps): every env's column depends only
    on that env, so a sample of columns checked against the oracle covers it."""
    from grasp_lab_salp_amd.ppo import compute_gae
    T, n = 256, 32768
    g = torch.Generator(device="cuda").manual_seed(7)
    rew = torch.randn(T, n, device="cuda", generator=g) * 30
    val = torch.randn(T, n, device="cuda", generator=g) * 10
    st = (torch.rand(T, n, device="cuda", generator=g) < 0.02).float()
    lv = torch.randn(n, device="cuda", generator=g)
    dn = (torch.rand(n, device="cuda", generator=g) < 0.1).float()
    adv, ret = compute_gae(rew, val, st, lv, dn)
    cols = torch.randperm(n, generator=torch.Generator().manual_seed(1))[:512].sort().values
    sub = lambda x: x[:, cols].cpu().numpy()  # noqa: E731
    a_ref, r_ref = compute_returns_and_advantage(sub(rew), sub(val), sub(st), lv[cols].cpu().numpy(),
                                                 dn[cols].cpu().numpy() != 0)
    assert np.array_equal(sub(adv), a_ref) and np.array_equal(sub(ret), r_ref)


def test_gae_rejects_bad_shapes():
    from grasp_lab_salp_amd.ppo import compute_gae
    x = torch.zeros(4, 8, device="cuda")
    with pytest.raises(ValueError):
        compute_gae(x, x, x, torch.zeros(7, device="cuda"), torch.zeros(8, device="cuda"))
    with pytest.raises(ValueError):
        compute_gae(x.double(), x, x, torch.zeros(8, device="cuda"), torch.zeros(8, device="cuda"))


def test_ppo_rollout_gae_and_learning():
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(512, seed=3, infos=False)
    model = PPO("MlpPolicy", env, n_steps=8, batch_size=1024, n_epochs=2, seed=0)
    model.collect_rollouts()
    torch.cuda.synchronize()
    b = model.buf
    # the buffer's GAE is SB3's, recomputed on the host from the same buffer
    with torch.no_grad():
        lv = model.policy.value(model._obs).cpu().numpy()
    a_ref, r_ref = compute_returns_and_advantage(b.rewards.cpu().numpy(), b.values.cpu().numpy(),
                                                 b.episode_starts.cpu().numpy(), lv,
                                                 model._episode_starts.cpu().numpy() != 0)
    assert np.array_equal(b.advantages.cpu().numpy(), a_ref)
    assert np.array_equal(b.returns.cpu().numpy(), r_ref)
    assert b.episode_starts[0].eq(1).all()          # first step of every env starts an episode
    p0 = torch.cat([p.detach().reshape(-1) for p in model.policy.parameters()]).clone()
    model.learn(total_timesteps=2 * 8 * 512)
    assert model.num_timesteps == 2 * 8 * 512
    for k in ("pg_loss", "vf_loss", "entropy"):
        assert np.isfinite(model.logger[k]), k
    p1 = torch.cat([p.detach().reshape(-1) for p in model.policy.parameters()])
    assert not torch.equal(p0, p1)
    env.close()


def test_graphed_update_equals_eager_update():
    """The HIP-graph minibatch update replays exactly the eager computation."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    params = []
    for graphs in (False, True):
        env = SalpVecEnv(256, seed=5, infos=False)
        model = PPO("MlpPolicy", env, n_steps=8, batch_size=256, n_epochs=3, seed=1, use_graphs=graphs)
        model.learn(total_timesteps=8 * 256)   # one rollout + one update (identical data)
        params.append(torch.cat([p.detach().reshape(-1) for p in model.policy.parameters()]).cpu())
        captured = model._graph is not None or model._epoch_graph is not None
        assert model.use_graphs == graphs and captured == graphs
        env.close()
    # same data and steps; only Adam's capturable (tensor-step) arithmetic differs by rounding
    assert torch.allclose(params[0], params[1], rtol=1e-4, atol=1e-6)


def _flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.policy.parameters()]).clone()


def test_fused_and_unfused_train_agree_on_the_same_buffer():
    """One PPO.train() with the fused HIP loss head and one with the torch
    loss, from the same weights on the same rollout buffer and minibatch order:
    parameters agree to float32 rounding (whole-update check)."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(256, seed=4, infos=False)
    # the torch update path with either loss head (the fused whole-step kernels
    # are checked against this path in tests/test_gpu_ppo_mlp.py)
    a = PPO("MlpPolicy", env, n_steps=4, batch_size=256, n_epochs=2, seed=2, use_graphs=False, fused_loss=True,
            fused_update=False)
    b = PPO("MlpPolicy", env, n_steps=4, batch_size=256, n_epochs=2, seed=2, use_graphs=False, fused_loss=False,
            fused_update=False)
    b.policy.load_state_dict(a.policy.state_dict())
    # plain SGD on both: Adam's per-parameter normalisation would turn float32
    # noise in near-zero gradients into +-lr steps and hide the comparison
    a.opt = torch.optim.SGD(a.policy.parameters(), lr=1e-2)
    b.opt = torch.optim.SGD(b.policy.parameters(), lr=1e-2)
    a.collect_rollouts()
    for k in ("obs", "actions", "rewards", "episode_starts", "values", "log_probs", "advantages", "returns"):
        getattr(b.buf, k).copy_(getattr(a.buf, k))
    b.gen.set_state(a.gen.get_state())
    la, lb = a.train(), b.train()
    pa, pb = _flat(a), _flat(b)
    assert torch.allclose(pa, pb, rtol=1e-4, atol=1e-6), (pa - pb).abs().max()
    for k in la:
        assert abs(la[k] - lb[k]) <= 1e-4 * max(1.0, abs(lb[k])), (k, la[k], lb[k])
    env.close()


def test_diverged_envs_are_reset_without_bootstrap():
    """The reference's blow-up action (test_reference_blowup_is_reproduced)
    on 4 of 8 envs: the learner's guard resets exactly those envs, records the
    step as a termination (no timeout bootstrap) with reward 0, and the next
    observation is the fresh reset observation."""
    from grasp_lab_salp_amd._abi import FIELD
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(8, seed=0, infos=False)
    model = PPO("MlpPolicy", env, n_steps=2, batch_size=16, n_epochs=1, seed=0)
    sim = model.sim
    sim.reset()
    act = torch.full((8, 3), 0.5, device="cuda")
    act[:4] = torch.tensor([0.0904393, 0.06936062, -0.76570743], device="cuda")
    r = sim.step(act, auto_reset=True, want_terminal_obs=True)
    raw = r.reward.float().clone()
    rew, bad = model._reset_diverged(r, r.reward.float())
    assert bad.tolist() == [True] * 4 + [False] * 4
    assert model.nonfinite_resets == 4
    assert torch.isfinite(r.obs).all() and torch.isfinite(rew).all()
    assert torch.equal(rew[:4], torch.zeros(4, device="cuda")) and torch.equal(rew[4:], raw[4:])
    assert r.terminated[:4].all() and r.truncated[:4].all()
    st = sim.get_state()
    assert (st[FIELD["ep_len"], :4] == 0).all()
    assert torch.isfinite(st[FIELD["v0"]:FIELD["ang2"] + 1, :4]).all()


def test_guard_sees_the_terminal_observation_of_an_ended_episode():
    """the blow-up action on 4 of 8 envs with max_cycles = 1, so the
    diverging step also ends the episode (time limit) and auto-reset already
    replaced r.obs by the fresh observation.  The guard must judge the
    terminal observation (as salp_collect does), zero the reward without a
    bootstrap, and not reset those envs a second time."""
    from grasp_lab_salp_amd._abi import FIELD, default_params
    from grasp_lab_salp_amd.ppo import PPO, diverged_mask
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(8, params=default_params(max_cycles=1), seed=0, infos=False)
    model = PPO("MlpPolicy", env, n_steps=2, batch_size=16, n_epochs=1, seed=0)
    sim = model.sim
    sim.reset()
    ep0 = sim.get_state()[FIELD["episode"]].clone()
    act = torch.full((8, 3), 0.5, device="cuda")
    act[:4] = torch.tensor([0.0904393, 0.06936062, -0.76570743], device="cuda")
    r = sim.step(act, auto_reset=True, want_terminal_obs=True)
    assert r.truncated.all()
    assert diverged_mask(r.terminal_obs, torch.zeros(8, device="cuda")).tolist() == [True] * 4 + [False] * 4
    assert torch.isfinite(r.obs).all()   # auto-reset observations
    fresh = r.obs.clone()
    rew, bad = model._reset_diverged(r, r.reward.float())
    assert bad.tolist() == [True] * 4 + [False] * 4
    assert torch.equal(rew[:4], torch.zeros(4, device="cuda"))
    assert r.terminated[:4].all()           # no gamma * V(terminal_obs) bootstrap
    # one reset per ended episode: the episode counter moved by exactly one
    assert torch.equal(sim.get_state()[FIELD["episode"]], ep0 + 1)
    assert torch.equal(r.obs, fresh)


def test_timeout_bootstrap_in_collection():
    """max_cycles = 1: every env-step ends by the time limit, so every buffer
    reward is the env reward + gamma * V(terminal_obs) (SB3 collect_rollouts)."""
    from grasp_lab_salp_amd._abi import default_params
    from grasp_lab_salp_amd.ppo import timeout_bootstrap, PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    p = default_params(max_cycles=1)
    env = SalpVecEnv(64, params=p, seed=6, infos=False)
    model = PPO("MlpPolicy", env, n_steps=1, batch_size=64, n_epochs=1, seed=3)
    model.collect_rollouts()
    twin = SalpVecEnv(64, params=p, seed=6, infos=False)
    twin.sim.reset()
    r = twin.sim.step(torch.clamp(model.buf.actions[0], model.low, model.high), auto_reset=True,
                      want_terminal_obs=True)
    assert r.truncated.all()
    with torch.no_grad():
        tv = model.policy.value(r.terminal_obs)
    want = timeout_bootstrap(r.reward.float(), r.terminated, r.truncated, tv, model.gamma)
    ok = ~r.terminated
    assert torch.equal(model.buf.rewards[0][ok], want[ok])
    assert not torch.equal(model.buf.rewards[0][ok], r.reward.float()[ok])


def test_collection_is_identical_in_sorted_and_env_order():
    """PPO collection through salp_step: the sorted lock-step launch order
    (default at this size) and env order fill identical rollout buffers."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    bufs = []
    for mode in (1, 0):
        env = SalpVecEnv(4096, seed=9, infos=False)
        env.sim.set_lockstep_order(mode)
        model = PPO("MlpPolicy", env, n_steps=6, batch_size=4096, n_epochs=1, seed=5)
        model.collect_rollouts()
        torch.cuda.synchronize()
        b = model.buf
        bufs.append([getattr(b, k).clone() for k in ("obs", "actions", "rewards", "episode_starts", "values",
                                                      "log_probs", "advantages", "returns")])
        assert all(torch.isfinite(t).all() for t in bufs[-1])
        env.close()
    for x, y in zip(*bufs):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))


def test_graphed_update_matches_eager_after_several_collections():
    """The torch-step HIP graph (custom policies), captured in the first
    update and KEPT, equals the same minibatch run eagerly from the same
    parameters and Adam state in updates 2-5, with lock-step collections
    (eager policy GEMMs) in between: n_steps 32 x 10 epochs, the setting in
    which a kept graph went stale before the collection moved to its own
    stream (tools/debug_ppo_graph_keep.py, profiles/r3i_torch_graph_keep_sweep.jsonl)."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(32768, seed=0, infos=False)
    model = PPO("MlpPolicy", env, n_steps=32, batch_size=32768, n_epochs=10, seed=0, use_graphs=True,
                fused_update=False, collect="lockstep")   # the torch path (the fused step: test_gpu_ppo_mlp.py)
    seen, graphs = {}, set()
    inner = model._graphed_minibatch

    def tensors():
        out = []
        for p in model.policy.parameters():
            out.append(p.data)
            out += [v for v in model.opt.state.get(p, {}).values() if torch.is_tensor(v)]
        return out

    def check(idx):
        upd = len(model.history) + 1
        if model._graph is None or upd < 2 or upd in seen:
            return inner(idx)
        graphs.add(id(model._graph))
        pre = [t.clone() for t in tensors()]
        inner(idx)
        g_graph = [p.grad.clone() for p in model.policy.parameters()]
        post = [t.clone() for t in tensors()]
        keep = [p.grad for p in model.policy.parameters()]
        for t, s in zip(tensors(), pre):
            t.copy_(s)
        for p in model.policy.parameters():
            p.grad = None
        model._minibatch(model._g_idx, torch.zeros(4, device=model.device))
        seen[upd] = all(torch.equal(a, p.grad) for a, p in zip(g_graph, model.policy.parameters()))
        for p, g in zip(model.policy.parameters(), keep):
            p.grad = g
        for t, s in zip(tensors(), post):
            t.copy_(s)

    model._graphed_minibatch = check
    model.learn(5 * 32 * 32768)
    assert sorted(seen) == [2, 3, 4, 5] and all(seen.values()), seen
    assert len(graphs) == 1, "the graph was recaptured"
    assert all(torch.isfinite(p).all() for p in model.policy.parameters())
    assert all(r["vf_loss"] == r["vf_loss"] for r in model.history)
    env.close()


def _graph_vs_eager_checker(model):
    """Wrap model._graphed_minibatch: at the first graphed minibatch of every
    update from the second on, replay the graph, then rerun the same minibatch
    eagerly from the same parameters / Adam state and record whether the
    gradients agree bit for bit (the graph's results are kept)."""
    seen, graphs = {}, []
    inner = model._graphed_minibatch

    def tensors():
        out = []
        for p in model.policy.parameters():
            out.append(p.data)
            out += [v for v in model.opt.state.get(p, {}).values() if torch.is_tensor(v)]
        return out

    def check(idx):
        upd = len(model.history) + 1
        if upd < 2 or upd in seen:
            return inner(idx)
        pre = [t.clone() for t in tensors()]
        inner(idx)
        graphs.append(model._graph)   # the object itself: a freed graph's id() can be reused
        g_graph = [p.grad.clone() for p in model.policy.parameters()]
        post = [t.clone() for t in tensors()]
        keep = [p.grad for p in model.policy.parameters()]
        for t, s in zip(tensors(), pre):
            t.copy_(s)
        for p in model.policy.parameters():
            p.grad = None
        model._minibatch(model._g_idx, torch.zeros(4, device=model.device))
        seen[upd] = all(torch.equal(a, p.grad) for a, p in zip(g_graph, model.policy.parameters()))
        for p, g in zip(model.policy.parameters(), keep):
            p.grad = g
        for t, s in zip(tensors(), post):
            t.copy_(s)

    model._graphed_minibatch = check
    return seen, graphs


def test_torch_graph_follows_a_clip_range_schedule():
    """the torch-step graph bakes clip_range in as a constant; with
    an SB3-style callable schedule it is recaptured whenever the value moves,
    so every update's graphed step equals the eager step at that update's clip."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(4096, seed=2, infos=False)
    model = PPO("MlpPolicy", env, n_steps=16, batch_size=4096, n_epochs=4, seed=0, use_graphs=True,
                fused_update=False, collect="lockstep", clip_range=lambda progress: 0.05 + 0.25 * progress)
    seen, graphs = _graph_vs_eager_checker(model)
    model.learn(4 * 16 * 4096)
    assert sorted(seen) == [2, 3, 4] and all(seen.values()), seen
    assert len({id(g) for g in graphs}) == 3, "one capture per clip value"
    env.close()


def test_eager_forward_between_learn_calls_leaves_the_kept_graph_exact():
    """the update runs on a stream the learner owns, so an eager
    policy forward on the default stream between two learn() calls (predict,
    an evaluation loop) cannot leave the kept torch-step graph reading a stale
    BLAS workspace: graphed == eager in updates 2-4, one graph."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(4096, seed=4, infos=False)
    model = PPO("MlpPolicy", env, n_steps=16, batch_size=4096, n_epochs=4, seed=0, use_graphs=True,
                fused_update=False, collect="lockstep")
    seen, graphs = _graph_vs_eager_checker(model)
    probe = torch.randn(4096, env.sim.obs_dim, device=model.device)
    for _ in range(4):
        model.learn(model.num_timesteps + 16 * 4096)
        with torch.no_grad():   # eager GEMMs on the default stream, as an evaluation callback would issue
            for _ in range(3):
                model.policy.value(probe)
                model.policy.act(probe)
    assert sorted(seen) == [2, 3, 4] and all(seen.values()), seen
    assert len({id(g) for g in graphs}) == 1, "the graph was recaptured"
    env.close()
