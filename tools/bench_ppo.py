"""BASELINE.json config 5: PPO on 32 768 envs per GPU with the HIP GAE scan.

    python tools/bench_ppo.py [--n-envs 32768] [--n-steps 32] [--iters 2] [--trend-iters 0]
    python -m torch.distributed.run --nproc-per-node N tools/bench_ppo.py ...

Prints one JSON line: full-iteration env-steps/s (collection + GAE + update,
max time over ranks), the split (HIP events on the stream: collection, GAE and
update each where the GPU ran them), the per-iteration history (losses, mean
return of the episodes that ended, envs reset by the divergence guard), and the
GAE kernel alone against the HBM roofline (12 B read + 8 B written per (step,
env)).  --trend-iters K first runs K untimed iterations and reports their
history (a learning trend), then the timed ones.

The reference's RecurrentPPO uses n_steps 2048, batch 64 with 4 envs
(src/train_robot_recurrent_ppo.py:91-93): 128 minibatches per epoch.  At
32 768 envs the buffer of n_steps 2048 (MLP policy: obs, actions, rewards,
starts, values, log-probs, advantages, returns = 19 floats per (step, env),
5.1 GB) fits in HBM easily; batch 64 would mean 1 048 576 minibatches per
epoch, so the batch is scaled with the env count (default 32 768).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0


def gae_roofline(T, n, reps=20):
    from grasp_lab_salp_amd.ppo import compute_gae
    g = torch.Generator(device="cuda").manual_seed(0)
    rew = torch.randn(T, n, device="cuda", generator=g)
    val = torch.randn(T, n, device="cuda", generator=g)
    st = (torch.rand(T, n, device="cuda", generator=g) < 0.02).float()
    lv, dn = torch.randn(n, device="cuda", generator=g), torch.zeros(n, device="cuda")
    adv, ret = torch.empty_like(rew), torch.empty_like(rew)
    compute_gae(rew, val, st, lv, dn, advantages=adv, returns=ret)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        compute_gae(rew, val, st, lv, dn, advantages=adv, returns=ret)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    byts = T * n * 20 + n * 8
    gbs = byts / (ms / 1e3) / 1e9
    return {"n_steps": T, "n_envs": n, "ms": ms, "bytes": byts,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-envs", type=int, default=32768)
    ap.add_argument("--n-steps", type=int, default=32)
    ap.add_argument("--batch-size", type=int, default=32768)
    ap.add_argument("--n-epochs", type=int, default=10)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--gae-steps", type=int, default=2048)
    ap.add_argument("--trend-iters", type=int, default=0)
    ap.add_argument("--lockstep-order", type=int, default=-1, help="salp_set_lockstep_order mode")
    ap.add_argument("--collect", default="auto", choices=("auto", "lockstep", "chained"),
                    help="collection: salp_step per env-step, or salp_collect (policy inside the kernel)")
    ap.add_argument("--no-graphs", action="store_true", help="eager minibatch steps (PPO(use_graphs=False))")
    ap.add_argument("--recurrent", action="store_true",
                    help="RecurrentPPO with the MlpLstmPolicy (LSTM 256) of src/train_robot_recurrent_ppo.py")
    ap.add_argument("--lstm-hidden", type=int, default=256)
    ap.add_argument("--seq-len", type=int, default=16)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.shard import env_id_offset, reduce_run
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(a.n_envs, seed=0, env_id_offset=env_id_offset(rank, a.n_envs), infos=False)
    env.sim.set_lockstep_order(a.lockstep_order)
    if a.recurrent:
        from grasp_lab_salp_amd.recurrent_ppo import RecurrentPPO
        model = RecurrentPPO("MlpLstmPolicy", env, n_steps=a.n_steps, batch_size=a.batch_size, n_epochs=a.n_epochs,
                             seed=0, seq_len=a.seq_len, policy_kwargs={"lstm_hidden_size": a.lstm_hidden})
    else:
        model = PPO("MlpPolicy", env, n_steps=a.n_steps, batch_size=a.batch_size, n_epochs=a.n_epochs, seed=0,
                    collect=a.collect, use_graphs=False if a.no_graphs else None)
    # warm-up (+ trend) iterations, one learn() call each so that a long trend
    # reports progress on stderr (a GPU job silent for minutes looks hung)
    for it in range(max(1, a.trend_iters)):
        model.learn((it + 1) * a.n_steps * a.n_envs)
        if rank == 0:
            print(json.dumps(model.history[-1]), file=sys.stderr, flush=True)
    trend = list(model.history)
    for k in model.timing:
        model.timing[k] = 0.0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    model.num_timesteps = 0
    h0 = len(model.history)
    model.learn(a.iters * a.n_steps * a.n_envs)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el, steps, _, _ = reduce_run(el, model.num_timesteps, 0.0, 0.0, device=torch.device("cuda", local))
    if rank == 0:
        res = {"metric": "PPO env-steps/sec (collect + GAE + update), config 5", "value": steps / el,
               "unit": "env-steps/s", "n_gpus": world, "n_envs_per_gpu": a.n_envs, "n_steps": a.n_steps,
               "batch_size": a.batch_size, "n_epochs": a.n_epochs, "iters": a.iters, "collect": model.collect,
               "policy": (f"MlpLstmPolicy (LSTM {a.lstm_hidden}, seq_len {a.seq_len})" if a.recurrent
                          else "MlpPolicy 64-64 tanh"),
               "timing_s": model.timing, "losses": model.logger,
               "history": model.history[h0:], "trend": trend if a.trend_iters else None,
               "diverged_envs_reset": model.nonfinite_resets,
               "gae_kernel": gae_roofline(a.gae_steps, a.n_envs)}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
