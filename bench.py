"""Throughput of the SALP env-step hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2]): 65 536 envs per GPU, canonical robot and
env of src/train_robot.py:11-21, synthetic random actions U(action box) from
on-device Philox, SB3-style auto-reset, rollout-buffer fill (obs, action,
reward, done per env-step).  One bench "step" = one launch of the chained
rollout kernel in which every env runs --tick-budget physics ticks (dt 0.01 s)
and completes as many env-steps (breathing cycles) as fit.  value = env-steps
completed by all ranks / wall time (max over ranks).  Envs shard by global id
with no collective on the data path (weak scaling); the only collectives are
the final counter reductions.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.shard import env_id_offset, reduce_run  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X fp64 vector spec (half the 157.3 TF fp32 rate)
# compulsory bytes per env-step B = 2 * S + outputs, S = the
# persistent per-env state an env-step reads and writes.  Here S = the 102
# fields before the randomisation block (the plain path never touches those).
STATE_BYTES = FIELD["cd"] * 8
STEP_OUT_BYTES = 10 * 4 + 3 * 4 + 4 + 1   # obs + action + reward(f32) + done per env-step
BYTES_PER_ENV_STEP = 2 * STATE_BYTES + STEP_OUT_BYTES


def pmc_profile(n, budget, chunk):
    """The committed PMC summary (tools/pmc_summary.py) measured on this exact
    configuration, if any: HBM traffic and fp64 VALU counts of k_rollout."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))):
        try:
            s = json.load(open(path))
        except (OSError, ValueError):
            continue
        if s.get("config") == {"n_envs": n, "tick_budget": budget, "chunk": chunk}:
            best = (os.path.basename(path), s)
    return best


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--tick-budget", type=int, default=8192, help="physics ticks per env per launch")
    ap.add_argument("--capacity", type=int, default=16, help="rollout-buffer slots per env")
    ap.add_argument("--chunk", type=int, default=128, help="ticks between env-step boundaries")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lockstep", action="store_true")
    return ap.parse_args()


def cpu_baseline(seconds):
    """The C oracle (reference restatement) on the host cores, bounded sample."""
    from oracle.oracle import Oracle
    threads = int(os.environ.get("SALP_CPU_THREADS", min(16, os.cpu_count() or 1)))
    n = 64 * threads
    o = Oracle(default_params(), n, seed=123)
    o.reset()
    steps, ticks, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, tk = o.step_random(1, threads=threads)
        steps += n
        ticks += tk
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs x {steps // n} random-action env-steps ({ticks} ticks, "
                      f"{dt:.1f} s) of the oracle C restatement, OpenMP {threads} threads",
            "ticks_per_sec": ticks / dt}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
    n = a.n_envs
    env = BatchedSalpEnv(n, params=default_params(), seed=a.seed, env_id_offset=env_id_offset(rank, n),
                         device=dev.index)
    cap = a.capacity
    bufs = {"obs": torch.zeros((cap, n, env.obs_dim), dtype=torch.float32, device=dev),
            "actions": torch.zeros((cap, n, 3), dtype=torch.float32, device=dev),
            "rewards": torch.zeros((cap, n), dtype=torch.float32, device=dev),
            "dones": torch.zeros((cap, n), dtype=torch.uint8, device=dev)}
    done = torch.zeros(n, dtype=torch.int64, device=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        env.rollout(a.tick_budget, buffers=bufs, steps_done=done, chunk=a.chunk)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    s0 = int(done.sum())
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for k in range(a.steps):
        starts[k].record()
        env.rollout(a.tick_budget, buffers=bufs, steps_done=done, chunk=a.chunk)
        ends[k].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    torch.cuda.synchronize()
    steps_local = int(done.sum()) - s0
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / a.steps

    # lock-step drop-in path (one env-step per env per launch) for reference
    lock = None
    if not a.no_lockstep:
        env.step_random(1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step_random(4)
        e1.record()
        torch.cuda.synchronize()
        lock = 4 * n / (e0.elapsed_time(e1) / 1e3)

    elapsed, steps_total, kern_ms, lock_total = reduce_run(elapsed, steps_local, kern_ms, lock, device=dev)
    if rank != 0:
        dist.destroy_process_group()
        return

    prof = pmc_profile(n, a.tick_budget, a.chunk)
    ticks_total = float(-(-a.tick_budget // a.chunk) * a.chunk) * n * a.steps * world
    steps_per_launch = steps_local / a.steps
    bytes_launch = steps_per_launch * BYTES_PER_ENV_STEP
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    res = {
        "metric": "env-steps/sec at 65536 parallel envs, 1/2/4/8 MI355X; % HBM roofline",
        "value": steps_total / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: Philox U(action box) actions, Philox targets/obstacles on auto-reset",
        "config": {"workload": "65536 envs/GPU random-action chained rollout + rollout-buffer fill, "
                               "canonical make_env robot (src/train_robot.py:11-21), 2 obstacles",
                   "n_envs_per_gpu": n, "tick_budget": a.tick_budget, "chunk": a.chunk, "rollout_capacity": cap,
                   "parallelism": f"env-shard x{world}"},
        "ticks_per_sec": ticks_total / elapsed,
        "mean_ticks_per_env_step": ticks_total / max(steps_total, 1.0),
        "kernel_ms_per_launch": kern_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": prof[1]["derived"].get("hbm_bytes") if prof else None,
                     "traffic_source": prof[0] if prof else None,
                     "bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": BYTES_PER_ENV_STEP,
                     "note": "algorithmic bytes = env-steps per launch x (2 x 816 B state + 57 B outputs) "
                             "(SURVEY 8(d)); the kernel is fp64-VALU bound (see roofline_valu)"},
        "lockstep_env_steps_per_sec": lock_total,
    }
    f_tick = prof[1]["derived"].get("fp64_flops_per_env_tick") if prof else None
    if f_tick:
        # executed fp64 flops (PMC, FMA = 2) per env-tick of budget x this run's kernel time
        fl = f_tick * float(a.tick_budget) * n / (kern_ms / 1e3) / 1e12
        res["roofline_valu"] = {"bound": "fp64-valu", "achieved": fl, "peak": FP64_VALU_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": fl / FP64_VALU_PEAK_TFLOPS,
                                "flops_per_env_tick": f_tick, "source": prof[0]}
    if world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(a.cpu_baseline_seconds)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
