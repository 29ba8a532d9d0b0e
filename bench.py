"""Throughput of the SALP env-step hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` (N > 1) without torchrun's environment starts N ranks itself: it
runs `torch.distributed.run` as a child process before anything touches the
GPU and exits with its status.  Each rank drives one GPU (RCCL process group,
`nccl` backend) and owns the global env ids [rank * n, (rank + 1) * n).  This
replaces the reference's 8 SubprocVecEnv workers (src/train_robot.py:25-26).
`--dry-run` runs the same launcher and reductions on the CPU (gloo, no GPU
kernels): the multi-rank plumbing test of tests/test_bench_launcher.py.

Workload (BASELINE.json configs[2]): 65 536 envs per GPU, canonical robot and
env of src/train_robot.py:11-21, synthetic random actions U(action box) from
on-device Philox, SB3-style auto-reset, rollout-buffer fill (obs, action,
reward, done and the observation the action was taken on, per env-step).  One
bench "step" = one launch of the chained
rollout kernel in which every env runs --tick-budget physics ticks (dt 0.01 s)
and completes as many env-steps (breathing cycles) as fit.  value = env-steps
completed by all ranks / wall time (max over ranks).  Envs shard by global id
with no collective on the data path (weak scaling); the only collectives are
the final counter reductions.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

from grasp_lab_salp_amd._abi import FIELD, default_params  # noqa: E402
from grasp_lab_salp_amd.shard import env_id_offset, reduce_run, reduce_sums  # noqa: E402

METRIC = "env-steps/sec at 65536 parallel envs, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X fp64 vector spec (half the 157.3 TF fp32 rate)
# compulsory bytes per env-step B = 2 * S + outputs, S = the
# persistent per-env state an env-step reads and writes.  Here S = the 102
# fields before the randomisation block (the plain path never touches those).
STATE_BYTES = FIELD["cd"] * 8
# per env-step into the rollout buffer: obs before and after the step, action,
# reward (f32) and done
STEP_OUT_BYTES = 2 * 10 * 4 + 3 * 4 + 4 + 1
BYTES_PER_ENV_STEP = 2 * STATE_BYTES + STEP_OUT_BYTES
# Algorithmic fp64 work of one physics tick ("F_TICK"): the
# reference's operations (src/robot.py:789-875, src/dynamics.py, src/geometry.py)
# with structural zeros removed; +,-,*,/,sqrt,sin,cos each one flop-equivalent.
# Newton 101 + Euler 98 + integration 90 + clock/phase 5 + geometry 93 (a tick
# outside JET; a JET tick adds 11).
F_TICK_ALGO = 387
# Mean ticks per env-step under the synthetic action distribution: the oracle
# over 3 seeds x 4096 envs x 20 env-steps (245 760 env-steps) gives 710.4.
# Only the fallback: a run with its parity check measures the mean of its own
# replayed env-steps (parity_sampled.ticks_per_env_step) and uses that.
MEAN_TICKS_PER_ENV_STEP = 710.4
HOT_FIELDS = slice(FIELD["v0"], FIELD["ang2"] + 1)   # kinematic state: NaN once an env diverged


STEADY_WARM, STEADY_TIMED = 40, 20


def summary_order(path):
    """Profile tags r<round><letters> in the order they were made: r3h < r3z <
    r3aa < r3at (round, then length, then name); the last matching summary wins."""
    tag = os.path.basename(path).split("_")[0]
    rnd = int("".join(ch for ch in tag[1:] if ch.isdigit()) or 0)
    return (rnd, len(tag), tag)


def pmc_profile(n, budget, chunk):
    """The committed PMC summary (tools/pmc_summary.py) measured on this exact
    configuration AND on this exact k_rollout machine code, if any: HBM
    traffic and fp64 VALU counts.  Returns (name, summary, None) or (None, None,
    reason): a summary whose kernel fingerprint differs from the library's is
    stale and is not reported as measured."""
    import glob
    from grasp_lab_salp_amd import _codeobj
    from grasp_lab_salp_amd._lib import LIB_PATH
    sha = _codeobj.kernel_sha(LIB_PATH, _codeobj.ROLLOUT_KERNEL)
    best = None
    stale = []
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")), key=summary_order):
        try:
            s = json.load(open(path))
        except (OSError, ValueError):
            continue
        # the latest summary of this configuration that holds the traffic passes
        # (FETCH_SIZE / WRITE_SIZE) and the fp64 instruction mix
        d = s.get("derived", {})
        if (s.get("config") == {"n_envs": n, "tick_budget": budget, "chunk": chunk}
                and d.get("hbm_bytes") and d.get("fp64_flops")):
            if s.get("kernel_sha16") == sha:
                best = (os.path.basename(path), s, None)
            else:
                stale.append(os.path.basename(path))
    if best is None:
        why = (f"no PMC summary of this config was measured on this k_rollout build (kernel_sha16 {sha}); "
               f"stale summaries: {stale[-3:]}" if stale else "no PMC summary of this config")
        return None, None, why
    return best


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one GPU each); >1 self-launches torchrun")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--tick-budget", type=int, default=8192, help="physics ticks per env per launch")
    ap.add_argument("--capacity", type=int, default=16, help="rollout-buffer slots per env")
    ap.add_argument("--chunk", type=int, default=64,
                    help="ticks between env-step boundaries (64 with q = 560: profiles/r5_experiments.md r5j-r5k)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lockstep", action="store_true")
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the sampled oracle replay after the timed region")
    ap.add_argument("--no-ppo", action="store_true", help="skip the config-5 PPO leg")
    ap.add_argument("--ppo-envs", type=int, default=32768, help="PPO leg: envs per GPU (BASELINE configs[4])")
    ap.add_argument("--ppo-steps", type=int, default=256, help="PPO leg: n_steps per collection")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + reductions only, gloo on the CPU, no GPU kernels")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a, argv):
    """Start `a.gpus` ranks of this script under torch.distributed.run (a child
    process; this process never touches the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count()
    return {"model": model, "logical_cpus": os.cpu_count(), "cpus_allowed": allowed}


def cpu_threads():
    """Host cores this job may use: the scheduler's share (OMP_NUM_THREADS, set
    to the box's per-GPU CPU share on the GPU pool) or, without it, every CPU
    in this process's affinity mask."""
    env = os.environ.get("SALP_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    if env:
        return max(1, int(env))
    return cpu_info()["cpus_allowed"] or 1


def cpu_baseline(seconds):
    """The C oracle (the reference's algorithm restated, oracle/salp_oracle.c)
    on the host cores, bounded samples, seeds 0/1/2:
      * config 1 (BASELINE.json configs[0]): 1 env x 1000 random-action
        env-steps on one core, the robot of src/test_robot.py:6-9 (== make_env);
      * throughput: 64 envs per thread, OpenMP over every core this job has,
        `seconds` split over the three seeds."""
    from oracle.oracle import Oracle
    threads = cpu_threads()
    p = default_params()
    # untimed warm-up: the first OpenMP region pays the thread-pool start (~1 s)
    w = Oracle(p, 64 * threads, seed=99)
    w.reset()
    w.step_random(1, threads=threads)
    n = 64 * threads
    per_seed = []
    for seed in (0, 1, 2):
        o = Oracle(p, n, seed=seed)
        o.reset()
        w.step_random(1, threads=threads)   # untimed, keeps the thread pool hot
        steps, ticks, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 3:
            _, tk = o.step_random(1, threads=threads)
            steps += n
            ticks += tk
        dt = time.perf_counter() - t0
        per_seed.append({"seed": seed, "env_steps": steps, "ticks": ticks, "seconds": dt,
                         "env_steps_per_sec": steps / dt})
    cfg1 = []
    for seed in (0, 1, 2):
        o = Oracle(p, 1, seed=seed)
        o.reset()
        t0 = time.perf_counter()
        _, tk = o.step_random(1000, threads=1)
        dt = time.perf_counter() - t0
        cfg1.append({"seed": seed, "seconds": dt, "env_steps_per_sec": 1000 / dt, "ticks": tk})
    steps = sum(s["env_steps"] for s in per_seed)
    secs = sum(s["seconds"] for s in per_seed)
    ticks = sum(s["ticks"] for s in per_seed)
    value = steps / secs
    return {"value": value, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "per_core": value / threads, "ticks_per_sec": ticks / secs, "cpu": cpu_info(),
            "sample": f"oracle C restatement, OpenMP {threads} threads, {n} envs x random-action env-steps, "
                      f"seeds 0/1/2 ({secs:.1f} s); config 1 = 1 env x 1000 env-steps on one core",
            "per_seed": per_seed,
            "config1": {"env_steps": 1000, "per_seed": cfg1,
                        "env_steps_per_sec": 3000 / sum(c["seconds"] for c in cfg1)},
            "note": "cores = the CPU share the GPU pool grants a one-GPU job (OMP_NUM_THREADS); "
                    "the interpreted Python reference itself does ~2.1 env-steps/s per core (SURVEY.md §6)"}


def ppo_leg(a, rank, world, dev):
    """BASELINE.json configs[4]: PPO on 32 768 envs per GPU with the HIP GAE
    scan (the learner of src/train_robot_recurrent_ppo.py:85-107 with its
    gamma / lambda / clip / epochs, MlpPolicy, SB3 semantics restated in
    grasp_lab_salp_amd/ppo.py).  One untimed iteration (warm-up: graph
    capture, allocator), then one timed iteration of collection (salp_collect
    at n_steps >= 256: the policy inside the chained kernel), GAE and 10
    epochs of minibatch updates (batch 32 768; one RCCL all-reduce of the
    gradients per minibatch when world > 1).  value = env-steps of the timed
    iteration over all ranks / its wall time (max over ranks); the split comes
    from HIP events on the stream.  k_gae alone is timed against the HBM
    roofline (12 B read + 8 B written per (step, env))."""
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    from tools.bench_ppo import gae_roofline
    n, T = a.ppo_envs, a.ppo_steps
    env = SalpVecEnv(n, seed=a.seed, env_id_offset=env_id_offset(rank, n), device=dev.index, infos=False)
    # SALP_BENCH_PPO_GRAPHS=0: eager update (tools/gpu_pmc_collect.sh: rocprofv3's counter collection does
    # not survive the update's HIP graphs; eager and graphed updates are equal bit for bit, so the
    # collection profiled is the same)
    graphs = os.environ.get("SALP_BENCH_PPO_GRAPHS", "1") != "0"
    model = PPO("MlpPolicy", env, n_steps=T, batch_size=32768, n_epochs=10, seed=a.seed, collect="auto",
                use_graphs=graphs)
    model.learn(T * n)   # warm-up iteration
    for k in model.timing:
        model.timing[k] = 0.0
    torch.cuda.synchronize()
    # the timed collection's starting point, for the sampled replay after it
    check = rank == 0 and not a.no_parity_check and model.collect == "chained"
    if check:
        state0 = model.sim.get_state().cpu().numpy()
        obs0 = model._obs.detach().cpu().numpy()
    if world > 1:
        dist.barrier()
    model.num_timesteps = 0
    t0 = time.perf_counter()
    model.learn(T * n)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el_max, steps, _, _ = reduce_run(el, model.num_timesteps, 0.0, 0.0, device=dev)
    collect_parity = None
    if check:
        # Parity of the timed collection (the checker, after the timed region):
        # blocks of env ids replayed on the C oracle from their state before the
        # call with the clipped actions the kernel recorded (oracle/sampled.py)
        from grasp_lab_salp_amd.ppo import DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS
        from oracle import sampled
        t_chk = time.perf_counter()
        b = model.buf
        collect_parity = sampled.check_collect(
            state0, obs0, {k: getattr(b, k).detach().cpu().numpy() for k in ("obs", "actions", "rewards",
                                                                             "episode_starts")},
            model._last_obs.detach().cpu().numpy(), model.sim.get_state().cpu().numpy(), default_params(), a.seed,
            env_offset=env_id_offset(rank, n),
            guard=(DIVERGED_OBS_ABS, DIVERGED_REWARD_ABS) if model.reset_nonfinite else None)
        collect_parity["seconds"] = time.perf_counter() - t_chk
        collect_parity["what"] = ("the timed salp_collect: blocks of 64 env ids (first, last, one random) replayed "
                                  "on the C oracle with the recorded clipped actions and the divergence guard; "
                                  "observations, rewards (no-bootstrap rows), episode starts, final obs and state "
                                  "bit for bit")
    gae = gae_roofline(T, n)
    timing = {k: reduce_run(v, 0, 0.0, 0.0, device=dev)[0] for k, v in model.timing.items()}
    env.close()
    del model, env
    torch.cuda.empty_cache()
    out = {"metric": "PPO env-steps/sec (collection + GAE + update), BASELINE configs[4]", "value": steps / el_max,
            "unit": "env-steps/s", "n_envs_per_gpu": n, "n_steps": T, "batch_size": 32768, "n_epochs": 10,
            "collect": "chained (salp_collect)" if T >= 256 else "lockstep (salp_step)",
            "iteration_s": el_max, "timing_s_max_over_ranks": timing,
            "gae_kernel": gae, "policy": "SB3 MlpPolicy 64-64 tanh (the reference's LSTM-256 RecurrentPPO: "
                                         "grasp_lab_salp_amd.recurrent_ppo, tools/bench_ppo.py --recurrent)"}
    if collect_parity is not None:
        out["collect_parity_sampled"] = collect_parity
    out["collect_roofline_valu"] = collect_roofline(n, T, timing.get("collect_s"), collect_parity)
    return out


def collect_roofline(n, T, collect_s, parity):
    """fp64 VALU roofline of the timed collection (the two-wave kernel of the
    auto choice at config 5's 32 768 envs, k_rollout_split<true> from round 6): algorithmic flops
    (F_TICK_ALGO per physics tick, the ticks measured by the collection's
    sampled replay) and, from a committed PMC summary of this config whose
    kernel fingerprint matches the library's, executed flops; both over the
    timed collection phase (HIP events: the kernel plus the bootstrap value
    GEMM)."""
    import glob
    from grasp_lab_salp_amd import _codeobj
    from grasp_lab_salp_amd._lib import LIB_PATH
    if not collect_s:
        return None
    tps = parity["ticks_per_env_step"] if parity else None
    symbol, kname = _codeobj.collect_kernel()
    res = {"bound": "fp64-valu", "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "kernel": kname,
           "collect_s": collect_s, "ticks_per_env_step": tps}
    if tps:
        fl = F_TICK_ALGO * n * T * tps / collect_s / 1e12
        res.update({"achieved": fl, "frac": fl / FP64_VALU_PEAK_TFLOPS, "count": "algorithmic (F_TICK_ALGO x "
                    "measured ticks of the replayed env-steps)"})
    sha = _codeobj.kernel_sha(LIB_PATH, symbol)
    res["kernel_sha16"] = sha
    best, stale = None, []
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_collect_summary.json")), key=summary_order):
        try:
            s = json.load(open(path))
        except (OSError, ValueError):
            continue
        if s.get("config") == {"n_envs": n, "n_steps": T} and s.get("derived", {}).get("fp64_flops_per_executed_tick"):
            if s.get("kernel_sha16") == sha:
                best = (os.path.basename(path), s)
            else:
                stale.append(os.path.basename(path))
    if best is None:
        res["executed"] = None
        res["executed_reason"] = (f"no PMC summary of this collection measured on this build (kernel_sha16 {sha}); "
                                  f"stale: {stale[-2:]}" if stale else "no PMC summary of this collection")
    elif tps:
        # the probe's executed fp64 flops per physics tick (its own collection, replayed for its
        # ticks) times this collection's ticks
        d = best[1]["derived"]
        ex = d["fp64_flops_per_executed_tick"] * n * T * tps / collect_s / 1e12
        res["executed"] = {"achieved": ex, "frac": ex / FP64_VALU_PEAK_TFLOPS, "source": best[0],
                           "fp64_flops_per_executed_tick": d["fp64_flops_per_executed_tick"],
                           "hbm_bytes_per_dispatch": d.get("hbm_bytes"), "active_valu_frac": d.get("active_valu_frac"),
                           "note": "PMC of tools/collect_pmc_probe.py (the same kernel, size and chunk, a fresh "
                                   "policy): fp64 VALU instructions x 64 lanes (FMA = 2) per executed tick, times "
                                   "the timed collection's measured ticks, over its collect phase"}
    else:
        res["executed"] = None
        res["executed_reason"] = "no measured ticks (the collection's sampled replay did not run)"
    return res


def per_env_gym_rate(dev, steps=200):
    """SalpRobotEnv.step, one env, on the host clock (NumPy action in, NumPy
    obs / reward / flags / info out): the per-env drop-in path of
    INTEGRATION.md section 1."""
    import numpy as np
    from grasp_lab_salp_amd.robot import Nozzle, Robot
    from grasp_lab_salp_amd.salp_robot_env import SalpRobotEnv
    nozzle = Nozzle(length1=0.05, length2=0.05, length3=0.05, area=0.00016, mass=1.0)
    robot = Robot(dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06, nozzle=nozzle)
    robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
    robot.set_environment(density=1000)
    genv = SalpRobotEnv(render_mode=None, robot=robot, device=dev.index if dev.index is not None else 0)
    rng = np.random.default_rng(1)
    acts = np.stack([rng.uniform(0, 1, steps + 3), rng.uniform(0, 1, steps + 3),
                     rng.uniform(-1, 1, steps + 3)], 1).astype(np.float32)
    for k in range(3):
        genv.step(acts[k])
    t0 = time.perf_counter()
    for k in range(3, steps + 3):
        _, _, term, trunc, _ = genv.step(acts[k])
        if term or trunc:
            genv.reset()
    rate = steps / (time.perf_counter() - t0)
    genv.close()
    return rate


def dry_run(a, world, rank):
    """Launcher plumbing without a GPU: same rank layout, offsets and
    reductions as the real run, over gloo."""
    n = a.n_envs
    off = env_id_offset(rank, n)
    offs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(offs, torch.tensor([off], dtype=torch.int64))
    else:
        offs = [torch.tensor([off])]
    elapsed, steps_total, _, _ = reduce_run(1.0 + rank, float(n), 0.0, None)
    seen = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "value": None, "unit": "env-steps/s",
                          "n_gpus": world, "world_size": seen, "steps": a.steps, "warmup": a.warmup,
                          "env_id_offsets": [int(o) for o in offs], "max_elapsed": elapsed,
                          "env_steps_sum": steps_total, "backend": "gloo" if world > 1 else None}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks")
    if a.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        dry_run(a, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    if world > 1:
        # SALP_BENCH_REHEARSAL=1: the multi-rank code path on fewer GPUs than
        # ranks (ranks share devices, gloo carries the reductions and the PPO
        # gradient all-reduce): for checking the N-rank run on a one-GPU box;
        # its timings mean nothing
        rehearsal = os.environ.get("SALP_BENCH_REHEARSAL") == "1"
        torch.cuda.set_device(local % torch.cuda.device_count() if rehearsal else local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != world:
            raise SystemExit("process group size differs from WORLD_SIZE")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from grasp_lab_salp_amd.batched_env import BatchedSalpEnv
    n = a.n_envs
    env = BatchedSalpEnv(n, params=default_params(), seed=a.seed, env_id_offset=env_id_offset(rank, n),
                         device=dev.index)
    cap = a.capacity
    bufs = {"obs": torch.zeros((cap, n, env.obs_dim), dtype=torch.float32, device=dev),
            "obs_before": torch.zeros((cap, n, env.obs_dim), dtype=torch.float32, device=dev),
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
    done0 = done.clone()
    finite0 = torch.isfinite(env.get_state()[HOT_FIELDS]).all(0)
    # HIP events on the stream the kernel is launched on (torch's current stream)
    stream = torch.cuda.current_stream(dev)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for k in range(a.steps):
        starts[k].record(stream)
        env.rollout(a.tick_budget, buffers=bufs, steps_done=done, chunk=a.chunk)
        ends[k].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    torch.cuda.synchronize()
    steps_local = int(done.sum()) - s0
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / a.steps

    # SURVEY.md §5 failure detection: envs whose explicit integration diverged
    # (the reference's own blow-up, test_reference_blowup_is_reproduced) at
    # the end of the run, and the non-finite observations among the last
    # `cap` env-steps of every env held in the rollout buffer.
    st = env.get_state()
    finite1 = torch.isfinite(st[HOT_FIELDS]).all(0)
    diverged = int((~finite1).sum())
    bad_rows = int((~torch.isfinite(bufs["obs"]).all(-1)).sum())
    # env-steps of the envs whose kinematic state was finite at both ends of
    # the timed region (an env that diverges stays NaN until its 500-cycle
    # timeout, longer than the timed region)
    finite_steps = int(((done - done0) * (finite0 & finite1)).sum())

    # Parity at the bench's own horizon (the checker, after the timed region):
    # sampled env ids replayed from creation on the C oracle for exactly the
    # env-steps each completed plus its in-flight cycle; state and the last
    # `cap` buffer rows compared bit for bit (oracle/sampled.py).
    parity = None
    if rank == 0 and not a.no_parity_check:
        from oracle import sampled
        t_chk = time.perf_counter()
        parity = sampled.check(st.cpu().numpy(), done.cpu().numpy(), {k: v.cpu().numpy() for k, v in bufs.items()},
                               default_params(), a.seed, env_offset=env_id_offset(rank, n), threads=cpu_threads(),
                               n_random=128)
        parity["seconds"] = time.perf_counter() - t_chk
        parity["what"] = ("rank 0's sampled envs (first and last workgroup, diverged envs, random ids) replayed "
                          "from creation on the C oracle; state + last buffer rows bit for bit")

    # the drop-in step paths beside the headline:
    # * lock-step: salp_step_random(1) x 4, one env-step per env per launch on
    #   k_step_random (a launch lasts as long as the longest cycle of the batch);
    # * policy-shaped: salp_step with caller-given actions and obs/reward/flag
    #   outputs, one env-step per launch, as SalpRobotEnv.step / a learner;
    # * chained k-step: salp_step_random(32), every env runs its 32 env-steps back
    #   to back on k_rollout (max_steps) and stops (from 32 env-steps per call on).
    lock = given = chained32 = gym_rate = None
    if not a.no_lockstep:
        env.step_random(1)
        torch.cuda.synchronize()

        def timed(fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 1e3

        lock = 4 * n / timed(lambda: [env.step_random(1) for _ in range(4)])
        gen = torch.Generator(device=dev).manual_seed(a.seed + 1)
        acts = [torch.rand((n, 3), device=dev, generator=gen) * torch.tensor([1.0, 1.0, 2.0], device=dev)
                - torch.tensor([0.0, 0.0, 1.0], device=dev) for _ in range(4)]
        given = 4 * n / timed(lambda: [env.step(x, auto_reset=True) for x in acts])
        chained32 = 32 * n / timed(lambda: env.step_random(32))
        if rank == 0 and world == 1:
            gym_rate = per_env_gym_rate(dev)

    # The same workload past its start-up transient: envs created and reset
    # together start their cycles in step and with roll / pitch near zero; over
    # the first ~25 launches the phases spread and the population's roll /
    # pitch spread too (tumbling envs), which costs every wave with such a lane
    # the full sin / cos path.  A fresh handle of the same
    # size runs STEADY_WARM untimed launches, then STEADY_TIMED timed ones.
    steady = None
    if not a.no_lockstep and world == 1:
        senv = BatchedSalpEnv(n, params=default_params(), seed=a.seed + 7, device=dev.index)
        sdone = torch.zeros(n, dtype=torch.int64, device=dev)
        for _ in range(STEADY_WARM):
            senv.rollout(a.tick_budget, buffers=bufs, steps_done=sdone, chunk=a.chunk)
        torch.cuda.synchronize()
        s_0 = int(sdone.sum())
        ts0 = time.perf_counter()
        for _ in range(STEADY_TIMED):
            senv.rollout(a.tick_budget, buffers=bufs, steps_done=sdone, chunk=a.chunk)
        torch.cuda.synchronize()
        steady = (int(sdone.sum()) - s_0) / (time.perf_counter() - ts0)
        senv.close()
        del senv

    ppo = None
    if not a.no_ppo:
        del bufs
        torch.cuda.empty_cache()
        ppo = ppo_leg(a, rank, world, dev)

    elapsed, steps_total, kern_ms, lock_total = reduce_run(elapsed, steps_local, kern_ms, lock, device=dev)
    given_total = reduce_sums([given or 0.0], device=dev)[0] if given is not None else None
    chained32_total = reduce_sums([chained32 or 0.0], device=dev)[0] if chained32 is not None else None
    diverged_total, bad_rows_total, finite_total = reduce_sums([diverged, bad_rows, finite_steps], device=dev)
    seen_world = dist.get_world_size() if world > 1 else 1
    if rank != 0:
        dist.destroy_process_group()
        return

    prof = pmc_profile(n, a.tick_budget, a.chunk)
    from grasp_lab_salp_amd import _codeobj
    from grasp_lab_salp_amd._lib import LIB_PATH
    kernel_sha = _codeobj.kernel_sha(LIB_PATH, _codeobj.ROLLOUT_KERNEL)
    budget_ticks = float(-(-a.tick_budget // a.chunk) * a.chunk) * n * a.steps * world
    steps_per_launch = steps_local / a.steps
    bytes_launch = steps_per_launch * BYTES_PER_ENV_STEP
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    # ticks per env-step: measured on this run's own replayed env-steps when the
    # parity check ran (rank 0's sample), else the oracle's 710.4
    if parity is not None and parity.get("env_steps_replayed"):
        tps, tps_src = parity["ticks_per_env_step"], (
            f"measured: parity_sampled replayed {parity['env_steps_replayed']} completed env-steps of this run "
            f"({parity['ticks_replayed']} ticks) on the oracle")
    else:
        tps, tps_src = MEAN_TICKS_PER_ENV_STEP, "constant: the oracle's mean over 245 760 random-action env-steps"
    env_ticks_per_launch = steps_per_launch * tps
    res = {
        "metric": METRIC,
        "value": steps_total / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "world_size": seen_world,
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
        "finite_env_steps_per_sec": finite_total / elapsed,
        "finite_note": "env-steps of envs whose kinematic state was finite at the start and at the end of the timed "
                       "region (diverged envs carry NaN, as the reference's integrator does, and count in value)",
        "ticks_per_env_step": tps,
        "ticks_per_env_step_source": tps_src,
        "ticks_per_sec": steps_total * tps / elapsed,
        "ticks_note": "ticks_per_sec = value x ticks_per_env_step: physics ticks (dt 0.01 s) of the completed "
                      "env-steps per second",
        "budget_full_tick_equivalents_per_sec": budget_ticks / elapsed,
        "budget_note": "tick_budget counts full-tick equivalents: per chunk a wave runs k full ticks, then "
                       "(chunk - k) x q / 256 steady ticks (q = 560: a settled tick costs ~0.39 of a full one), so "
                       "a lane's executed ticks per launch exceed tick_budget by up to q / 256 = 2.19x; "
                       "ticks_per_sec above this rate is expected, not a contradiction",
        "kernel_ms_per_launch": kern_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": prof[1]["derived"].get("hbm_bytes") if prof[1] else None,
                     "traffic_source": prof[0] if prof[1] else prof[2],
                     "kernel_sha16": kernel_sha,
                     "bytes_per_launch": bytes_launch,
                     "bytes_per_env_step": BYTES_PER_ENV_STEP,
                     "note": "algorithmic bytes = env-steps per launch x (2 x 816 B state + 97 B outputs) "
                             "(SURVEY 8(d)); the kernel is fp64-VALU bound (see roofline_valu)"},
        "lockstep_env_steps_per_sec": lock_total,
        "step_given_actions_env_steps_per_sec": given_total,
        "step_random32_chained_env_steps_per_sec": chained32_total,
        "per_env_gym_step_env_steps_per_sec": gym_rate,
        "steady_state_env_steps_per_sec": steady,
        "steady_state_note": f"the same workload on a fresh handle after {STEADY_WARM} untimed launches, "
                             f"{STEADY_TIMED} timed (rank 0 of a 1-GPU run): past the start-up transient that value's "
                             "launches (after `warmup`) still partly cover (DESIGN.md section 5)",
        "step_paths_note": "lockstep: salp_step_random(1) x4 (k_step_random); given actions: salp_step x4 "
                           "with obs/reward/flags out (the SalpRobotEnv.step path); chained: salp_step_random(32) "
                           "on k_rollout with max_steps (each env 32 env-steps back to back); per-env gym: the unchanged "
                           "drop-in SalpRobotEnv.step (one env, src/train_robot.py:11-21's robot) on the host clock, "
                           "200 env-steps of U(action box) actions, rank 0 of a 1-GPU run (k_step_wave)",
        "divergence": {"diverged_envs_at_end": diverged_total, "envs": n * world,
                       "nonfinite_obs_rows_in_buffer": bad_rows_total, "buffer_rows": cap * n * world,
                       "note": "the reference integrator itself diverges for some actions (jet_time < dt); "
                               "such envs carry NaN until the 500-cycle timeout resets them"},
    }
    # fp64 VALU roofline: algorithmic flops (F_TICK_ALGO per executed env-tick)
    # and, where a PMC summary of this configuration exists, executed flops
    fl_algo = F_TICK_ALGO * env_ticks_per_launch / (kern_ms / 1e3) / 1e12
    res["roofline_valu"] = {"bound": "fp64-valu", "achieved": fl_algo, "peak": FP64_VALU_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": fl_algo / FP64_VALU_PEAK_TFLOPS,
                            "flops_per_env_tick": F_TICK_ALGO, "ticks_per_env_step": tps,
                            "env_ticks_per_launch": env_ticks_per_launch,
                            "count": "algorithmic (DESIGN.md §5) x env-ticks per launch (env-steps per launch x "
                                     "ticks_per_env_step)"}
    if prof[1]:
        d = prof[1]["derived"]
        per = prof[1]["per_dispatch"]
        if d.get("fp64_flops"):
            fl = d["fp64_flops"] / (kern_ms / 1e3) / 1e12
            mix = {k.replace("SQ_INSTS_VALU_", "").lower(): per[k]["mean"] / max(d["fp64_valu_insts"], 1.0)
                   for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                             "SQ_INSTS_VALU_TRANS_F64") if k in per}
            res["roofline_valu"]["executed"] = {
                "achieved": fl, "frac": fl / FP64_VALU_PEAK_TFLOPS,
                "flops_per_budget_tick": d.get("fp64_flops_per_env_tick"),
                "flops_per_env_tick": d["fp64_flops"] / env_ticks_per_launch, "instruction_mix": mix,
                "active_valu_frac": d.get("active_valu_frac"), "waves": per.get("SQ_WAVES", {}).get("mean"),
                "source": prof[0],
                "note": "PMC fp64 VALU instructions x 64 lanes (FMA = 2): both arms of branch-free selects, "
                        "Newton steps of divisions and polynomial transcendentals included"}
    if parity is not None:
        res["parity_sampled"] = parity
    if ppo is not None:
        res["ppo"] = ppo
    if not a.no_cpu_baseline:
        # rank 0, after every rank's timed region (the other ranks have left):
        # the same bounded oracle sample at every N, on rank 0's CPU share
        res["cpu_baseline"] = cpu_baseline(a.cpu_baseline_seconds)
        if world > 1:
            res["cpu_baseline"]["note"] += (f"; measured on rank 0 after the {world}-rank timed region, "
                                            f"with rank 0's CPU share ({res['cpu_baseline']['cores']} threads)")
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
