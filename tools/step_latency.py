"""Where the per-env drop-in's step time goes.

One SalpRobotEnv (the reference make_env's robot, src/train_robot.py:11-21)
stepped with uniform random actions; for the same action sequence, on fresh
envs with the same seeds:

* gym: SalpRobotEnv.step on the host clock (upload, launches, download, dicts);
* device: BatchedSalpEnv(1).step with a device-resident action and
  preallocated outputs, host clock around step + synchronize;
* kernel: HIP events around the salp_step call alone (its stream);
* ticks: physics ticks per env-step (the env's `time` field advances by dt).

One JSON line.  STEPS (default 300), SALP_STEP_KERNEL passes through to the
library (latency kernel choice, if any).
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd._abi import FIELD, INFO_DIM  # noqa: E402
from grasp_lab_salp_amd.batched_env import BatchedSalpEnv  # noqa: E402
from grasp_lab_salp_amd.robot import Nozzle, Robot  # noqa: E402
from grasp_lab_salp_amd.salp_robot_env import SalpRobotEnv  # noqa: E402


def _actions(steps, seed=1):
    rng = np.random.default_rng(seed)
    return [np.array([rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(-1, 1)], dtype=np.float32)
            for _ in range(steps)]


def gym(acts):
    nozzle = Nozzle(length1=0.05, length2=0.05, length3=0.05, area=0.00016, mass=1.0)
    robot = Robot(dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06, nozzle=nozzle)
    robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
    robot.set_environment(density=1000)
    env = SalpRobotEnv(render_mode=None, robot=robot)
    np.random.seed(0)
    env.reset(seed=0)
    for a in acts[:3]:
        env.step(a)
    t0 = time.perf_counter()
    for a in acts[3:]:
        _, _, term, trunc, _ = env.step(a)
        if term or trunc:
            env.reset()
    el = time.perf_counter() - t0
    env.close()
    return (len(acts) - 3) / el


def device(acts):
    sim = BatchedSalpEnv(1, seed=0)
    sim.reset()
    dev = torch.from_numpy(np.stack(acts)).cuda()
    od = sim.obs_dim
    out = {"obs": torch.empty((1, od), dtype=torch.float32, device="cuda"),
           "reward": torch.empty(1, dtype=torch.float64, device="cuda"),
           "terminated": torch.empty(1, dtype=torch.uint8, device="cuda"),
           "truncated": torch.empty(1, dtype=torch.uint8, device="cuda"),
           "terminal_obs": torch.empty((1, od), dtype=torch.float32, device="cuda"),
           "info": torch.empty((1, INFO_DIM), dtype=torch.float64, device="cuda")}
    for k in range(3):
        sim.step(dev[k:k + 1], auto_reset=True, out=out)
    torch.cuda.synchronize()
    t_start = float(sim.field("time")[0])
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in acts[3:]]
    t0 = time.perf_counter()
    for k, (e0, e1) in enumerate(ev):
        e0.record()
        sim.step(dev[k + 3:k + 4], auto_reset=True, out=out)
        e1.record()
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern = [e0.elapsed_time(e1) for e0, e1 in ev]
    # ticks: time advances by dt per tick; resets restart it, so count only a
    # reset-free run of the same actions without auto-reset for the estimate
    t_end = float(sim.field("time")[0])
    sim.close()
    return len(ev) / el, float(np.mean(kern)) * 1e3, float(np.median(kern)) * 1e3, t_start, t_end


def chained(kernel, k=64, reps=3):
    """One env, k random-action env-steps per salp_step_random call (the
    chained kernel: k_rollout, or k_rollout_pair with kernel=1): us per env-step
    from HIP events; plus the lock-step k_step_random for one env-step."""
    sim = BatchedSalpEnv(1, seed=0)
    sim.set_rollout_kernel(kernel)
    sim.reset()
    sim.step_random(k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sim.step_random(k)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / k)
    one = []
    for _ in range(2 * k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sim.step_random(1)
        e1.record()
        torch.cuda.synchronize()
        one.append(e0.elapsed_time(e1) * 1e3)
    sim.close()
    return float(np.median(ts)), float(np.mean(one))


def ticks_and_boundary(acts):
    """salp_step's two kernels on the same env and actions, stepped alternately
    (same clocks): ticks per env-step (the env's `time` advances by dt per
    tick; env-steps that end the episode are left out), kernel ns per tick
    (HIP events) and the kernel time of zero-tick env-steps (action [0, 0, 0]:
    the env-step boundary and the launch only)."""
    sims = []
    for mode in (0, 1):
        s = BatchedSalpEnv(1, seed=0)
        s.set_step_kernel(mode)
        s.reset()
        sims.append(s)
    ticks, kern = [], {0: [], 1: []}
    for a in acts:
        at = torch.from_numpy(a[None].copy()).cuda()
        t0 = float(sims[0].field("time")[0])
        done = False
        for m, s in enumerate(sims):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = s.step(at, auto_reset=True)
            e1.record()
            torch.cuda.synchronize()
            kern[m].append(e0.elapsed_time(e1) * 1e3)
            done = done or bool(r.terminated[0] or r.truncated[0])
        t1 = float(sims[0].field("time")[0])
        ticks.append(round((t1 - t0) / 0.01) if (not done and t1 > t0) else -1)
    ticks = np.array(ticks)
    ok = ticks > 0
    out = {"ticks_per_env_step": float(ticks[ok].mean()), "env_steps_counted": int(ok.sum())}
    z = torch.zeros((1, 3), dtype=torch.float32, device="cuda")
    for m, s in enumerate(sims):
        k = np.array(kern[m])
        zero = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.step(z, auto_reset=True)
            e1.record()
            torch.cuda.synchronize()
            zero.append(e0.elapsed_time(e1) * 1e3)
        out[f"step_kernel{m}"] = {"kernel_ns_per_tick": float(1e3 * k[ok].sum() / ticks[ok].sum()),
                                  "kernel_us_per_env_step": float(k[ok].mean()),
                                  "zero_tick_step_us": float(np.median(zero))}
        s.close()
    return out


def main():
    steps = int(os.environ.get("STEPS", 300))
    acts = _actions(steps + 3)
    warm = BatchedSalpEnv(4096, seed=1)   # ~0.5 s of work first: the clocks ramp up
    for _ in range(20):
        warm.step_random(1)
    torch.cuda.synchronize()
    warm.close()
    rate_dev, kern_mean_us, kern_med_us, t0, t1 = device(acts)
    tb = ticks_and_boundary(acts[:150])
    ch0, lock0 = chained(0)
    ch1, _ = chained(1)
    out = {"per_kernel": tb, "chained_k_rollout_us_per_env_step": ch0, "chained_pair_us_per_env_step": ch1,
           "lockstep_step_random1_us": lock0,
           "gym_env_steps_per_s": gym(acts), "device_steps_per_s": rate_dev,
           "kernel_us_mean": kern_mean_us, "kernel_us_median": kern_med_us,
           "sim_time_advanced_s": t1 - t0, "steps": steps,
           "note": "gym = SalpRobotEnv.step host clock; device = BatchedSalpEnv(1).step(out=...) + synchronize; "
                   "kernel = HIP events around salp_step; sim_time_advanced_s / dt / steps ~ ticks per env-step "
                   "when no reset happened"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
