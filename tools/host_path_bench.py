"""PCIe-inclusive rates of the host-buffer boundaries: the
SB3-shaped SalpVecEnv fed NumPy actions and returning NumPy obs / rewards /
dones / infos (65 536 envs), and the per-env Gym SalpRobotEnv (the reference
make_env's robot, src/train_robot.py:11-21), each timed on the host clock
around whole steps (upload, kernel, download, Python).  One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from grasp_lab_salp_amd.robot import Nozzle, Robot  # noqa: E402
from grasp_lab_salp_amd.salp_robot_env import SalpRobotEnv  # noqa: E402
from grasp_lab_salp_amd.vec_env import SalpVecEnv  # noqa: E402


def _read_done(dones, infos):
    """What SB3's collect_rollouts / Monitor buffer read: the envs that finished."""
    for i in np.nonzero(dones)[0]:
        d = infos[i]
        d["episode"], d["terminal_observation"], d.get("TimeLimit.truncated")


def _scan(dones, infos):
    """src/tensorboard_callback.py:72: `for idx, info in enumerate(infos): if 'episode' in info`."""
    for _idx, info in enumerate(infos):
        if "episode" in info:
            info["episode"]["r"]


def vec_rate(n, steps, infos, consume=None):
    env = SalpVecEnv(n, seed=0, infos=infos)
    env.reset()
    rng = np.random.default_rng(0)
    acts = [np.stack([rng.uniform(0, 1, n), rng.uniform(0, 1, n), rng.uniform(-1, 1, n)], 1).astype(np.float32)
            for _ in range(steps + 2)]
    for a in acts[:2]:
        env.step(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts[2:]:
        _, _, dones, inf = env.step(a)
        if consume is not None:
            consume(dones, inf)
    el = time.perf_counter() - t0
    env.close()
    return n * steps / el


def gym_rate(steps):
    nozzle = Nozzle(length1=0.05, length2=0.05, length3=0.05, area=0.00016, mass=1.0)
    robot = Robot(dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06, nozzle=nozzle)
    robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
    robot.set_environment(density=1000)
    env = SalpRobotEnv(render_mode=None, robot=robot)
    env.reset(seed=0)
    rng = np.random.default_rng(1)
    for _ in range(3):
        env.step(np.array([rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(-1, 1)], dtype=np.float32))
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, term, trunc, _ = env.step(np.array([rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(-1, 1)],
                                                 dtype=np.float32))
        if term or trunc:
            env.reset()
    return steps / (time.perf_counter() - t0)


def main():
    n = int(os.environ.get("N", 65536))
    out = {"n_envs": n,
           "vec_env_infos_off": vec_rate(n, 10, False),
           "vec_env_infos_on": vec_rate(n, 10, True),
           "vec_env_infos_on_sb3_done_reads": vec_rate(n, 10, True, _read_done),
           "vec_env_infos_on_full_scan": vec_rate(n, 4, True, _scan),
           "gym_env_single": gym_rate(200),
           "unit": "env-steps/s",
           "note": "host clock around whole steps: NumPy actions uploaded, salp_step, obs/reward/flags (and info "
                   "dicts of the envs that finished) downloaded; infos are built on access (vec_env.StepInfos): "
                   "_sb3_done_reads reads the finished envs' episode / terminal_observation / TimeLimit entries "
                   "as SB3 does, _full_scan visits every env's dict as src/tensorboard_callback.py:72 does; the "
                   "device-resident rate is bench.py's step_given_actions_env_steps_per_sec"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
