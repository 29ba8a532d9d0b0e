"""Generate golden fixtures by running the *reference* Python implementation.

Runs ONLY in the build container (it reads /root/reference, which never
travels to the GPU box).  The reference imports `numba`, `gymnasium` and
`pygame`, none of which is installed here; following SURVEY.md §8(c) this
script writes minimal offline stand-ins into a temporary directory:

* ``numba.jit``      -> identity decorator (the jitted bodies run as NumPy),
* ``gymnasium.Env``  -> a class whose ``reset(seed)`` does nothing,
* ``gymnasium.spaces.Box`` -> a holder of ``low/high/shape/dtype``,
* ``pygame``         -> an empty module (rendering is never reached).

No reference source is copied: the stand-ins only let
``/root/reference/src/{robot,salp_robot_env}.py`` import.  What is stored is
data: inputs (actions, targets, obstacles, full pre-step state snapshots) and
the reference's outputs (post-step state, obs, reward, flags, info metrics).

Fixture files (all ``np.savez_compressed``):

``episodes.npz``   env-level rollouts (src/salp_robot_env.py:114-299), one row
                   per ``env.step``: snapshot before, action, snapshot after,
                   obs / reward / terminated / truncated / reward components
                   and the episode metrics dict on done.  Auto-reset after
                   done (SB3 VecEnv semantics) with the reference's own
                   target/obstacle draws recorded in the post-reset snapshot.
``tick_trace.npz`` robot-level per-tick histories (``record=True``,
                   src/robot.py:740-777) for a few cycles.
``robot_trace.npz`` the bare-robot call sequence of src/compare_trajectories.py:
                   142-150 / src/robot.py:1149-1155 with Python-float controls
                   (float64 geometry throughout), per-tick histories and the
                   robot state after every cycle, for the canonical robot and
                   the demo robot of src/robot.py:1104-1107.

Usage:  python tests/golden/make_golden.py  [--jobs 8] [--only robot]
"""
import argparse
import multiprocessing as mp
import os
import sys
import tempfile
import textwrap

import numpy as np

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

# Canonical config: src/train_robot.py:11-21 (make_env).
CANON = dict(length1=0.05, length2=0.05, length3=0.05, area=0.00016, nozzle_mass=1.0,
             dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06,
             density=1000)

# Fixed action sequence of src/salp_robot_env.py:1568-1579 (already in the
# action box); used as float32 like SB3 would pass it.
FIXED_ACTIONS = np.array([
    [0.695722, 0.01922786, -0.06692487],
    [0.2808507, 0.8017318, 0.87773895],
    [0.57452214, 0.11145315, -0.82465506],
    [0.32618135, 0.11088043, 0.88842094],
    [0.17267734, 0.6958977, -0.9337022],
    [0.49285844, 0.2883283, 0.81122017],
    [0.34796143, 0.35572827, -0.8472595],
    [0.49369425, 0.27951986, 0.8069289],
    [0.37975544, 0.338947, -0.8655774],
    [0.4979022, 0.23918751, 0.7962456],
], dtype=np.float32)

MAX_OBS = 4  # obstacle slots in the fixture arrays


def _write_stubs(d):
    os.makedirs(os.path.join(d, "gymnasium"), exist_ok=True)
    with open(os.path.join(d, "numba.py"), "w") as f:
        f.write(textwrap.dedent("""
            def jit(*a, **k):
                if a and callable(a[0]) and not k:
                    return a[0]
                return lambda f: f
            njit = jit
        """))
    with open(os.path.join(d, "gymnasium", "__init__.py"), "w") as f:
        f.write(textwrap.dedent("""
            from . import spaces
            class Env:
                def reset(self, seed=None, options=None):
                    return None
        """))
    with open(os.path.join(d, "gymnasium", "spaces.py"), "w") as f:
        f.write(textwrap.dedent("""
            import numpy as np
            class Box:
                def __init__(self, low, high, dtype=np.float32, shape=None):
                    self.low = np.asarray(low, dtype=dtype)
                    self.high = np.asarray(high, dtype=dtype)
                    self.dtype = dtype
                    self.shape = self.low.shape
        """))
    with open(os.path.join(d, "pygame.py"), "w") as f:
        f.write("")


def _import_reference():
    d = tempfile.mkdtemp(prefix="salp_refstub_")
    _write_stubs(d)
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, d)
    import robot  # noqa: F401
    import salp_robot_env  # noqa: F401
    return robot, salp_robot_env


def make_env(ref_robot, ref_env, init_angles=(0.0, 0.0), num_obstacles=2):
    c = CANON
    nozzle = ref_robot.Nozzle(length1=c["length1"], length2=c["length2"], length3=c["length3"],
                              area=c["area"], mass=c["nozzle_mass"])
    robot = ref_robot.Robot(dry_mass=c["dry_mass"], init_length=c["init_length"],
                            init_width=c["init_width"], max_contraction=c["max_contraction"],
                            nozzle=nozzle)
    robot.nozzle.set_angles(angle1=init_angles[0], angle2=init_angles[1])
    robot.set_environment(density=c["density"])
    return ref_env.SalpRobotEnv(render_mode=None, robot=robot, num_obstacles=num_obstacles)


# --------------------------------------------------------------------------
# Snapshot of every attribute the hot path reads or writes
# --------------------------------------------------------------------------
VEC3 = ["velocity", "angular_velocity", "acceleration", "angular_acceleration", "euler_angle",
        "position_world", "position", "angle", "prev_position", "prev_angle", "velocity_world",
        "avg_cycle_velocity", "avg_cycle_angular_velocity", "center_of_mass",
        "prev_center_of_mass", "center_of_mass_rate", "prev_center_of_mass_rate",
        "center_of_mass_acc_rate", "area", "trans_drag_coefficient", "rot_drag_coefficient"]
SCAL = ["length", "width", "volume", "prev_water_volume", "water_mass", "prev_water_mass",
        "cycle_time", "time", "refill_time", "jet_time", "coast_time", "contraction",
        "_contract_rate", "_release_rate"]
NOZ = ["angle1", "angle2", "prev_angle1", "prev_angle2", "yaw", "prev_yaw", "turn_time"]


def snapshot(env):
    r = env.robot
    s = {}
    for k in VEC3:
        s["r_" + k] = np.array(getattr(r, k), dtype=np.float64, copy=True).reshape(3)
    for k in SCAL:
        s["r_" + k] = np.float64(getattr(r, k))
    s["r_mass"] = np.float64(r.mass[0, 0])
    s["r_mass_rate"] = np.float64(r.mass_rate[0, 0])
    s["r_prev_I"] = np.diag(r.prev_I).astype(np.float64)
    s["r_prev_I_offdiag_absmax"] = np.float64(np.abs(r.prev_I - np.diag(np.diag(r.prev_I))).max())
    s["r_len_is_f32"] = np.int64(isinstance(r.length, np.float32))
    s["r_width_is_f32"] = np.int64(isinstance(r.width, np.float32))
    s["r_vol_is_f32"] = np.int64(isinstance(r.volume, np.float32))
    s["r_pvol_is_f32"] = np.int64(isinstance(r.prev_water_volume, np.float32))
    s["r_mass_is_f32"] = np.int64(r.mass.dtype == np.float32)
    s["r_phase"] = np.int64(r.state.value)
    s["r_cycle"] = np.int64(r.cycle)
    for k in NOZ:
        s["n_" + k] = np.float64(getattr(r.nozzle, k))
    s["e_target"] = np.array(env.target_point, dtype=np.float32, copy=True).reshape(2)
    obs = np.zeros((MAX_OBS, 2), np.float32)
    for i, o in enumerate(env.obstacles):
        obs[i] = o
    s["e_obstacles"] = obs
    s["e_n_obstacles"] = np.int64(len(env.obstacles))
    s["e_prev_dist"] = np.float64(env.prev_dist)
    pa = np.asarray(env.prev_action)
    s["e_prev_action"] = pa.astype(np.float64)
    s["e_prev_action_is_f32"] = np.int64(pa.dtype == np.float32)
    # episode trackers (src/salp_robot_env.py:145-153, 199, 237-248)
    pos = env.episode_positions
    s["e_ep_len"] = np.int64(len(env.episode_actions))
    pl = 0
    for i in range(len(pos) - 1):
        pl = pl + np.linalg.norm(pos[i + 1] - pos[i])
    s["e_path_length"] = np.float64(pl)
    s["e_last_pos"] = np.array(pos[-1], np.float64, copy=True)
    acts = np.array(env.episode_actions, np.float64).reshape(-1, 3)
    s["e_sum_a0"] = np.float64(sum(acts[:, 0].tolist()))
    s["e_sum_a1"] = np.float64(sum(acts[:, 1].tolist()))
    s["e_sum_abs_a2"] = np.float64(sum(np.abs(acts[:, 2]).tolist()))
    s["e_sum_vel"] = np.float64(sum(float(v) for v in env.episode_velocities))
    s["e_initial_distance"] = np.float64(env.initial_target_distance)
    s["e_sum_reward"] = np.float64(sum(float(x) for x in env.episode_rewards))
    comp_keys = ['rewards/track', 'rewards/heading', 'rewards/smooth', 'rewards/yaw',
                 'rewards/time', 'rewards/sideslip', 'rewards/obstacle']
    s["e_sum_comp"] = np.array([sum(c[k] for c in env.episode_reward_components)
                                for k in comp_keys], np.float64)
    return s


COMP_KEYS = ['rewards/track', 'rewards/heading', 'rewards/smooth', 'rewards/yaw',
             'rewards/time', 'rewards/sideslip', 'rewards/obstacle']
METRIC_KEYS = ['path_length', 'direct_distance', 'path_efficiency', 'final_distance',
               'initial_distance', 'avg_compression', 'avg_coast_time', 'avg_nozzle_angle',
               'avg_velocity', 'avg_rewards_track', 'avg_rewards_heading', 'avg_rewards_smooth',
               'avg_rewards_yaw', 'avg_rewards_time', 'avg_rewards_sideslip',
               'avg_rewards_obstacle']


def _pad_obs(o):
    out = np.full(6 + 2 * MAX_OBS, np.nan, np.float32)
    o = np.asarray(o, np.float32)
    out[:len(o)] = o
    return out


def run_episode_job(job):
    """One scripted rollout; returns a list of per-step records."""
    ref_robot, ref_env = _import_reference()
    seed, kind, n_steps = job["seed"], job["kind"], job["n_steps"]
    np.random.seed(seed)  # reference draws targets/obstacles from global np.random
    env = make_env(ref_robot, ref_env, num_obstacles=job.get("num_obstacles", 2))
    obs0, _ = env.reset()
    if "inject" in job:  # place target / obstacles by hand (edge cases)
        tgt, obst = job["inject"]
        env.target_point = np.asarray(tgt, np.float32)
        env.obstacles = [np.asarray(o, np.float32) for o in obst]
        env.prev_dist = np.linalg.norm(env.robot.position_world[0:-1] - env.target_point)
        env.episode_distances_to_target = [env.prev_dist]
        env.initial_target_distance = env.prev_dist
        obs0 = env._get_observation()
    rng = np.random.default_rng(1000 + seed)
    recs = []
    reset_obs = [np.asarray(obs0, np.float32)]
    for t in range(n_steps):
        if kind == "fixed":
            a = FIXED_ACTIONS[t % len(FIXED_ACTIONS)].copy()
        elif kind == "random":
            a = rng.uniform([0, 0, -1], [1, 1, 1]).astype(np.float32)
        elif kind == "script":
            a = np.asarray(job["actions"][t % len(job["actions"])], np.float32)
        else:
            raise ValueError(kind)
        before = snapshot(env)
        obs, rew, term, trunc, info = env.step(a)
        after = snapshot(env)
        rec = {"action": a, "obs": _pad_obs(obs), "obs_dim": np.int64(len(obs)),
               "reward": np.float64(rew),
               "terminated": np.int64(bool(term)), "truncated": np.int64(bool(trunc)),
               "comp": np.array([info[k] for k in COMP_KEYS], np.float64),
               "metrics": np.array([info.get(k, np.nan) for k in METRIC_KEYS], np.float64),
               "has_metrics": np.int64("final_distance" in info)}
        for k, v in before.items():
            rec["b_" + k] = v
        for k, v in after.items():
            rec["a_" + k] = v
        if term or trunc:
            o, _ = env.reset()
            rec["reset_obs"] = _pad_obs(o)
            for k, v in snapshot(env).items():
                rec["r_" + k] = v
        recs.append(rec)
    return {"job": job, "recs": recs, "reset_obs0": _pad_obs(reset_obs[0])}


def run_trace_job(job):
    """Per-tick histories of a bare robot (src/robot.py:740-777, record=True)."""
    ref_robot, _ = _import_reference()
    c = CANON
    nozzle = ref_robot.Nozzle(length1=c["length1"], length2=c["length2"], length3=c["length3"],
                              area=c["area"], mass=c["nozzle_mass"])
    robot = ref_robot.Robot(dry_mass=c["dry_mass"], init_length=c["init_length"],
                            init_width=c["init_width"], max_contraction=c["max_contraction"],
                            nozzle=nozzle)
    robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
    robot.set_environment(density=c["density"])
    robot.reset()
    robot.enable_history_recording()
    keys = ["position_world_history", "velocity_history", "acceleration_history",
            "euler_angle_history", "euler_angle_rate_history", "angular_velocity_history",
            "angular_acceleration_history", "length_history", "width_history",
            "volume_history", "mass_history", "inertia_tensor_history",
            "center_of_mass_history", "center_of_mass_rate_history",
            "center_of_mass_acc_rate_history", "jet_velocity_history", "jet_force_history",
            "jet_torque_history", "drag_force_history", "drag_torque_history",
            "coriolis_force_history", "coriolis_torque_history", "added_mass_force_history",
            "added_mass_torque_history", "deform_torque_history", "acceleration_force_history",
            "state_history"]
    out = {k: [] for k in keys}
    cycle_id = []
    acts = job["actions"]
    for i, a in enumerate(acts):
        a = np.asarray(a, np.float32)
        # same arithmetic as SalpRobotEnv._rescale_action (src/salp_robot_env.py:166-174)
        resc = np.zeros_like(a)
        resc[0] = a[0] * 0.06
        resc[1] = a[1] * 10.0
        resc[2] = a[2] * (np.pi / 2)
        robot.nozzle.set_yaw_angle(yaw_angle=resc[2])
        robot.nozzle.solve_angles()
        robot.set_control(resc[0], resc[1], np.array([robot.nozzle.angle1, robot.nozzle.angle2]))
        robot.step_through_cycle()
        n = len(robot.length_history)
        for k in keys:
            v = getattr(robot, k)
            if k == "state_history":
                v = np.array([s.value for s in v])
            v = np.asarray(v, np.float64)
            if k.startswith(("jet_", "drag_", "coriolis_", "added_", "deform_", "acceleration_force")):
                # force histories have one entry fewer (no initial value)
                v = np.concatenate([np.full((1,) + v.shape[1:], np.nan), v], 0)
            out[k].append(v)
        cycle_id.append(np.full(n, i))
    res = {k: np.concatenate(v, 0) for k, v in out.items()}
    res["cycle_id"] = np.concatenate(cycle_id)
    res["actions"] = np.asarray(acts, np.float32)
    return res


HIST_KEYS = ["position_world_history", "velocity_history", "acceleration_history",
             "euler_angle_history", "euler_angle_rate_history", "angular_velocity_history",
             "angular_acceleration_history", "length_history", "width_history", "area_history",
             "volume_history", "mass_history", "mass_rate_history", "nozzle_yaw_history",
             "inertia_tensor_history", "trans_drag_coefficient_history",
             "rot_drag_coefficient_history", "center_of_mass_history",
             "center_of_mass_rate_history", "center_of_mass_acc_rate_history",
             "position_front_world_history", "jet_velocity_history", "jet_force_history",
             "jet_torque_history", "drag_force_history", "drag_torque_history",
             "coriolis_force_history", "coriolis_torque_history", "added_mass_force_history",
             "added_mass_torque_history", "deform_torque_history", "asymmetry_torque_history",
             "acceleration_force_history", "state_history"]
FORCE_KEYS = ("jet_", "drag_", "coriolis_", "added_", "deform_", "asymmetry_", "acceleration_force")
ROBOT_STATE = ["velocity", "angular_velocity", "acceleration", "angular_acceleration", "euler_angle",
               "position_world", "position", "angle", "prev_position", "prev_angle",
               "avg_cycle_velocity", "avg_cycle_angular_velocity"]
ROBOT_SCAL = ["length", "width", "volume", "prev_water_volume", "cycle_time", "time", "refill_time",
              "jet_time", "coast_time", "contraction", "_contract_rate", "_release_rate"]


def run_robot_job(job):
    """Bare robot driven with Python-float controls (float64 geometry)."""
    ref_robot, _ = _import_reference()
    c = job["robot"]
    nozzle = ref_robot.Nozzle(length1=c["length1"], length2=c["length2"], length3=c["length3"],
                              area=c["area"], mass=c["nozzle_mass"])
    robot = ref_robot.Robot(dry_mass=c["dry_mass"], init_length=c["init_length"],
                            init_width=c["init_width"], max_contraction=c["max_contraction"],
                            nozzle=nozzle)
    robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
    robot.set_environment(density=c["density"])
    robot.enable_history_recording()
    robot.reset()
    hist = {k: [] for k in HIST_KEYS}
    cyc, end = [], {}
    for i, (contraction, coast, yaw) in enumerate(job["controls"]):
        if i == job.get("reset_at", -1):
            robot.reset()
        robot.nozzle.set_yaw_angle(yaw_angle=float(yaw))
        robot.nozzle.solve_angles()
        robot.set_control(contraction=float(contraction), coast_time=float(coast),
                          nozzle_angles=np.array([robot.nozzle.angle1, robot.nozzle.angle2]))
        robot.step_through_cycle()
        n = len(robot.length_history)
        for k in HIST_KEYS:
            v = getattr(robot, k)
            if k == "state_history":
                v = [s.value for s in v]
            elif k in ("mass_history", "mass_rate_history"):
                v = [np.asarray(x, np.float64).reshape(-1)[0] for x in v]
            elif k == "inertia_tensor_history":
                v = [np.asarray(x, np.float64).reshape(3) for x in v]
            v = np.asarray(v, np.float64)
            if k.startswith(FORCE_KEYS):
                v = np.concatenate([np.full((1,) + v.shape[1:], np.nan), v], 0)
            hist[k].append(v)
        cyc.append(np.full(n, i))
        for k in ROBOT_STATE:
            end.setdefault("end_" + k, []).append(np.array(getattr(robot, k), np.float64).reshape(3))
        for k in ROBOT_SCAL:
            end.setdefault("end_" + k, []).append(np.float64(getattr(robot, k)))
        end.setdefault("end_center_of_mass", []).append(np.float64(robot.center_of_mass[0]))
        end.setdefault("end_prev_I", []).append(np.diag(robot.prev_I).astype(np.float64))
        end.setdefault("end_phase", []).append(np.int64(robot.state.value))
        end.setdefault("end_cycle", []).append(np.int64(robot.cycle))
        for k in ("angle1", "angle2", "prev_angle1", "prev_angle2", "yaw", "prev_yaw", "turn_time"):
            end.setdefault("end_n_" + k, []).append(np.float64(getattr(robot.nozzle, k)))
    res = {k: np.concatenate(v, 0) for k, v in hist.items()}
    res["cycle_id"] = np.concatenate(cyc)
    res.update({k: np.asarray(v) for k, v in end.items()})
    res["controls"] = np.asarray(job["controls"], np.float64)
    res["reset_at"] = np.int64(job.get("reset_at", -1))
    return res


# the demo robot of src/robot.py:1104-1107
DEMO = dict(length1=0.052, length2=0.039, length3=0.031, area=np.pi * 0.01 ** 2, nozzle_mass=0.440,
            dry_mass=0.756, init_length=0.26, init_width=0.14, max_contraction=0.04, density=1000)
ROBOT_JOBS = [
    # src/robot.py:1149-1152: contraction 0.03, coast 2, yaw 0 (Python floats)
    dict(name="canon", robot=CANON, controls=[(0.03, 2.0, 0.0), (0.03, 2.0, 0.0),
                                              (0.05, 0.5, 0.7), (0.012, 0.3, -1.2),
                                              (0.06, 1.0, 1.5707963267948966)], reset_at=4),
    dict(name="demo", robot=DEMO, controls=[(0.03, 2.0, 0.0), (0.04, 1.0, -0.4),
                                            (0.02, 0.2, 0.9), (0.035, 0.7, -1.5)]),
]


def build_jobs():
    jobs = [dict(seed=0, kind="fixed", n_steps=40)]
    for s in range(1, 17):
        jobs.append(dict(seed=s, kind="random", n_steps=30))
    # zero-tick / negative-polynomial cycles, then a timeout at cycle 500
    jobs.append(dict(seed=101, kind="script", n_steps=503,
                     actions=[[0.0, 0.0, 0.0]] * 499 + [[0.05, 0.02, 0.3]] * 4))
    # tiny contractions (refill<0, jet<0) with coasting
    jobs.append(dict(seed=102, kind="script", n_steps=12,
                     actions=[[0.05, 0.3, 0.5], [0.08, 0.1, -0.7], [0.0, 0.5, 1.0],
                              [0.089, 0.0, -1.0], [0.09, 0.01, 0.0], [1.0, 1.0, 1.0],
                              [1.0, 0.0, -1.0], [0.0, 0.001, 0.0]]))
    # drive into an obstacle placed straight ahead (-x is the jet direction's opposite)
    jobs.append(dict(seed=103, kind="script", n_steps=10, inject=([1.9, 0.0], [[0.45, 0.0], [0.0, 1.2]]),
                     actions=[[1.0, 0.05, 0.0]]))
    # target right next to start -> success after a short hop
    jobs.append(dict(seed=104, kind="script", n_steps=6, inject=([0.25, 0.0], [[1.0, 1.0], [1.5, -1.0]]),
                     actions=[[1.0, 0.05, 0.0]]))
    # no obstacles env (obs_dim 6) and 4 obstacles env (obs_dim 14)
    jobs.append(dict(seed=105, kind="random", n_steps=12, num_obstacles=0))
    jobs.append(dict(seed=106, kind="random", n_steps=12, num_obstacles=4))
    return jobs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", choices=["robot"], default=None)
    args = ap.parse_args()
    ctx = mp.get_context("fork")
    with ctx.Pool(args.jobs) as pool:
        robots = pool.map(run_robot_job, ROBOT_JOBS, chunksize=1)
    out = {}
    for job, res in zip(ROBOT_JOBS, robots):
        for k, v in res.items():
            out[f"{job['name']}/{k}"] = v
        for k, v in job["robot"].items():
            out[f"{job['name']}/param_{k}"] = np.float64(v)
    np.savez_compressed(os.path.join(OUT_DIR, "robot_trace.npz"), **out)
    if args.only == "robot":
        print("robot trace samples", {j["name"]: len(r["cycle_id"]) for j, r in zip(ROBOT_JOBS, robots)})
        return
    jobs = build_jobs()
    ctx = mp.get_context("fork")
    with ctx.Pool(args.jobs) as pool:
        trace_async = pool.apply_async(run_trace_job, (dict(actions=FIXED_ACTIONS[:4]),))
        results = pool.map(run_episode_job, jobs, chunksize=1)
        trace = trace_async.get()
    np.savez_compressed(os.path.join(OUT_DIR, "tick_trace.npz"), **trace)

    # flatten episode records into columns
    cols = {}
    keys = set()
    for res in results:
        for rec in res["recs"]:
            keys.update(rec.keys())
    keys = sorted(keys)
    rows = []
    for ji, res in enumerate(results):
        for t, rec in enumerate(res["recs"]):
            rows.append((ji, t, rec))
    template = {}
    for _, _, rec in rows:
        for k, v in rec.items():
            template.setdefault(k, np.asarray(v))
    for k in keys:
        tv = template[k]
        arr = np.zeros((len(rows),) + tv.shape, dtype=tv.dtype)
        if arr.dtype.kind == "f":
            arr[:] = np.nan
        for i, (_, _, rec) in enumerate(rows):
            if k in rec:
                arr[i] = rec[k]
        cols[k] = arr
    cols["job_index"] = np.array([r[0] for r in rows], np.int64)
    cols["step_index"] = np.array([r[1] for r in rows], np.int64)
    cols["has_reset"] = np.array(["reset_obs" in r[2] for r in rows], np.int64)
    cols["num_obstacles_cfg"] = np.array([results[r[0]]["job"].get("num_obstacles", 2) for r in rows],
                                         np.int64)
    cols["reset_obs0"] = np.zeros((len(results), 6 + 2 * MAX_OBS), np.float32)
    for ji, res in enumerate(results):
        o = res["reset_obs0"]
        cols["reset_obs0"][ji, :len(o)] = o
    # obs arrays vary in length with num_obstacles: store padded
    np.savez_compressed(os.path.join(OUT_DIR, "episodes.npz"), **cols)
    print("rows", len(rows), "trace ticks", len(trace["length_history"]))


if __name__ == "__main__":
    main()
