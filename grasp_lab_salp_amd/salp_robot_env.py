"""Drop-in ``SalpRobotEnv`` (reference: src/salp_robot_env.py:22-670).

Same constructor, spaces, ``reset`` / ``step`` signatures, return types,
reward, termination and ``info`` keys as the reference's Gymnasium env, so the
``make_env`` of src/train_robot.py:11-21 runs unchanged with
``from grasp_lab_salp_amd.salp_robot_env import SalpRobotEnv``.  One env-step
(one breathing cycle, hundreds of physics ticks) runs as one launch of the
HIP step kernel on a 1-env :class:`BatchedSalpEnv`; for many envs use
:class:`~grasp_lab_salp_amd.vec_env.SalpVecEnv`, which runs them all in one
launch.

Targets and obstacles are drawn on the host from the process-global
``np.random`` exactly as the reference draws them
(src/salp_robot_env.py:449-559), then handed to the device: seeding
``np.random`` reproduces the reference's episodes.

The action / observation randomisation and latency options (off in every
reference script, src/salp_robot_env.py:54-56) run on the device with Philox
draws (grasp_lab_salp_amd/csrc/salp_random.h).  Not on the device (fail
loudly): pygame rendering / GIF recording / the interactive loop
(visualisation, src/salp_robot_env.py:586-1595).
"""
import ctypes
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._abi import EPISODE_METRIC_KEYS, FIELD, INFO, INFO_DIM, MAX_OBSTACLES, REWARD_COMPONENT_KEYS
from .batched_env import BatchedSalpEnv
from .robot import Robot
from .spaces import Box, GymEnv

__all__ = ["SalpRobotEnv", "draw_target", "draw_obstacles", "TANK_MARGIN", "SCALE"]

TANK_MARGIN = 50          # pixels (src/salp_robot_env.py:42)
SCALE = 200.0             # pixels per meter (src/salp_robot_env.py:470)
TARGET_RADIUS = 0.2       # success radius, m (src/salp_robot_env.py:43)
MIN_CLEAR = 0.5           # obstacle clearance from start and target, m (:543)


def _tank(width, height, margin=TANK_MARGIN):
    return ((-width / 2 + margin) / SCALE, (width / 2 - margin) / SCALE,
            (-height / 2 + margin) / SCALE, (height / 2 - margin) / SCALE)


def draw_target(width, height, strategy="random", current_pos=None, center=None, max_distance=2.0):
    """generate_target_point (src/salp_robot_env.py:449-533): a float32 [x, y]
    drawn from the global np.random in the reference's call order, clamped to
    the tank.  Unknown strategies raise ValueError like the reference."""
    x_min, x_max, y_min, y_max = _tank(width, height)
    cur = np.zeros(2) if current_pos is None else np.asarray(current_pos, np.float64)[:2]
    if strategy == "random":
        tx = np.random.uniform(x_min, x_max)
        ty = np.random.uniform(y_min, y_max)
        target = np.array([tx, ty])
    elif strategy == "relative":
        c = cur if center is None else np.asarray(center)
        dist = np.random.uniform(0.1, max_distance)
        ang = np.random.uniform(0, 2 * np.pi)
        target = c + dist * np.array([np.cos(ang), np.sin(ang)])
    elif strategy == "circle":
        c = cur if center is None else np.asarray(center)
        ang = np.random.uniform(0, 2 * np.pi)
        target = c + max_distance * np.array([np.cos(ang), np.sin(ang)])
    elif strategy == "corridor":
        c = cur if center is None else np.asarray(center)
        target = np.array([np.random.uniform(x_min, x_max), c[1]])
    else:
        raise ValueError(f"Unknown target generation strategy: {strategy}")
    target[0] = np.clip(target[0], x_min, x_max)
    target[1] = np.clip(target[1], y_min, y_max)
    return target.astype(np.float32)


def _frozen(a):
    """A read-only copy of an array-like attribute (None stays None)."""
    if a is None:
        return None
    a = np.array(a, copy=True)
    a.flags.writeable = False
    return a


def draw_obstacles(width, height, num_obstacles, obstacle_radius, target):
    """_generate_obstacles (src/salp_robot_env.py:535-559): rejection sampling
    from the global np.random, at most 200 tries per obstacle; the list can
    come out shorter than num_obstacles."""
    x_min, x_max, y_min, y_max = _tank(width, height)
    sep = 2 * obstacle_radius + 0.1
    placed = []
    for _ in range(num_obstacles):
        for _try in range(200):
            px = np.random.uniform(x_min, x_max)
            py = np.random.uniform(y_min, y_max)
            pos = np.array([px, py], dtype=np.float32)
            ok = np.linalg.norm(pos) > MIN_CLEAR and np.linalg.norm(pos - target) > MIN_CLEAR
            ok = ok and not any(np.linalg.norm(pos - o) < sep for o in placed)
            if ok:
                placed.append(pos)
                break
    return placed


class _StepIO:
    """The per-env step's host boundary at its cheapest: the action goes up
    through a pinned buffer, salp_step (no auto-reset) writes obs / reward /
    flags / info into one packed device buffer, which comes back in one copy
    into a pinned buffer with NumPy views made once; the C ABI is called with
    pointers made once (BatchedSalpEnv.step validates and allocates per call)."""

    def __init__(self, sim):
        self.sim = sim
        od, dev = sim.obs_dim, sim.device
        parts = [("info", INFO_DIM, np.float64), ("reward", 1, np.float64), ("obs", od, np.float32),
                 ("terminated", 1, np.uint8), ("truncated", 1, np.uint8)]
        off, lay = 0, {}
        for name, count, dt in parts:
            lay[name] = (off, count, dt)
            off += (count * np.dtype(dt).itemsize + 15) // 16 * 16
        self.act_host = torch.empty((1, 3), dtype=torch.float32, pin_memory=True)
        self.act_np = self.act_host.numpy()
        self.act_dev = torch.empty((1, 3), dtype=torch.float32, device=dev)
        self.out_dev = torch.empty(off, dtype=torch.uint8, device=dev)
        self.out_host = torch.empty(off, dtype=torch.uint8, pin_memory=True)
        raw = self.out_host.numpy()
        self.views = {k: raw[o:o + c * np.dtype(dt).itemsize].view(dt) for k, (o, c, dt) in lay.items()}
        base = self.out_dev.data_ptr()
        p = {k: ctypes.c_void_p(base + o) for k, (o, _c, _dt) in lay.items()}
        self.args = (ctypes.c_void_p(self.act_dev.data_ptr()), p["obs"], p["reward"], p["terminated"],
                     p["truncated"], 0, None, p["info"])

    # k_step_wave's two waves meet through LDS once per tick; a wait that gives
    # up (never seen: a workgroup's waves are co-resident) invalidates the env's
    # results and is counted on the device.  Read every CHECK_EVERY steps and at
    # close (a read costs a synchronising copy; include/salp.h salp_pair_timeouts).
    CHECK_EVERY = 1024

    def check(self):
        self.sim.check_pair()

    def step(self, a):
        sim = self.sim
        self.n_steps = getattr(self, "n_steps", 0) + 1
        if self.n_steps % self.CHECK_EVERY == 0:
            self.check()
        self.act_np[0] = a
        stream = torch.cuda.current_stream(sim.device)
        self.act_dev.copy_(self.act_host, non_blocking=True)
        sim._run(_lib.load().salp_step(sim.handle, *self.args, ctypes.c_void_p(stream.cuda_stream)))
        self.out_host.copy_(self.out_dev, non_blocking=True)
        stream.synchronize()
        return self.views


class SalpRobotEnv(GymEnv):
    """The reference task env on the device (see module docstring)."""

    metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 60}

    def __init__(self, render_mode: Optional[str] = None, width: int = 900, height: int = 700,
                 robot: Optional[Robot] = None, num_obstacles: int = 2, obstacle_radius: float = 0.2,
                 device: Optional[int] = None):
        if robot is None:
            raise AttributeError("SalpRobotEnv needs a Robot (the reference fails in reset() without one)")
        if not 0 <= num_obstacles <= MAX_OBSTACLES:
            raise ValueError(f"num_obstacles must be in [0, {MAX_OBSTACLES}] on the device")
        self.width, self.height = width, height
        self.pos_init = np.array([width / 2, height / 2])
        self.tank_margin = TANK_MARGIN
        self.target_radius = TARGET_RADIUS
        self.num_obstacles = num_obstacles
        self.obstacle_radius = obstacle_radius
        self._obstacles = []
        self._target_point = None
        self.render_mode = render_mode
        self.action_randomization = False
        self.observation_randomization = False
        self.latency = False
        self.robot = robot
        self.action = np.array([0.0, 0.0, 0.0])
        self.prev_action = np.array([0.0, 0.0, 0.0])
        self.action_space = Box(low=np.array([0.0, 0.0, -1.0]), high=np.array([1.0, 1.0, 1.0]),
                                dtype=np.float32)
        obs_dim = 6 + 2 * num_obstacles
        self.observation_space = Box(low=np.full(obs_dim, -np.inf, dtype=np.float32),
                                     high=np.full(obs_dim, np.inf, dtype=np.float32), dtype=np.float32)
        self.np_random = np.random.default_rng()
        params = robot.salp_params(width=int(width), height=int(height), num_obstacles=int(num_obstacles),
                                   obstacle_radius=float(obstacle_radius))
        self._sim = BatchedSalpEnv(1, params=params, device=device)
        self._io = _StepIO(self._sim)
        robot._bind(self._sim, 0, owner=self)
        self._last_obs = None
        self._last_info = None
        self.reset()

    # ------------------------------------------------------------ options
    def enable_action_randomization(self):
        """src/salp_robot_env.py:157-158, 176-181 (device Philox draws)."""
        self.action_randomization = True
        self._sync_randomization()

    def enable_observation_randomization(self):
        """src/salp_robot_env.py:160-161, 183-194; the observation stays float32
        (the reference's randomised observation is a float64 array)."""
        self.observation_randomization = True
        self._sync_randomization()

    def enable_latency(self):
        """src/salp_robot_env.py:163-164, 292-297."""
        self.latency = True
        self._sync_randomization()

    def _sync_randomization(self):
        self._sim.set_randomization(self.robot.dynamics_randomization, self.robot.disturbances,
                                    self.action_randomization, self.observation_randomization, self.latency)

    # ------------------------------------------------------------ task attributes
    # Plain attributes in the reference, read by its own step() every cycle
    # (src/salp_robot_env.py:349-397, 561-568, 651-670).  Assigning one between
    # steps - placing a target or obstacles by hand, as the edge-case episodes
    # of tests/golden/make_golden.py do - changes what the next step computes,
    # so here the setters write the value through to the env's device state.
    # The observation is recomputed by the next step() / reset().  Only a whole
    # assignment reaches the device: the getters hand out read-only copies (a
    # tuple of read-only arrays for the obstacles), so an in-place edit
    # (env.obstacles[0][0] = ..., env.obstacles.append(...)) raises instead of
    # silently changing a host copy the simulation never reads.
    @property
    def target_point(self):
        return _frozen(self._target_point)

    @target_point.setter
    def target_point(self, value):
        self._target_point = value
        v = np.asarray(value, dtype=np.float64).reshape(-1)
        self._write_fields({"target0": v[0], "target1": v[1]})

    @property
    def obstacles(self):
        return tuple(_frozen(o) for o in self._obstacles)

    @obstacles.setter
    def obstacles(self, value):
        value = list(value)
        if len(value) > self.num_obstacles:
            raise ValueError(f"at most num_obstacles = {self.num_obstacles} obstacles (observation size)")
        self._obstacles = value
        vals = {"n_obst": float(len(value))}
        for k in range(MAX_OBSTACLES):
            o = np.asarray(value[k], dtype=np.float64).reshape(-1) if k < len(value) else np.zeros(2)
            vals[f"obst{2 * k}"], vals[f"obst{2 * k + 1}"] = o[0], o[1]
        self._write_fields(vals)

    @property
    def prev_dist(self):
        return float(self._sim.field("prev_dist")[0])

    @prev_dist.setter
    def prev_dist(self, value):
        self._write_fields({"prev_dist": value})

    @property
    def initial_target_distance(self):
        return float(self._sim.field("init_dist")[0])

    @initial_target_distance.setter
    def initial_target_distance(self, value):
        self._write_fields({"init_dist": value})

    def _write_fields(self, values):
        sim = getattr(self, "_sim", None)
        if sim is None:   # during __init__, before the device env exists
            return
        st = sim.get_state()
        for name, v in values.items():
            st[FIELD[name], 0] = float(v)
        sim.set_state(st)

    # ------------------------------------------------------------ helpers
    def generate_target_point(self, strategy: str = "random", center=None, max_distance: float = 2.0):
        cur = self.robot.position_world[:2] if self.robot._bound else None
        return draw_target(self.width, self.height, strategy, cur, center, max_distance)

    def _generate_obstacles(self):
        self._obstacles = draw_obstacles(self.width, self.height, self.num_obstacles,
                                         self.obstacle_radius, self.target_point)

    @staticmethod
    def _rescale_action(action):
        """src/salp_robot_env.py:166-174 (the device does the same in float32)."""
        r = np.zeros_like(action)
        r[0] = action[0] * 0.06
        r[1] = action[1] * 10.0
        r[2] = action[2] * (np.pi / 2)
        return r

    def sample_random_action(self) -> np.ndarray:
        return self.action_space.sample().astype(np.float32)

    def get_cycle_count(self) -> int:
        return self.robot.cycle

    def _obs_len(self):
        return 6 + 2 * len(self.obstacles)

    def _get_observation(self) -> np.ndarray:
        """Observation of the current state (src/salp_robot_env.py:651-670),
        as computed by the last device call."""
        return self._last_obs.copy()

    def _check_obstacle_collision(self) -> bool:
        return bool(self._last_info is not None and self._last_info[INFO["hit_obstacle"]] != 0)

    def _calculate_episode_metrics(self) -> Dict[str, float]:
        row = self._last_info
        return {k: float(row[INFO[k]]) for k in EPISODE_METRIC_KEYS}

    # ------------------------------------------------------------ gym API
    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None) -> Tuple[np.ndarray, Dict]:
        """src/salp_robot_env.py:114-155.  Like the reference, `seed` only
        seeds self.np_random; targets and obstacles come from np.random."""
        if seed is not None:
            self.np_random = np.random.default_rng(seed)
        # drawn on the host, handed to the device by reset_to below
        self._target_point = self.generate_target_point(strategy="random")
        self._generate_obstacles()
        ob = np.zeros((1, MAX_OBSTACLES, 2), np.float32)
        for k, o in enumerate(self.obstacles):
            ob[0, k] = o
        obs = self._sim.reset_to(np.array(self._target_point, dtype=np.float32)[None], ob, [len(self._obstacles)])
        self.prev_action = np.array([0.0, 0.0, 0.0])
        self.action = np.array([0.0, 0.0, 0.0])
        self._last_obs = obs[0, :self._obs_len()].cpu().numpy()
        self._last_info = None
        self.robot._clear_history()
        return self._get_observation(), {}

    def step(self, action: np.ndarray) -> Tuple[np.ndarray, float, bool, bool, Dict]:
        """src/salp_robot_env.py:196-299: one breathing cycle on the device."""
        a = np.asarray(action, dtype=np.float32).reshape(3)   # SB3 passes the Box dtype
        self.action = a.copy()
        record = self.robot.record
        if record and self._sim._trace is None:
            self._sim.enable_trace(Robot._trace_capacity())
        elif not record and self._sim._trace is not None:
            self._sim.disable_trace()
        io = self._io.step(a)
        obs = io["obs"][:self._obs_len()].copy()
        reward, done, truncated = float(io["reward"][0]), bool(io["terminated"][0]), bool(io["truncated"][0])
        self._last_obs = obs
        self._last_info = io["info"].copy()
        if record:
            self.robot._load_history()
        info = {"position_history": self.robot.position_world_history,
                "length_history": self.robot.length_history,
                "width_history": self.robot.width_history}
        info.update({k: float(self._last_info[INFO[k]]) for k in REWARD_COMPONENT_KEYS})
        if done or truncated:
            info.update(self._calculate_episode_metrics())
        self.prev_action = self.action
        return obs.copy(), reward, done, truncated, info

    def render(self):
        raise NotImplementedError("rendering (pygame, src/salp_robot_env.py:1198-1258) is out of scope")

    def close(self):
        self._io.check()
        self._sim.close()
