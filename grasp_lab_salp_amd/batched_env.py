"""BatchedSalpEnv — n SALP envs on one GPU, torch tensors in and out.

This is the batched form of the reference's ``SalpRobotEnv``
(src/salp_robot_env.py:22-670): every call runs the corresponding reference
method for all envs at once in libsalp.so (HIP, gfx950).  Tensors are
torch.cuda tensors on the handle's device; work is enqueued on torch's
current stream and nothing synchronises unless a result is read on the host.
"""
import ctypes

import torch

from . import _lib
from ._abi import (EPISODE_METRIC_KEYS, FIELD, FIELDS, INFO, INFO_DIM, INFO_KEYS, MAX_OBSTACLES, POLICY_SIZE,
                   NUM_FIELDS, REWARD_COMPONENT_KEYS, TRACE_DIM, SalpParams, default_params)

__all__ = ["BatchedSalpEnv", "StepResult"]


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class StepResult:
    """Outputs of one batched env.step (all device tensors)."""

    __slots__ = ("obs", "reward", "terminated", "truncated", "terminal_obs", "info")

    def __init__(self, obs, reward, terminated, truncated, terminal_obs, info):
        self.obs, self.reward = obs, reward
        self.terminated, self.truncated = terminated, truncated
        self.terminal_obs, self.info = terminal_obs, info

    def __iter__(self):  # obs, reward, terminated, truncated, info — gymnasium order
        return iter((self.obs, self.reward, self.terminated, self.truncated, self.info))


class BatchedSalpEnv:
    """``n_envs`` independent reference envs simulated in one kernel per call.

    Args:
        n_envs: number of envs on this device.
        params: :class:`SalpParams` (constructor arguments of Nozzle / Robot /
            SalpRobotEnv); defaults to the canonical ``make_env`` config of
            src/train_robot.py:11-21.
        seed: Philox key for synthetic actions and reset draws.
        env_id_offset: global id of env 0 (multi-GPU sharding: trajectories of
            a given global env id do not depend on the sharding).
        device: CUDA (HIP) device index.
    """

    def __init__(self, n_envs, params=None, seed=0, env_id_offset=0, device=None):
        if not torch.cuda.is_available():
            raise _lib.SalpError("BatchedSalpEnv needs a ROCm GPU (no CPU fallback)")
        L = _lib.load()
        self.params = params if params is not None else default_params()
        if not isinstance(self.params, SalpParams):
            raise TypeError("params must be a SalpParams")
        self.n_envs = int(n_envs)
        self.seed = int(seed)
        self.env_id_offset = int(env_id_offset)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.salp_create(ctypes.byref(self.params), self.n_envs, self.seed,
                                     self.env_id_offset, self.device.index, ctypes.byref(h)))
        self._h = h
        self.obs_dim = L.salp_obs_dim(h)
        self.num_obstacles = self.params.num_obstacles
        self._trace = None
        self.version = 0   # bumped by every call that changes the device state

    # ------------------------------------------------------------ plumbing
    @property
    def handle(self):
        return self._h

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc):
        return _lib.check(rc, self._h)

    def _run(self, rc):
        """check + mark the state as changed (host-side caches key on version)."""
        self.version += 1
        return _lib.check(rc, self._h)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().salp_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _f32(self, x, shape):
        t = torch.as_tensor(x, dtype=torch.float32, device=self.device).reshape(shape).contiguous()
        return t

    def _mask(self, mask):
        if mask is None:
            return None
        return torch.as_tensor(mask, device=self.device).reshape(self.n_envs).to(torch.uint8).contiguous()

    # ------------------------------------------------------------- env API
    def reset(self, mask=None):
        """reset() of every env (or of the masked ones); returns obs [n, obs_dim].

        Targets and obstacles come from the env's Philox stream (the reference
        uses the process-global np.random, src/salp_robot_env.py:484-487)."""
        obs = torch.zeros((self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        m = self._mask(mask)
        self._run(_lib.load().salp_reset(self._h, _ptr(m), _ptr(obs), self._stream()))
        return obs

    def reset_to(self, targets, obstacles, n_obstacles=None, mask=None):
        """reset() with caller-given targets [n,2] and obstacles [n,k,2]."""
        t = self._f32(targets, (self.n_envs, 2))
        ob = torch.as_tensor(obstacles, dtype=torch.float32, device=self.device).reshape(self.n_envs, -1, 2)
        o = torch.zeros((self.n_envs, MAX_OBSTACLES, 2), dtype=torch.float32, device=self.device)
        o[:, :ob.shape[1]] = ob
        if n_obstacles is None:
            n_obstacles = torch.full((self.n_envs,), min(ob.shape[1], self.num_obstacles))
        k = torch.as_tensor(n_obstacles, device=self.device).reshape(self.n_envs).to(torch.int32).contiguous()
        obs = torch.zeros((self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        m = self._mask(mask)
        self._run(_lib.load().salp_reset_to(self._h, _ptr(m), _ptr(t), _ptr(o.contiguous()), _ptr(k),
                                              _ptr(obs), self._stream()))
        return obs

    def step(self, actions, auto_reset=False, want_terminal_obs=True, out=None):
        """One env.step per env. actions [n,3] float32 in Box([0,0,-1],[1,1,1]).

        Returns a :class:`StepResult`; ``info`` is an [n, INFO_DIM] fp64 tensor
        (columns ``_abi.INFO_KEYS``; see :meth:`info_dicts`).  ``out``: a dict of
        preallocated contiguous device tensors to write into instead ("obs" [n,
        obs_dim] f32, "reward" [n] f64, "terminated" / "truncated" [n] u8,
        "terminal_obs" [n, obs_dim] f32 or None, "info" [n, INFO_DIM] f64 or
        None); the result then holds those tensors (flags as u8)."""
        a = self._f32(actions, (self.n_envs, 3))
        if out is not None:
            n, od = self.n_envs, self.obs_dim
            want = {"obs": ((n, od), torch.float32), "reward": ((n,), torch.float64),
                    "terminated": ((n,), torch.uint8), "truncated": ((n,), torch.uint8),
                    "terminal_obs": ((n, od), torch.float32), "info": ((n, INFO_DIM), torch.float64)}
            for k, (shape, dt) in want.items():
                t = out.get(k)
                if t is None and k in ("terminal_obs", "info"):
                    continue
                if (t is None or tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous()
                        or t.device != self.device):
                    raise ValueError(f"step(out=...): {k!r} must be a contiguous {dt} tensor of shape {shape} "
                                     f"on {self.device}")
            obs, rew, term, trunc = out["obs"], out["reward"], out["terminated"], out["truncated"]
            tobs, info = out.get("terminal_obs"), out.get("info")
            self._run(_lib.load().salp_step(self._h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc),
                                              int(bool(auto_reset)), _ptr(tobs), _ptr(info), self._stream()))
            return StepResult(obs, rew, term, trunc, tobs, info)
        obs = torch.empty((self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        rew = torch.empty(self.n_envs, dtype=torch.float64, device=self.device)
        term = torch.empty(self.n_envs, dtype=torch.uint8, device=self.device)
        trunc = torch.empty(self.n_envs, dtype=torch.uint8, device=self.device)
        tobs = (torch.empty((self.n_envs, self.obs_dim), dtype=torch.float32, device=self.device)
                if want_terminal_obs else None)
        info = torch.empty((self.n_envs, INFO_DIM), dtype=torch.float64, device=self.device)
        self._run(_lib.load().salp_step(self._h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc),
                                          int(bool(auto_reset)), _ptr(tobs), _ptr(info), self._stream()))
        return StepResult(obs, rew, term.bool(), trunc.bool(), tobs, info)

    def step_random(self, n_steps):
        """n_steps synthetic random-action env-steps per env (lock-step, auto-reset).
        Returns the per-env reward sum (fp64)."""
        rs = torch.empty(self.n_envs, dtype=torch.float64, device=self.device)
        self._run(_lib.load().salp_step_random(self._h, int(n_steps), _ptr(rs), self._stream()))
        return rs

    def set_lockstep_order(self, mode):
        """Launch order of :meth:`step` / :meth:`step_random` (salp_set_lockstep_order):
        1 = envs sorted by the predicted length of their next cycle, 0 = env
        order, -1 = sorted from 1 024 envs on (default).  Results are identical
        in every mode."""
        self._check(_lib.load().salp_set_lockstep_order(self._h, int(mode)))

    def set_rollout_kernel(self, mode):
        """Kernel of :meth:`rollout`, :meth:`collect` and chained
        :meth:`step_random` (salp_set_rollout_kernel): 1 = two waves per env
        meeting once per tick (k_rollout_pair), 2 = two waves per env with the
        tick split one way (k_rollout_split), 0 = one env per lane (k_rollout),
        -1 = a two-wave kernel up to 128 envs per compute unit (default).
        Results are identical in every mode."""
        self._check(_lib.load().salp_set_rollout_kernel(self._h, int(mode)))

    def set_step_kernel(self, mode):
        """Kernel of :meth:`step` (salp_set_step_kernel): 1 = one env per wave
        (k_step_wave: the geometry of 64 ticks at once, then their dynamics),
        0 = one env per lane (k_step), -1 = one env per wave up to 1 024 envs
        (default).  Recording always uses k_step.  Results are identical in
        every mode."""
        self._check(_lib.load().salp_set_step_kernel(self._h, int(mode)))

    def pair_timeouts(self):
        """Partner waits of the two-wave kernels that gave up since the last
        call (salp_pair_timeouts; synchronises the stream).  Nonzero means some
        env's results of those launches are invalid."""
        c = ctypes.c_uint64(0)
        self._check(_lib.load().salp_pair_timeouts(self._h, ctypes.byref(c), self._stream()))
        return int(c.value)

    def check_pair(self):
        """Raise SalpError if a two-wave launch since the last check gave up
        on a partner wave (its envs' results are invalid)."""
        n = self.pair_timeouts()
        if n:
            raise _lib.SalpError(f"two-wave kernels (k_rollout_pair / k_step_wave): {n} partner wait(s) timed out; "
                                 "the affected envs' results are invalid")

    def rollout(self, tick_budget, buffers=None, steps_done=None, max_steps=0, chunk=64):
        """Chained random-action rollout: each env runs ``tick_budget`` physics
        ticks, completing as many env-steps as fit (auto-reset).  ``buffers`` is
        an optional dict of preallocated device tensors {obs [cap,n,obs_dim]
        (after the step), obs_before [cap,n,obs_dim] (the observation the
        action was taken from, SB3's buffer obs), actions [cap,n,3], rewards
        [cap,n] f32, dones [cap,n] u8}; ``steps_done`` an int64 [n] tensor
        updated in place."""
        B = _lib.SalpRolloutBuffers()
        cap = 0
        if buffers:
            for k in ("obs", "obs_before", "actions", "rewards", "dones"):
                t = buffers.get(k)
                if t is not None:
                    if not t.is_contiguous() or t.device != self.device:
                        raise ValueError(f"buffer {k} must be contiguous on {self.device}")
                    if t.shape[1] != self.n_envs:
                        raise ValueError(f"buffer {k} must be [capacity, n_envs, ...]")
                    cap = t.shape[0] if cap == 0 else min(cap, t.shape[0])
                    setattr(B, k, t.data_ptr())
        B.capacity = cap
        if steps_done is not None:
            if steps_done.dtype != torch.int64 or steps_done.numel() != self.n_envs:
                raise ValueError("steps_done must be an int64 tensor with n_envs elements")
            B.steps_done = steps_done.data_ptr()
        B.max_steps = int(max_steps)
        B.chunk = int(chunk)
        self._run(_lib.load().salp_rollout(self._h, int(tick_budget), ctypes.byref(B), self._stream()))
        return steps_done

    def collect(self, weights, n_steps, buffers, episode_start, last_obs, ep_stats, diverged, noise_seed=0,
                gamma=0.99, diverged_obs_abs=0.0, diverged_reward_abs=0.0):
        """Policy-in-the-loop collection (salp_collect): every env runs
        ``n_steps`` env-steps back to back with actions drawn by the packed
        MlpPolicy ``weights`` (:func:`ppo.pack_policy`) at its env-step
        boundaries.  ``buffers``: dict of float32 [n_steps, n, ...] tensors
        obs, actions, rewards, episode_starts, values, log_probs (SB3's
        RolloutBuffer fields); ``episode_start`` [n] f32 in/out, ``last_obs``
        [n, obs_dim] in/out (in: the observation each env's first step is
        taken on, e.g. the one reset() returned), ``ep_stats`` [4] f64 (return, episodes,
        successes, length sums) and ``diverged`` [1] i64
        accumulated.  See include/salp.h for the exact semantics."""
        R = _lib.SalpPolicyRollout()
        w = weights
        if w.dtype != torch.float32 or w.numel() != POLICY_SIZE or not w.is_contiguous() or w.device != self.device:
            raise ValueError(f"weights must be a contiguous float32 [{POLICY_SIZE}] tensor on {self.device}")
        R.weights = w.data_ptr()
        shapes = {"obs": (n_steps, self.n_envs, self.obs_dim), "actions": (n_steps, self.n_envs, 3),
                  "rewards": (n_steps, self.n_envs), "episode_starts": (n_steps, self.n_envs),
                  "values": (n_steps, self.n_envs), "log_probs": (n_steps, self.n_envs)}
        for k, shp in shapes.items():
            t = buffers[k]
            if t.dtype != torch.float32 or tuple(t.shape) != shp or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"buffer {k} must be a contiguous float32 tensor of shape {shp} on {self.device}")
            setattr(R, k, t.data_ptr())
        for name, t, dt, shp in (("episode_start", episode_start, torch.float32, (self.n_envs,)),
                                 ("last_obs", last_obs, torch.float32, (self.n_envs, self.obs_dim)),
                                 ("ep_stats", ep_stats, torch.float64, (4,)),
                                 ("diverged", diverged, torch.int64, (1,))):
            if t.dtype != dt or tuple(t.shape) != shp or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"{name} must be a contiguous {dt} tensor of shape {shp} on {self.device}")
            setattr(R, name, t.data_ptr())
        R.n_steps = int(n_steps)
        R.noise_seed = int(noise_seed) & 0xFFFFFFFFFFFFFFFF
        R.gamma = float(gamma)
        R.diverged_obs_abs = float(diverged_obs_abs)
        R.diverged_reward_abs = float(diverged_reward_abs)
        self._run(_lib.load().salp_collect(self._h, ctypes.byref(R), self._stream()))

    # ------------------------------------------- Robot / Nozzle level
    # The reference's bare-robot call sequence (src/compare_trajectories.py:
    # 142-150): nozzle.set_yaw_angle + solve_angles, set_control,
    # step_through_cycle.  Arguments are per-env tensors; *_f32 says the
    # reference would hold an np.float32 there instead of a Python float.
    def _f64(self, x, shape):
        return torch.as_tensor(x, dtype=torch.float64, device=self.device).reshape(shape).contiguous()

    def robot_reset(self, mask=None):
        """Robot.reset() (src/robot.py:452-501) of every (or every masked) env."""
        m = self._mask(mask)
        self._run(_lib.load().salp_robot_reset(self._h, _ptr(m), self._stream()))

    def nozzle_set_angles(self, angles):
        """Nozzle.set_angles(angle1, angle2) (src/robot.py:50-60); angles [n, 2]."""
        a = self._f64(angles, (self.n_envs, 2))
        self._run(_lib.load().salp_nozzle_set_angles(self._h, _ptr(a), self._stream()))

    def nozzle_solve(self, yaw, yaw_f32=False):
        """Nozzle.set_yaw_angle(yaw) + Nozzle.solve_angles() (src/robot.py:62-98)."""
        y = self._f64(yaw, (self.n_envs,))
        self._run(_lib.load().salp_nozzle_solve(self._h, _ptr(y), int(bool(yaw_f32)), self._stream()))

    def robot_set_control(self, control, contraction_f32=False):
        """Robot.set_control(contraction, coast_time, [angle1, angle2])
        (src/robot.py:544-592); control [n, 4]."""
        c = self._f64(control, (self.n_envs, 4))
        self._run(_lib.load().salp_robot_set_control(self._h, _ptr(c), int(bool(contraction_f32)),
                                                       self._stream()))

    def robot_step_through_cycle(self):
        """Robot.step_through_cycle() (src/robot.py:740-777) of every env."""
        self._run(_lib.load().salp_robot_step_through_cycle(self._h, self._stream()))

    # --------------------------------------------------------- recording
    def enable_trace(self, max_samples):
        """Robot.enable_history_recording: from now on step() and
        robot_step_through_cycle() record per-tick samples of the last cycle
        (columns _abi.TRACE_COLUMNS) into device buffers; see :meth:`trace`."""
        rows = torch.full((int(max_samples), TRACE_DIM, self.n_envs), float("nan"), dtype=torch.float64,
                          device=self.device)
        ns = torch.zeros(self.n_envs, dtype=torch.int64, device=self.device)
        B = _lib.SalpTraceBuffer(int(max_samples), rows.data_ptr(), ns.data_ptr())
        self._check(_lib.load().salp_set_trace(self._h, ctypes.byref(B)))
        self._trace = (rows, ns)

    def disable_trace(self):
        self._check(_lib.load().salp_set_trace(self._h, None))
        self._trace = None

    def trace(self):
        """(rows [max_samples, TRACE_DIM, n] fp64, n_samples [n] int64) of the
        last recorded cycle; rows past n_samples are stale."""
        if self._trace is None:
            raise _lib.SalpError("recording is not enabled (enable_trace)")
        return self._trace

    # --------------------------------------------------- randomisation
    def set_randomization(self, dynamics=False, disturbances=False, actions=False, observations=False,
                          latency=False):
        """The reference's enable_* switches (Robot.enable_dynamic_randomization,
        enable_disturbances; SalpRobotEnv.enable_action_randomization,
        enable_observation_randomization, enable_latency) for this batch.  Draws
        come from the device Philox stream (salp_random.h)."""
        flags = [int(bool(x)) for x in (dynamics, disturbances, actions, observations, latency)]
        self._check(_lib.load().salp_set_randomization(self._h, *flags))
        (self.params.dynamics_randomization, self.params.disturbances, self.params.action_randomization,
         self.params.observation_randomization, self.params.latency) = flags

    # ------------------------------------------------------------ state
    def get_state(self):
        """[NUM_FIELDS, n] fp64 copy of the struct-of-arrays state."""
        s = torch.empty((NUM_FIELDS, self.n_envs), dtype=torch.float64, device=self.device)
        self._check(_lib.load().salp_get_state(self._h, _ptr(s), self._stream()))
        return s

    def set_state(self, state):
        s = torch.as_tensor(state, dtype=torch.float64, device=self.device).reshape(NUM_FIELDS, self.n_envs)
        s = s.contiguous()
        self._run(_lib.load().salp_set_state(self._h, _ptr(s), self._stream()))
        torch.cuda.current_stream(self.device).synchronize()

    def field(self, name):
        return self.get_state()[FIELD[name]]

    # ------------------------------------------------------------- info
    @staticmethod
    def info_dicts(info, dones=None):
        """Build reference-style info dicts (src/salp_robot_env.py:279-289) on the
        host — reward components always, episode metrics only where done."""
        info = info.detach().cpu().numpy()
        out = []
        for row in info:
            d = {k: float(row[INFO[k]]) for k in REWARD_COMPONENT_KEYS}
            if row[INFO["has_metrics"]] != 0:
                for k in EPISODE_METRIC_KEYS:
                    d[k] = float(row[INFO[k]])
            out.append(d)
        return out


FIELDS = FIELDS
INFO_KEYS = INFO_KEYS
