"""SB3-shaped vectorised env over one batched device simulator.

The reference trains through Stable-Baselines3's ``make_vec_env(make_env,
n_envs, vec_env_cls=SubprocVecEnv|DummyVecEnv)`` (src/train_robot.py:26,
src/train_robot_recurrent_ppo.py:65), i.e. one Python env object per env,
stepped in worker processes and wrapped in ``Monitor``.  Here all envs live in
one :class:`BatchedSalpEnv` and one ``step`` is one kernel launch.  The
VecEnv semantics the learners and callbacks rely on are reproduced:

* ``step_async`` / ``step_wait`` -> ``(obs [n, obs_dim] f32, rewards [n] f32,
  dones [n] bool, infos)``, auto-reset of finished envs with the final
  observation in ``info["terminal_observation"]`` and
  ``info["TimeLimit.truncated"] = truncated and not terminated``;
* Monitor's ``info["episode"] = {"r", "l", "t"}`` on the step that ends an
  episode (return includes the terminal bonuses), plus the env's reward
  components on every step and its episode metrics on the last step
  (src/salp_robot_env.py:279-289, read by src/tensorboard_callback.py:70-123).

stable_baselines3 is not installed in this image, so those semantics are
restated from its documented behaviour and are not pinned by a reference
test ("parity unpinned").  When stable_baselines3 is importable
the class derives from its ``VecEnv``.

Differences from a list of reference envs, by design: targets / obstacles
come from the device's Philox stream keyed by (seed, env id, episode) instead
of the process-global ``np.random`` (SURVEY.md §7 hard part 7); when
obstacle placement fails the observation keeps its length with zeros in the
missing slots (the reference returns a shorter vector).

For throughput, :meth:`SalpVecEnv.step_tensors` returns device tensors and
builds no Python dicts.
"""
import time

import numpy as np
import torch

from ._abi import EPISODE_METRIC_KEYS, INFO, REWARD_COMPONENT_KEYS, SalpParams, default_params
from .batched_env import BatchedSalpEnv
from .spaces import Box

try:  # pragma: no cover - depends on the environment
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase
except ImportError:  # pragma: no cover
    class _VecEnvBase:
        """The parts of stable_baselines3.common.vec_env.VecEnv used here."""

        def __init__(self, num_envs, observation_space, action_space):
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space
            self.reset_infos = [{} for _ in range(num_envs)]
            self.render_mode = None

        def step(self, actions):
            self.step_async(actions)
            return self.step_wait()

        @property
        def unwrapped(self):
            return self

__all__ = ["SalpVecEnv", "make_vec_env"]


class SalpVecEnv(_VecEnvBase):
    """``num_envs`` SalpRobotEnv's stepped together on one GPU."""

    metadata = {"render_modes": []}

    def __init__(self, num_envs, params=None, seed=0, device=None, env_id_offset=0, infos=True):
        params = params if params is not None else default_params()
        if not isinstance(params, SalpParams):
            raise TypeError("params must be a SalpParams")
        self.sim = BatchedSalpEnv(num_envs, params=params, seed=seed, env_id_offset=env_id_offset,
                                  device=device)
        od = self.sim.obs_dim
        obs_space = Box(low=np.full(od, -np.inf, dtype=np.float32), high=np.full(od, np.inf, dtype=np.float32),
                        dtype=np.float32)
        act_space = Box(low=np.array([0.0, 0.0, -1.0]), high=np.array([1.0, 1.0, 1.0]), dtype=np.float32)
        super().__init__(num_envs, obs_space, act_space)
        self.build_infos = bool(infos)
        self._actions = None
        self._t0 = time.time()

    # ------------------------------------------------------------- VecEnv
    def reset(self):
        obs = self.sim.reset()
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_tensors(self, actions):
        """One env-step of every env, auto-reset, all outputs on the device
        (:class:`~grasp_lab_salp_amd.batched_env.StepResult`)."""
        return self.sim.step(actions, auto_reset=True, want_terminal_obs=True)

    def step_wait(self):
        a = self._actions
        if not torch.is_tensor(a):
            a = torch.as_tensor(np.asarray(a, np.float32))
        r = self.step_tensors(a)
        obs = r.obs.cpu().numpy()
        rew = r.reward.float().cpu().numpy()
        term = r.terminated.cpu().numpy()
        trunc = r.truncated.cpu().numpy()
        dones = term | trunc
        infos = self._infos(r, term, trunc, dones) if self.build_infos else [{} for _ in range(self.num_envs)]
        return obs, rew, dones, infos

    def _infos(self, r, term, trunc, dones):
        info = r.info.cpu().numpy()
        comp = info[:, [INFO[k] for k in REWARD_COMPONENT_KEYS]].tolist()
        out = [dict(zip(REWARD_COMPONENT_KEYS, c)) for c in comp]
        idx = np.nonzero(dones)[0]
        if len(idx):
            tobs = r.terminal_obs[torch.as_tensor(idx, device=r.terminal_obs.device)].cpu().numpy()
            t = round(time.time() - self._t0, 6)
            for j, i in enumerate(idx):
                row = info[i]
                d = out[i]
                d["terminal_observation"] = tobs[j]
                d["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                d["episode"] = {"r": round(float(row[INFO["ep_return"]]), 6),
                                "l": int(row[INFO["ep_len"]]), "t": t}
                d.update({k: float(row[INFO[k]]) for k in EPISODE_METRIC_KEYS})
        return out

    def close(self):
        self.sim.close()

    def seed(self, seed=None):
        """Re-key the device RNG (targets, obstacles, synthetic actions)."""
        if seed is None:
            return [None] * self.num_envs
        p = self.sim.params
        self.sim.close()
        self.sim = BatchedSalpEnv(self.num_envs, params=p, seed=int(seed),
                                  env_id_offset=self.sim.env_id_offset, device=self.sim.device.index)
        return [int(seed) + i for i in range(self.num_envs)]

    def get_attr(self, attr_name, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        v = getattr(self, attr_name)
        return [v for _ in idx]

    def set_attr(self, attr_name, value, indices=None):
        setattr(self, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        idx = range(self.num_envs) if indices is None else indices
        return [getattr(self, method_name)(*args, **kwargs) for _ in idx]

    def env_is_wrapped(self, wrapper_class, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        return [False for _ in idx]

    def get_images(self):
        raise NotImplementedError("rendering is out of scope")


def make_vec_env(env_id, n_envs=1, seed=None, vec_env_cls=None, **kwargs):
    """Stand-in for SB3's ``make_vec_env`` with the reference's ``make_env``:
    calls ``env_id()`` once to read the robot / env configuration it builds,
    then returns one :class:`SalpVecEnv` of ``n_envs`` envs (``vec_env_cls`` is
    accepted and ignored: all envs share one kernel launch)."""
    if not callable(env_id):
        raise TypeError("env_id must be the reference-style make_env callable")
    env = env_id()
    try:
        params = env.robot.salp_params(width=int(env.width), height=int(env.height),
                                       num_obstacles=int(env.num_obstacles),
                                       obstacle_radius=float(env.obstacle_radius))
    finally:
        env.close()
    return SalpVecEnv(n_envs, params=params, seed=0 if seed is None else seed)
