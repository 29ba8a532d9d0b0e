"""ctypes wrapper of the CPU oracle (oracle/libsalp_oracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See
oracle/salp_oracle.c for what is restated and where it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

from grasp_lab_salp_amd._abi import (INFO_DIM, MATH_SELFTEST_ROWS, MAX_OBSTACLES, NUM_FIELDS, OBS_DIM_MAX,
                                     TRACE_DIM, SalpParams, default_params)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsalp_oracle.so")
# the same restatement with NumPy's unfused product-sums (SALP_FMA=0,
# salp_math.h); libsalp.so and LIB_PATH are built with SALP_FMA=1
EXACT_LIB_PATH = os.path.join(HERE, "libsalp_oracle_exact.so")

_libs = {}


SOURCES = [os.path.join(HERE, "salp_oracle.c"), os.path.join(HERE, "..", "include", "salp.h")] + [
    os.path.join(HERE, "..", "grasp_lab_salp_amd", "csrc", f) for f in ("salp_math.h", "salp_philox.h",
                                                                          "salp_random.h")]


def build(force=False):
    stale = any(not os.path.exists(p) or any(os.path.getmtime(s) > os.path.getmtime(p) for s in SOURCES)
                for p in (LIB_PATH, EXACT_LIB_PATH))
    if force or stale:
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib(exact=False):
    """The oracle library: the product's arithmetic mode, or (exact) NumPy's
    unfused products and sums."""
    if exact not in _libs:
        build()
        L = ctypes.CDLL(EXACT_LIB_PATH if exact else LIB_PATH)
        P = ctypes.POINTER
        d, f, u8, i32, i64, u32 = (ctypes.c_double, ctypes.c_float, ctypes.c_uint8,
                                   ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32)
        sp = P(SalpParams)
        L.oracle_num_fields.restype = ctypes.c_int
        L.oracle_init.argtypes = [sp, i64, P(d)]
        L.oracle_reset_to.argtypes = [sp, i64, P(d), P(u8), P(f), P(f), P(i32), P(f), ctypes.c_int]
        L.oracle_reset.argtypes = [sp, i64, P(d), P(u8), ctypes.c_uint64, i64, P(f), ctypes.c_int]
        L.oracle_step.argtypes = [sp, i64, P(d), P(f), P(f), P(d), P(u8), P(u8), ctypes.c_int,
                                  P(f), P(d), P(i64), ctypes.c_uint64, i64, ctypes.c_int]
        L.oracle_step_random.argtypes = [sp, i64, P(d), i32, ctypes.c_uint64, i64, P(d),
                                         ctypes.c_int]
        L.oracle_step_random.restype = i64
        L.oracle_replay.argtypes = [sp, i64, P(i64), P(i64), P(d), ctypes.c_uint64, P(d), i64, P(f), P(f),
                                    P(f), P(f), P(u8), ctypes.c_int, ctypes.c_int, P(i64)]
        L.oracle_replay.restype = i64
        L.oracle_robot_trace.argtypes = [sp, P(f), ctypes.c_int, P(d), i64]
        L.oracle_robot_trace.restype = i64
        L.oracle_math_selftest.argtypes = [P(d), P(d), i64, P(d)]
        L.oracle_robot_reset.argtypes = [sp, i64, P(d), P(u8)]
        L.oracle_nozzle_set_angles.argtypes = [sp, i64, P(d), P(d)]
        L.oracle_nozzle_solve.argtypes = [sp, i64, P(d), P(d), ctypes.c_int]
        L.oracle_robot_set_control.argtypes = [sp, i64, P(d), P(d), ctypes.c_int, ctypes.c_uint64, i64]
        L.oracle_robot_cycle.argtypes = [sp, i64, P(d), P(d), i64, P(i64), P(i64), ctypes.c_uint64, i64]
        L.oracle_philox.argtypes = [u32] * 6 + [P(u32)]
        if L.oracle_num_fields() != NUM_FIELDS:
            raise RuntimeError("oracle / _abi field count mismatch")
        _libs[exact] = L
    return _libs[exact]


def _p(a, ct):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ct))


class Oracle:
    """Batch of reference-equivalent envs on the CPU; state is [NUM_FIELDS, n]."""

    def __init__(self, params=None, n_envs=1, seed=0, env_offset=0, exact=False):
        self._L = lib(exact)
        self.params = params if params is not None else default_params()
        self.n = int(n_envs)
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.obs_dim = 6 + 2 * self.params.num_obstacles
        self.state = np.zeros((NUM_FIELDS, self.n), np.float64)
        self._L.oracle_init(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double))

    def _mask(self, mask):
        if mask is None:
            return None
        return np.ascontiguousarray(mask, dtype=np.uint8)

    def reset(self, mask=None):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        m = self._mask(mask)
        self._L.oracle_reset(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                           _p(m, ctypes.c_uint8), self.seed, self.env_offset,
                           _p(obs, ctypes.c_float), self.obs_dim)
        return obs

    def reset_to(self, targets, obstacles, n_obstacles, mask=None):
        t = np.ascontiguousarray(targets, np.float32).reshape(self.n, 2)
        o = np.zeros((self.n, MAX_OBSTACLES, 2), np.float32)
        ob = np.asarray(obstacles, np.float32).reshape(self.n, -1, 2)
        o[:, :ob.shape[1]] = ob
        k = np.ascontiguousarray(n_obstacles, np.int32).reshape(self.n)
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        m = self._mask(mask)
        self._L.oracle_reset_to(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                              _p(m, ctypes.c_uint8), _p(t, ctypes.c_float), _p(o, ctypes.c_float),
                              _p(k, ctypes.c_int32), _p(obs, ctypes.c_float), self.obs_dim)
        return obs

    def step(self, actions, auto_reset=False):
        a = np.ascontiguousarray(actions, np.float32).reshape(self.n, 3)
        out = dict(obs=np.zeros((self.n, self.obs_dim), np.float32),
                   reward=np.zeros(self.n, np.float64),
                   terminated=np.zeros(self.n, np.uint8), truncated=np.zeros(self.n, np.uint8),
                   terminal_obs=np.zeros((self.n, self.obs_dim), np.float32),
                   info=np.zeros((self.n, INFO_DIM), np.float64),
                   ticks=np.zeros(self.n, np.int64))
        self._L.oracle_step(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                          _p(a, ctypes.c_float), _p(out["obs"], ctypes.c_float),
                          _p(out["reward"], ctypes.c_double), _p(out["terminated"], ctypes.c_uint8),
                          _p(out["truncated"], ctypes.c_uint8), int(bool(auto_reset)),
                          _p(out["terminal_obs"], ctypes.c_float), _p(out["info"], ctypes.c_double),
                          _p(out["ticks"], ctypes.c_int64), self.seed, self.env_offset,
                          self.obs_dim)
        return out

    # ---- Robot / Nozzle level (salp_robot_*, salp_nozzle_* of include/salp.h)
    def robot_reset(self, mask=None):
        self._L.oracle_robot_reset(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                                 _p(self._mask(mask), ctypes.c_uint8))

    def nozzle_set_angles(self, angles):
        a = np.ascontiguousarray(angles, np.float64).reshape(self.n, 2)
        self._L.oracle_nozzle_set_angles(ctypes.byref(self.params), self.n,
                                       _p(self.state, ctypes.c_double), _p(a, ctypes.c_double))

    def nozzle_solve(self, yaw, yaw_f32):
        y = np.ascontiguousarray(yaw, np.float64).reshape(self.n)
        self._L.oracle_nozzle_solve(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                                  _p(y, ctypes.c_double), int(bool(yaw_f32)))

    def robot_set_control(self, control, contraction_f32):
        c = np.ascontiguousarray(control, np.float64).reshape(self.n, 4)
        self._L.oracle_robot_set_control(ctypes.byref(self.params), self.n,
                                       _p(self.state, ctypes.c_double), _p(c, ctypes.c_double),
                                       int(bool(contraction_f32)), self.seed, self.env_offset)

    def robot_cycle(self, max_samples=0):
        """step_through_cycle; returns (ticks [n], rows [max_samples, DIM, n] or
        None, n_samples [n] or None)."""
        ticks = np.zeros(self.n, np.int64)
        rows = ns = None
        if max_samples > 0:
            rows = np.full((max_samples, TRACE_DIM, self.n), np.nan)
            ns = np.zeros(self.n, np.int64)
        self._L.oracle_robot_cycle(ctypes.byref(self.params), self.n, _p(self.state, ctypes.c_double),
                                 _p(rows, ctypes.c_double), int(max_samples),
                                 _p(ns, ctypes.c_int64), _p(ticks, ctypes.c_int64), self.seed,
                                 self.env_offset)
        return ticks, rows, ns

    def set_randomization(self, dynamics=False, disturbances=False, actions=False, observations=False,
                          latency=False):
        """The reference's enable_* switches (include/salp.h SalpParams).
        Switching a feature off restores the reference's defaults (mean
        coefficients, calm OU processes), as salp_set_randomization does."""
        from grasp_lab_salp_amd._abi import FIELD
        if self.params.dynamics_randomization and not dynamics:
            means = {"cd": 0.3, "dfr": 0.25, "dtr": 0.1, "amf0": 0.5, "amf1": 0.6, "amf2": 0.6,
                     "amt0": 0.3, "amt1": 0.6, "amt2": 0.6}
            for j in range(3):
                means[f"amrf{j}"] = 0.2
                means[f"amrt{j}"] = 0.2
            for k, v in means.items():
                self.state[FIELD[k]] = v
        if self.params.disturbances and not disturbances:
            for j in range(3):
                self.state[FIELD[f"ouf{j}"]] = 0.0
                self.state[FIELD[f"out{j}"]] = 0.0
        p = SalpParams.from_buffer_copy(self.params)
        p.dynamics_randomization, p.disturbances = int(bool(dynamics)), int(bool(disturbances))
        p.action_randomization, p.observation_randomization = int(bool(actions)), int(bool(observations))
        p.latency = int(bool(latency))
        self.params = p

    def step_random(self, n_steps, threads=0):
        rs = np.zeros(self.n, np.float64)
        ticks = self._L.oracle_step_random(ctypes.byref(self.params), self.n,
                                         _p(self.state, ctypes.c_double), int(n_steps), self.seed,
                                         self.env_offset, _p(rs, ctypes.c_double), int(threads))
        return rs, int(ticks)


def replay(env_ids, n_steps, ct_stop=None, seed=0, params=None, capacity=0, threads=0, exact=False,
           ticks_out=None):
    """Sampled envs of a chained random-action rollout (oracle_replay): env j,
    global id env_ids[j], from creation through n_steps[j] env-steps, then the
    in-flight cycle up to cycle_time ct_stop[j] (< 0: none).  Returns (state
    [NUM_FIELDS, n], buffers {obs, obs_before, actions, rewards, dones} with
    `capacity` slots (slot = step % capacity, the last `capacity` steps).
    ticks_out (int64 [n], optional) receives the physics ticks of each env's
    n_steps[j] completed env-steps (src/robot.py:756-757 loop iterations; the
    in-flight cycle is not counted)."""
    params = params if params is not None else default_params()
    ids = np.ascontiguousarray(env_ids, np.int64)
    n = len(ids)
    ks = np.ascontiguousarray(n_steps, np.int64).reshape(n)
    ct = None if ct_stop is None else np.ascontiguousarray(ct_stop, np.float64).reshape(n)
    od = 6 + 2 * params.num_obstacles
    state = np.zeros((NUM_FIELDS, n), np.float64)
    cap = int(capacity)
    b = {"obs": np.full((max(cap, 1), n, od), np.nan, np.float32),
         "obs_before": np.full((max(cap, 1), n, od), np.nan, np.float32),
         "actions": np.full((max(cap, 1), n, 3), np.nan, np.float32),
         "rewards": np.full((max(cap, 1), n), np.nan, np.float32),
         "dones": np.full((max(cap, 1), n), 255, np.uint8)}
    lib(exact).oracle_replay(ctypes.byref(params), n, _p(ids, ctypes.c_int64), _p(ks, ctypes.c_int64),
                        _p(ct, ctypes.c_double), int(seed), _p(state, ctypes.c_double), cap,
                        _p(b["obs"], ctypes.c_float), _p(b["obs_before"], ctypes.c_float),
                        _p(b["actions"], ctypes.c_float), _p(b["rewards"], ctypes.c_float),
                        _p(b["dones"], ctypes.c_uint8), od, int(threads),
                        None if ticks_out is None else _p(ticks_out, ctypes.c_int64))
    return state, (b if cap > 0 else None)


def robot_trace(actions, params=None, max_rows=200000, exact=False):
    params = params if params is not None else default_params()
    a = np.ascontiguousarray(actions, np.float32).reshape(-1, 3)
    out = np.zeros((max_rows, 29), np.float64)
    n = lib(exact).oracle_robot_trace(ctypes.byref(params), _p(a, ctypes.c_float), len(a),
                                 _p(out, ctypes.c_double), max_rows)
    if n < 0:
        raise RuntimeError("trace buffer too small")
    return out[:n]


def math_selftest(x, y, exact=False):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros((MATH_SELFTEST_ROWS, len(x)), np.float64)
    lib(exact).oracle_math_selftest(_p(x, ctypes.c_double), _p(y, ctypes.c_double), len(x),
                               _p(out, ctypes.c_double))
    return out


def philox(ctr, key):
    out = (ctypes.c_uint32 * 4)()
    lib().oracle_philox(*[int(c) & 0xFFFFFFFF for c in ctr], *[int(k) & 0xFFFFFFFF for k in key],
                        out)
    return [int(v) for v in out]
