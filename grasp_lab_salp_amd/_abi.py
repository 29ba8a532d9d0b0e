"""Python mirror of the C ABI in include/salp.h (struct layout, field ids).

Kept as the single Python-side description of the boundary; tests check it
against the names exported by libsalp.so (salp_field_name) so the two cannot
drift apart silently.
"""
import ctypes

ABI_VERSION = 13
# rows of salp_math_selftest's output (include/salp.h)
MATH_SELFTEST_ROWS = 23
MAX_OBSTACLES = 4
OBS_DIM_MAX = 6 + 2 * MAX_OBSTACLES

# salp_collect's packed policy (include/salp.h SALP_POLICY_*), offsets in floats
POLICY_HIDDEN = 64
POLICY_OFFSETS = {}
_off = 0
for _name, _size in (("pi_w1", POLICY_HIDDEN * OBS_DIM_MAX), ("pi_b1", POLICY_HIDDEN),
                     ("pi_w2", POLICY_HIDDEN * POLICY_HIDDEN), ("pi_b2", POLICY_HIDDEN),
                     ("act_w", 3 * POLICY_HIDDEN), ("act_b", 3), ("log_std", 3),
                     ("vf_w1", POLICY_HIDDEN * OBS_DIM_MAX), ("vf_b1", POLICY_HIDDEN),
                     ("vf_w2", POLICY_HIDDEN * POLICY_HIDDEN), ("vf_b2", POLICY_HIDDEN),
                     ("val_w", POLICY_HIDDEN), ("val_b", 1)):
    POLICY_OFFSETS[_name] = (_off, _size)
    _off += _size
POLICY_SIZE = _off


class SalpParams(ctypes.Structure):
    """Constructor arguments of Nozzle / Robot / SalpRobotEnv (include/salp.h)."""

    _fields_ = [
        ("nozzle_length1", ctypes.c_double),
        ("nozzle_length2", ctypes.c_double),
        ("nozzle_length3", ctypes.c_double),
        ("nozzle_area", ctypes.c_double),
        ("nozzle_mass", ctypes.c_double),
        ("dry_mass", ctypes.c_double),
        ("init_length", ctypes.c_double),
        ("init_width", ctypes.c_double),
        ("max_contraction", ctypes.c_double),
        ("density", ctypes.c_double),
        ("init_angle1", ctypes.c_double),
        ("init_angle2", ctypes.c_double),
        ("obstacle_radius", ctypes.c_double),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("num_obstacles", ctypes.c_int32),
        ("max_cycles", ctypes.c_int32),
        # randomisation switches (include/salp.h): all off in the reference scripts
        ("dynamics_randomization", ctypes.c_int32),
        ("disturbances", ctypes.c_int32),
        ("action_randomization", ctypes.c_int32),
        ("observation_randomization", ctypes.c_int32),
        ("latency", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def default_params(**overrides):
    """Canonical configuration of src/train_robot.py:11-21 (make_env)."""
    p = SalpParams(
        nozzle_length1=0.05, nozzle_length2=0.05, nozzle_length3=0.05, nozzle_area=0.00016,
        nozzle_mass=1.0, dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06,
        density=1000.0, init_angle1=0.0, init_angle2=0.0, obstacle_radius=0.2, width=900,
        height=700, num_obstacles=2, max_cycles=500)
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown SalpParams field {k!r}")
        setattr(p, k, v)
    return p


def _vec(name):
    return [f"{name}{i}" for i in range(3)]


# Order == enum SalpField in include/salp.h
FIELDS = (
    _vec("v") + _vec("w") + _vec("acc") + _vec("alpha") + _vec("eta") + _vec("pw") + _vec("pos")
    + _vec("ang") + _vec("ppos") + _vec("pang") + _vec("avgv") + _vec("avgw")
    + ["length", "width", "volume", "prev_volume", "com", "com_rate", "com_acc"]
    + _vec("prev_I") + ["geom32", "pvol32"]
    + ["cycle_time", "time", "refill_time", "jet_time", "coast_time", "contraction",
       "contract_rate", "release_rate", "phase", "cycle", "contr32"]
    + ["angle1", "angle2", "prev_angle1", "prev_angle2", "yaw", "prev_yaw", "turn_time"]
    + ["target0", "target1"] + [f"obst{i}" for i in range(2 * MAX_OBSTACLES)]
    + ["n_obst", "prev_dist", "prev_a2"]
    + ["ep_len", "ep_return", "path_len", "last_px", "last_py", "sum_a0", "sum_a1", "sum_abs_a2",
       "sum_vel", "init_dist"] + [f"sum_r{i}" for i in range(7)]
    + ["act0", "act1", "act2", "pending", "step_count", "episode"]
    + ["cd", "dfr", "dtr"] + [f"amf{i}" for i in range(3)] + [f"amrf{i}" for i in range(3)]
    + [f"amt{i}" for i in range(3)] + [f"amrt{i}" for i in range(3)]
    + [f"ouf{i}" for i in range(3)] + [f"out{i}" for i in range(3)] + ["rng_ctl", "rng_tick"]
)
NUM_FIELDS = len(FIELDS)
FIELD = {name: i for i, name in enumerate(FIELDS)}

INFO_KEYS = (
    "rewards/track", "rewards/heading", "rewards/smooth", "rewards/yaw", "rewards/time",
    "rewards/sideslip", "rewards/obstacle",
    "path_length", "direct_distance", "path_efficiency", "final_distance", "initial_distance",
    "avg_compression", "avg_coast_time", "avg_nozzle_angle", "avg_velocity",
    "avg_rewards_track", "avg_rewards_heading", "avg_rewards_smooth", "avg_rewards_yaw",
    "avg_rewards_time", "avg_rewards_sideslip", "avg_rewards_obstacle",
    "ep_return", "ep_len", "has_metrics", "hit_obstacle",
)
INFO_DIM = len(INFO_KEYS)
INFO = {k: i for i, k in enumerate(INFO_KEYS)}
REWARD_COMPONENT_KEYS = INFO_KEYS[:7]
EPISODE_METRIC_KEYS = INFO_KEYS[7:23]

PHASES = ("REFILL", "JET", "COAST", "REST")  # src/robot.py:252-257

# Columns of a trace sample (enum SalpTraceCol in include/salp.h); names are
# the reference's *_history attributes (src/robot.py:687-738) without the
# suffix, vectors split per component.
TRACE_COLUMNS = (
    ["state"] + _vec("position_world") + _vec("velocity") + _vec("acceleration")
    + _vec("euler_angle") + _vec("euler_angle_rate") + _vec("angular_velocity")
    + _vec("angular_acceleration") + ["length", "width"] + _vec("area")
    + ["volume", "mass", "mass_rate", "nozzle_yaw"] + _vec("inertia_tensor")
    + _vec("trans_drag_coefficient") + _vec("rot_drag_coefficient")
    + ["center_of_mass", "center_of_mass_rate", "center_of_mass_acc_rate"]
    + _vec("position_front_world")
    + _vec("jet_velocity") + _vec("jet_force") + _vec("jet_torque") + _vec("drag_force")
    + _vec("drag_torque") + _vec("coriolis_force") + _vec("coriolis_torque")
    + _vec("added_mass_force") + _vec("added_mass_torque") + _vec("deform_torque")
    + _vec("acceleration_force")
)
TRACE_DIM = len(TRACE_COLUMNS)
TRACE = {k: i for i, k in enumerate(TRACE_COLUMNS)}
TRACE_FIRST_FORCE = TRACE["jet_velocity0"]
# history name -> (first column, width) ; width 1 = scalar history
TRACE_HISTORIES = {}
for _i, _k in enumerate(TRACE_COLUMNS):
    _base = _k[:-1] if _k[-1] in "012" and _k[:-1] + "1" in TRACE else _k
    if _base not in TRACE_HISTORIES:
        TRACE_HISTORIES[_base] = (_i, 3 if _base != _k else 1)
