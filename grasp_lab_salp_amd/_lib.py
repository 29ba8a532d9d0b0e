"""ctypes binding of libsalp.so (the HIP/gfx950 build of include/salp.h).

The library is built in-tree (``python -m grasp_lab_salp_amd.build`` or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no CPU fallback: if the library or a GPU is missing, :func:`lib` raises.
"""
import ctypes
import os

from ._abi import ABI_VERSION, FIELDS, NUM_FIELDS, TRACE_DIM, SalpParams

HERE = os.path.dirname(os.path.abspath(__file__))
# SALP_LIB overrides the library path (A/B runs of alternative builds)
LIB_PATH = os.environ.get("SALP_LIB") or os.path.join(HERE, "libsalp.so")

_lib = None


class SalpError(RuntimeError):
    pass


class SalpRolloutBuffers(ctypes.Structure):
    _fields_ = [
        ("capacity", ctypes.c_int64),
        ("obs", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("rewards", ctypes.c_void_p),
        ("dones", ctypes.c_void_p),
        ("steps_done", ctypes.c_void_p),
        ("max_steps", ctypes.c_int64),
        ("chunk", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("obs_before", ctypes.c_void_p),
    ]


class SalpPolicyRollout(ctypes.Structure):
    _fields_ = [
        ("weights", ctypes.c_void_p),
        ("noise_seed", ctypes.c_uint64),
        ("gamma", ctypes.c_double),
        ("diverged_obs_abs", ctypes.c_double),
        ("diverged_reward_abs", ctypes.c_double),
        ("n_steps", ctypes.c_int64),
        ("obs", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("rewards", ctypes.c_void_p),
        ("episode_starts", ctypes.c_void_p),
        ("values", ctypes.c_void_p),
        ("log_probs", ctypes.c_void_p),
        ("episode_start", ctypes.c_void_p),
        ("last_obs", ctypes.c_void_p),
        ("ep_stats", ctypes.c_void_p),
        ("diverged", ctypes.c_void_p),
    ]


N_MLP_TENSORS = 13   # include/salp.h SALP_MLP_N_TENSORS


class SalpPpoMinibatch(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int64),
        ("obs_dim", ctypes.c_int32),
        ("normalize_advantage", ctypes.c_int32),
        ("idx", ctypes.c_void_p),
        ("obs", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("old_log_prob", ctypes.c_void_p),
        ("advantages", ctypes.c_void_p),
        ("returns", ctypes.c_void_p),
        ("params", ctypes.c_void_p * N_MLP_TENSORS),
        ("grads", ctypes.c_void_p),
        ("clip_range", ctypes.c_double),
        ("ent_coef", ctypes.c_double),
        ("vf_coef", ctypes.c_double),
        ("workspace", ctypes.c_void_p),
        ("stats", ctypes.c_void_p),
        ("adv_part", ctypes.c_void_p),
        ("norm_part", ctypes.c_void_p),
    ]


ADV_PARTIAL_DOUBLES = 512   # include/salp.h SALP_PPO_ADV_PARTIAL_DOUBLES
APPLY_WORKSPACE_DOUBLES = 256   # include/salp.h SALP_PPO_APPLY_WORKSPACE_DOUBLES


class SalpPpoAdam(ctypes.Structure):
    _fields_ = [
        ("obs_dim", ctypes.c_int32),
        ("norm_ready", ctypes.c_int32),
        ("params", ctypes.c_void_p * N_MLP_TENSORS),
        ("grads", ctypes.c_void_p),
        ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p),
        ("step", ctypes.c_void_p),
        ("grad_norm", ctypes.c_void_p),
        ("lr", ctypes.c_double),
        ("beta1", ctypes.c_double),
        ("beta2", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("max_grad_norm", ctypes.c_double),
        ("workspace", ctypes.c_void_p),
    ]


class SalpTraceBuffer(ctypes.Structure):
    _fields_ = [
        ("max_samples", ctypes.c_int64),
        ("rows", ctypes.c_void_p),
        ("n_samples", ctypes.c_void_p),
    ]


# name -> (restype, argtypes); exactly the functions declared in include/salp.h
_V, _H = ctypes.c_void_p, ctypes.c_void_p
SIGNATURES = {
    "salp_abi_version": (ctypes.c_int, []),
    "salp_default_params": (None, [ctypes.POINTER(SalpParams)]),
    "salp_create": (ctypes.c_int, [ctypes.POINTER(SalpParams), ctypes.c_int64, ctypes.c_uint64,
                                   ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "salp_destroy": (ctypes.c_int, [_H]),
    "salp_last_error": (ctypes.c_char_p, [_H]),
    "salp_num_envs": (ctypes.c_int64, [_H]),
    "salp_obs_dim": (ctypes.c_int, [_H]),
    "salp_reset": (ctypes.c_int, [_H, _V, _V, _V]),
    "salp_reset_to": (ctypes.c_int, [_H, _V, _V, _V, _V, _V, _V]),
    "salp_step": (ctypes.c_int, [_H, _V, _V, _V, _V, _V, ctypes.c_int, _V, _V, _V]),
    "salp_rollout": (ctypes.c_int, [_H, ctypes.c_int64, ctypes.POINTER(SalpRolloutBuffers), _V]),
    "salp_step_random": (ctypes.c_int, [_H, ctypes.c_int32, _V, _V]),
    "salp_collect": (ctypes.c_int, [_H, ctypes.POINTER(SalpPolicyRollout), _V]),
    "salp_lstm_cell_forward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, _V, _V, _V, _V, _V, _V, _V]),
    "salp_lstm_cell_backward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "salp_lstm_step_forward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    "salp_lstm_step_backward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [_V] * 11),
    "salp_set_lockstep_order": (ctypes.c_int, [_H, ctypes.c_int]),
    "salp_set_rollout_kernel": (ctypes.c_int, [_H, ctypes.c_int]),
    "salp_set_step_kernel": (ctypes.c_int, [_H, ctypes.c_int]),
    "salp_pair_timeouts": (ctypes.c_int, [_H, ctypes.POINTER(ctypes.c_uint64), _V]),
    "salp_robot_reset": (ctypes.c_int, [_H, _V, _V]),
    "salp_nozzle_set_angles": (ctypes.c_int, [_H, _V, _V]),
    "salp_nozzle_solve": (ctypes.c_int, [_H, _V, ctypes.c_int, _V]),
    "salp_robot_set_control": (ctypes.c_int, [_H, _V, ctypes.c_int, _V]),
    "salp_robot_step_through_cycle": (ctypes.c_int, [_H, _V]),
    "salp_set_trace": (ctypes.c_int, [_H, ctypes.POINTER(SalpTraceBuffer)]),
    "salp_set_randomization": (ctypes.c_int, [_H] + [ctypes.c_int] * 5),
    "salp_num_fields": (ctypes.c_int, []),
    "salp_field_name": (ctypes.c_char_p, [ctypes.c_int]),
    "salp_trace_dim": (ctypes.c_int, []),
    "salp_get_state": (ctypes.c_int, [_H, _V, _V]),
    "salp_set_state": (ctypes.c_int, [_H, _V, _V]),
    "salp_state_ptr": (ctypes.c_int64, [_H]),
    "salp_bench_ticks": (ctypes.c_int, [_H, ctypes.c_int32, _V]),
    "salp_math_selftest": (ctypes.c_int, [_V, _V, ctypes.c_int64, _V, _V]),
    "salp_gae": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, _V, _V, _V, _V, _V, ctypes.c_double,
                                ctypes.c_double, _V, _V, _V]),
    "salp_ppo_loss": (ctypes.c_int, [ctypes.c_int64, _V, _V, _V, _V, _V, _V, _V, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_int, _V, _V, _V, _V, _V]),
    "salp_ppo_mlp_num_params": (ctypes.c_int64, [ctypes.c_int]),
    "salp_ppo_mlp_offset": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int]),
    "salp_ppo_mlp_workspace_doubles": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int]),
    "salp_ppo_mlp_grads": (ctypes.c_int, [ctypes.POINTER(SalpPpoMinibatch), _V]),
    "salp_ppo_mlp_apply": (ctypes.c_int, [ctypes.POINTER(SalpPpoAdam), _V]),
    "salp_ppo_mlp_adv_partials": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, _V, _V, _V, _V]),
}


def load(path=LIB_PATH):
    """Load and type the shared library (no GPU needed for loading)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SalpError(f"{path} not found: build it with `python -m grasp_lab_salp_amd.build` "
                        "(there is no CPU fallback for the simulator)")
    L = ctypes.CDLL(path)
    # SALP_AB_OLD_ABI=1: an A/B run (tools/gpu_*_ab.sh) against a library of an
    # earlier round -- its older ABI number passes and its missing newer entry
    # points stay unbound.  Only for an explicit SALP_LIB other than the
    # in-tree build, never silently: it warns, and the PPO paths that need a
    # newer entry point are switched to their older equivalents (a library
    # without salp_ppo_mlp_adv_partials gets SALP_PPO_EPOCH_ADV=0).  The state
    # and trace layouts must still match.
    old_ok = (os.environ.get("SALP_AB_OLD_ABI") == "1" and bool(os.environ.get("SALP_LIB"))
              and os.path.abspath(path) != os.path.join(HERE, "libsalp.so"))
    if os.environ.get("SALP_AB_OLD_ABI") == "1" and not old_ok:
        raise SalpError("SALP_AB_OLD_ABI=1 is for A/B runs of another library: set SALP_LIB to it")
    missing = []
    for name, (res, args) in SIGNATURES.items():
        if old_ok and not hasattr(L, name):
            missing.append(name)
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if old_ok:
        import warnings
        warnings.warn(f"SALP_AB_OLD_ABI=1: {path} loaded without the ABI check (ABI "
                      f"{L.salp_abi_version()} vs {ABI_VERSION}; unbound: {missing or 'none'}) -- A/B use only",
                      RuntimeWarning, stacklevel=2)
        if "salp_ppo_mlp_adv_partials" in missing:
            os.environ["SALP_PPO_EPOCH_ADV"] = "0"
    if L.salp_abi_version() != ABI_VERSION and not old_ok:
        raise SalpError("libsalp ABI version mismatch")
    if L.salp_num_fields() != NUM_FIELDS:
        raise SalpError("libsalp state layout does not match grasp_lab_salp_amd._abi")
    if L.salp_trace_dim() != TRACE_DIM:
        raise SalpError("libsalp trace layout does not match grasp_lab_salp_amd._abi")
    for i, name in enumerate(FIELDS):
        if L.salp_field_name(i).decode() != name:
            raise SalpError(f"field {i}: library says {L.salp_field_name(i)!r}, _abi says {name!r}")
    _lib = L
    return L


def check(rc, handle=None):
    if rc != 0:
        msg = load().salp_last_error(handle)
        raise SalpError(f"libsalp error {rc}: {msg.decode() if msg else ''}")
    return rc
