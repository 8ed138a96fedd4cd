"""ctypes binding of libdxrl.so (the C ABI declared in include/dxrl.h).

The library is built in-tree by ``build.build_native()`` (hipcc, gfx950) and
loaded here.  There is no fallback: if the library is missing or no GPU is
visible, every product entry point raises.  torch is imported first so the
library binds to the HIP runtime torch already loaded (one runtime per
process; streams and device pointers are shared).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (loads libamdhip64 first; see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DXRL_LIB") or os.path.join(PKG_DIR, "libdxrl.so")  # DXRL_LIB: A/B builds

DXRL_OK = 0
DXRL_E_INVALID = -1
DXRL_E_HIP = -2
DXRL_E_UNSUPPORTED = -3
DXRL_E_TAPE = -4
REWARD_SPARSE = 0
REWARD_DENSE = 1
RESET_EXTRA = 6
MAX_CURRICULA = 256
SUCCESS_TRAINING = 0
SUCCESS_TERMINATED = 1
ABI_VERSION = 1
EVAL_POLICY_SIMPLE = 0
EVAL_POLICY_HEURISTIC = 1
EVAL_POLICY_RANDOM = 2


class Curriculum(C.Structure):
    _fields_ = [("object_size", C.c_double), ("object_mass", C.c_double), ("friction_coefficient", C.c_double),
                ("size_range", C.c_double * 2), ("mass_range", C.c_double * 2), ("friction_range", C.c_double * 2),
                ("spawn_x_range", C.c_double * 2), ("spawn_y_range", C.c_double * 2),
                ("spawn_z_range", C.c_double * 2),
                ("has_size_range", C.c_int32), ("has_mass_range", C.c_int32), ("has_friction_range", C.c_int32),
                ("friction_is_f64_scalar", C.c_int32)]


class EnvConfig(C.Structure):
    _fields_ = [("num_envs", C.c_int32), ("num_fingers", C.c_int32), ("joints_per_finger", C.c_int32),
                ("max_episode_steps", C.c_int32), ("reward_type", C.c_int32), ("has_object_position", C.c_int32),
                ("object_position", C.c_double * 3),
                ("distance_weight", C.c_double), ("contact_weight", C.c_double), ("closure_weight", C.c_double),
                ("stability_weight", C.c_double), ("seed", C.c_uint64), ("global_env_offset", C.c_int64)]


class EnvLayout(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("total_bytes", "jp", "jv", "op", "ov", "flags", "step_count", "size",
                                         "mass", "friction", "cfg_index", "reset_ctr", "curricula")]


class LearnerLayout(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("total_bytes", "mean", "best", "ep_return", "noise_ctr")]


class LearnerConfig(C.Structure):
    _fields_ = [("learning_rate", C.c_double), ("exploration_noise", C.c_double),
                ("action_clip_range", C.c_double), ("seed", C.c_uint64)]


class RolloutIO(C.Structure):
    _fields_ = [("gauss", C.c_void_p), ("gauss_stride", C.c_int64), ("reset_draws", C.c_void_p),
                ("reset_stride", C.c_int64), ("record_cap", C.c_int32), ("ep_return", C.c_void_p),
                ("ep_length", C.c_void_p), ("ep_success", C.c_void_p), ("ep_end_step", C.c_void_p),
                ("ep_count", C.c_void_p), ("gauss_used", C.c_void_p), ("status", C.c_void_p),
                ("episode_budget", C.c_void_p)]


class PgRolloutArgs(C.Structure):
    _fields_ = [("horizon", C.c_int32), ("max_steps", C.c_int32), ("policy_seed", C.c_uint64),
                ("iteration", C.c_uint64), ("obs_noise_std", C.c_double), ("dyn_noise_std", C.c_double)] + \
               [(k, C.c_void_p) for k in ("obs_rm", "obs_fm", "act", "logp", "rew", "done", "ep_return", "ep_count",
                                          "ep_sum_return", "ep_sum_length", "ep_successes")] + \
               [("diag_flags", C.c_int32), ("success_rule", C.c_int32), ("record_cap", C.c_int32),
                ("rec_return", C.c_void_p), ("rec_length", C.c_void_p), ("rec_success", C.c_void_p),
                ("rec_end_step", C.c_void_p), ("ep_code", C.c_void_p), ("applied_act", C.c_void_p),
                ("dyn_noise_tape", C.c_void_p), ("obs_noise_tape", C.c_void_p), ("h2_tape", C.c_void_p)]


class PgHeadsArgs(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("mu", "values", "act", "logp_old", "adv", "ret", "stats", "params")] + \
               [("num_samples", C.c_int64), ("inv_total_samples", C.c_double), ("clip_eps", C.c_double),
                ("vf_coef", C.c_double), ("ent_coef", C.c_double)] + \
               [(k, C.c_void_p) for k in ("dmu_rm", "dmu_fm", "dv_rm", "dv_fm", "dlogstd_partial", "loss_partial",
                                          "grads")]


class PgFusedArgs(C.Structure):
    _fields_ = [("net", C.c_int32), ("train", C.c_int32), ("rows", C.c_int64)] + \
               [(k, C.c_void_p) for k in ("packed", "params", "obs", "act", "logp_old", "adv", "ret", "stats")] + \
               [(k, C.c_double) for k in ("inv_total_samples", "clip_eps", "vf_coef", "ent_coef")] + \
               [(k, C.c_void_p) for k in ("values", "h1", "dh2", "partial", "loss_partial")] + \
               [("grid", C.c_int32), ("wgrad_splits", C.c_int32), ("wgrad_partial", C.c_void_p),
                ("grads", C.c_void_p), ("h1_mode", C.c_int32), ("h2_in", C.c_void_p), ("h2_out", C.c_void_p)]


class SchedArgs(C.Structure):
    _fields_ = [("codes", C.c_void_p), ("world", C.c_int32), ("horizon", C.c_int32), ("num_envs", C.c_int64),
                ("window", C.c_int32), ("max_candidates", C.c_int32), ("threshold", C.c_double),
                ("min_episodes", C.c_int64), ("episodes_before", C.c_int64)] + \
               [(k, C.c_void_p) for k in ("tail_in", "tail_len_in", "tail_out", "tail_len_out", "scratch")] + \
               [("scratch_bytes", C.c_int64), ("summary", C.c_void_p)]


class SchedPackedArgs(C.Structure):
    _fields_ = [("packs", C.c_void_p), ("pack_words", C.c_int64), ("bits", C.c_int32), ("world", C.c_int32),
                ("horizon", C.c_int32), ("num_envs", C.c_int64), ("window", C.c_int32),
                ("max_candidates", C.c_int32), ("threshold", C.c_double), ("min_episodes", C.c_int64),
                ("episodes_before", C.c_int64)] + \
               [(k, C.c_void_p) for k in ("tail_in", "tail_len_in", "tail_out", "tail_len_out", "scratch")] + \
               [("scratch_bytes", C.c_int64), ("summary", C.c_void_p), ("where", C.c_void_p)]


SCHED_MAX_CANDIDATES = 64  # DXRL_SCHED_MAX_CANDIDATES


class EvalSegment(C.Structure):
    _fields_ = [("curriculum_row", C.c_int32), ("num_episodes", C.c_int32), ("first_episode", C.c_int32),
                ("reserved", C.c_int32), ("obs_noise_std", C.c_double), ("dyn_noise_std", C.c_double),
                ("noise_offset", C.c_int64), ("noise_count", C.c_int64)]


class EvalArgs(C.Structure):
    _fields_ = [("num_lanes", C.c_int32), ("policy", C.c_int32), ("max_steps", C.c_int32),
                ("total_episodes", C.c_int32), ("lane_segments", C.c_void_p), ("segments", C.c_void_p),
                ("mean_action", C.c_void_p), ("exploration_noise", C.c_double), ("policy_tape", C.c_void_p),
                ("policy_stride", C.c_int64), ("noise_tape", C.c_void_p), ("reset_tape", C.c_void_p),
                ("policy_seed", C.c_uint64), ("noise_seed", C.c_uint64), ("reset_seed", C.c_uint64)] + \
               [(k, C.c_void_p) for k in ("ep_return", "ep_length", "ep_success", "ep_contacts", "contact_hist",
                                          "policy_used", "status", "obs_traj", "act_traj", "work_queue")]


_P = C.c_void_p
_I32, _I64, _F64 = C.c_int32, C.c_int64, C.c_double
_SIGS = {
    "dxrl_abi_version": (C.c_int, []),
    "dxrl_last_error": (C.c_char_p, []),
    "dxrl_env_layout_for": (C.c_int, [C.POINTER(EnvConfig), C.POINTER(EnvLayout)]),
    "dxrl_env_create": (C.c_int, [C.POINTER(EnvConfig), C.c_int32, _P, _P, C.POINTER(_P)]),
    "dxrl_env_destroy": (C.c_int, [_P]),
    "dxrl_env_set_curricula": (C.c_int, [_P, C.POINTER(Curriculum), C.c_int32, _P, _P]),
    "dxrl_env_set_curricula_async": (C.c_int, [_P, _P, C.c_int32, _P, _P]),
    "dxrl_env_reset": (C.c_int, [_P, _P, _P, _P, _P]),
    "dxrl_env_step": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "dxrl_env_observe": (C.c_int, [_P, _P, _P]),
    "dxrl_reward_compute": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, _P, _P,
                                      _P, _P, _P]),
    "dxrl_env_set_max_episode_steps": (C.c_int, [_P, C.c_int32]),
    "dxrl_learner_layout_for": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(LearnerLayout)]),
    "dxrl_learner_init": (C.c_int, [C.c_int32, C.c_int32, _P, _P]),
    "dxrl_learner_reset": (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P]),
    "dxrl_learner_select": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_double, _P, _P, _P]),
    "dxrl_learner_update": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_double, C.c_double, _P, _P, _P, _P]),
    "dxrl_rollout_simple": (C.c_int, [_P, _P, C.POINTER(LearnerConfig), C.c_int32, C.c_int32, C.c_int32,
                                      C.POINTER(RolloutIO), _P]),
    "dxrl_gemm_bf16": (C.c_int, [_I32, _P, _I64, _P, _I64, _I64, _I32, _I32, _P, _I64, _I32, _P, _I64, _P, _I64,
                                 _P, _I64, _P, _I64, _P, _I64, _I32, _P, _P]),
    "dxrl_wgrad_bf16": (C.c_int, [_I32, _P, _I64, _I32, _P, _I64, _I32, _I64, _I32, _P, _P, _P]),
    "dxrl_pg_sizes": (C.c_int, [C.POINTER(_I64), C.POINTER(_I64)]),
    "dxrl_pg_pack_weights": (C.c_int, [_I32, _P, _P, _P]),
    "dxrl_pg_rollout": (C.c_int, [_P, _P, _P, C.POINTER(PgRolloutArgs), _P]),
    "dxrl_pg_gae": (C.c_int, [_I32, _P, _P, _P, _I64, _I64, _F64, _F64, _P, _P, _P, _P, _P]),
    "dxrl_pg_gae_partial_doubles": (C.c_int, [_I64, _I64, C.POINTER(_I64)]),
    "dxrl_pg_adv_finalize": (C.c_int, [_I32, _I32, _P, _I64, _P, _P, _P]),
    "dxrl_pg_adv_combine": (C.c_int, [_I32, _P, _I32, _P, _P]),
    "dxrl_pg_heads": (C.c_int, [_I32, C.POINTER(PgHeadsArgs), _P]),
    "dxrl_pg_grad_sumsq": (C.c_int, [_I32, _P, _I64, _P, _P, _P]),
    "dxrl_pg_fused_sizes": (C.c_int, [C.POINTER(_I32), C.POINTER(_I64)]),
    "dxrl_pg_fused": (C.c_int, [_I32, C.POINTER(PgFusedArgs), _P]),
    "dxrl_pg_fused_pair": (C.c_int, [_I32, C.POINTER(PgFusedArgs), C.POINTER(PgFusedArgs), _P]),
    "dxrl_pg_fused_pair_gnorm": (C.c_int, [_I32, C.POINTER(PgFusedArgs), C.POINTER(PgFusedArgs), _P, _I32,
                                           C.POINTER(_I32), _P]),
    "dxrl_pg_rollout_kernel": (C.c_int, [C.c_void_p, _I32, C.POINTER(_I32)]),
    "dxrl_pg_gnorm_blocks": (C.c_int, [C.POINTER(_I32)]),
    "dxrl_evaluate": (C.c_int, [_P, C.POINTER(EvalArgs), _P]),
    "dxrl_sched_scratch_bytes": (C.c_int, [_I32, _I32, _I64, _I32, C.POINTER(_I64)]),
    "dxrl_sched_scan": (C.c_int, [_I32, C.POINTER(SchedArgs), _P]),
    "dxrl_sched_pack_words": (C.c_int, [_I32, _I64, _I32, _I32, C.POINTER(_I64)]),
    "dxrl_sched_pack": (C.c_int, [_I32, _P, _I32, _I64, _I32, _I32, _P, _P]),
    "dxrl_sched_packed_scratch_bytes": (C.c_int, [_I32, _I32, _I64, _I32, C.POINTER(_I64)]),
    "dxrl_sched_scan_packed": (C.c_int, [_I32, C.POINTER(SchedPackedArgs), _P]),
    "dxrl_sched_candidate_steps": (C.c_int, [_I32, _P, _I32, _I64, _I32, _I32, _P, _P, _P, _P]),
    "dxrl_sched_finish": (C.c_int, [_I32, _P, _P, _P]),
    "dxrl_pg_adam": (C.c_int, [_I32, _P, _P, _P, _P, _I64, _F64, _F64, _F64, _F64, _I64, _P, _F64, _P]),
    "dxrl_pg_optimizer_step": (C.c_int, [_I32, _P, _P, _P, _P, _P, _P, _P, _I64, _F64, _F64, _F64, _F64, _I64, _F64,
                                         _P, _P, _P, _P]),
    "dxrl_pg_adam_step": (C.c_int, [_I32, _P, _P, _P, _P, _P, _P, _P, _I64, _F64, _F64, _F64, _F64, _I64, _F64, _P,
                                    _I32, _P, _P, _P]),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def lib():
    """Load libdxrl.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                                  "(there is no CPU fallback)")
            h = C.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            if h.dxrl_abi_version() != ABI_VERSION:
                raise NativeError("libdxrl.so ABI version mismatch; rebuild")
            _lib = h
    return _lib


def check(rc: int, what: str = ""):
    if rc == DXRL_OK:
        return
    msg = lib().dxrl_last_error().decode(errors="replace")
    if rc in (DXRL_E_INVALID, DXRL_E_UNSUPPORTED):
        raise ValueError(f"{what}: {msg}")
    raise NativeError(f"{what}: {msg} (status {rc})")


def call(name: str, *args):
    check(getattr(lib(), name)(*args), name)


def gae_partial_doubles(num_envs: int, horizon: int) -> int:
    """f64 elements of dxrl_pg_gae's `partial` scratch (include/dxrl.h)."""
    out = C.c_int64()
    call("dxrl_pg_gae_partial_doubles", num_envs, horizon, C.byref(out))
    return out.value


def ptr(t) -> int | None:
    """Device address of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_of(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise NativeError("no HIP device visible: the dxrl hot path runs only on the GPU (no CPU fallback)")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise ValueError(f"device must be a GPU device, got {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def aligned_empty(nbytes: int, device, align: int = 256):
    """uint8 device buffer whose data_ptr is `align`-aligned; returns (owner, view)."""
    owner = torch.empty(nbytes + align, dtype=torch.uint8, device=device)
    off = (-owner.data_ptr()) % align
    return owner, owner[off:off + nbytes]
