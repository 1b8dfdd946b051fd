"""ctypes bridge to libsacmi.so (the C ABI declared in include/sacmi.h).

The library is the product: there is no CPU fallback.  Loading fails loudly when
the shared object is missing or was built for another ABI version.

``import torch`` happens before the library is loaded on purpose: torch ships its
own HIP runtime (``libamdhip64.so.7``); loading it first makes the dynamic linker
resolve libsacmi's HIP dependency to the same runtime instance, so device
pointers and streams are shared with torch (needed for the RCCL all-reduce of the
data-parallel path).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SACMI_LIB_PATH") or os.path.join(_HERE, "libsacmi.so")   # override: tuning builds
ABI_VERSION = 3

c_f32p = ctypes.POINTER(ctypes.c_float)
c_f64p = ctypes.POINTER(ctypes.c_double)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_vp = ctypes.c_void_p

SACMI_OK, SACMI_EVALUE, SACMI_ESTATE, SACMI_EDEVICE, SACMI_ENAN = range(5)
REPLAY_UNIFORM, REPLAY_PER = 0, 1
COMPUTE_FP32, COMPUTE_BF16 = 0, 1
RCCL_ID_BYTES = 128          # SACMI_RCCL_ID_BYTES
POLICY, Q1, Q2, Q1_TARGET, Q2_TARGET = range(5)
SLOT_PARAM, SLOT_GRAD, SLOT_ADAM_M, SLOT_ADAM_V = range(4)
(S_LOG_ALPHA, S_ALPHA, S_ALPHA_IS_TENSOR, S_STEP_POLICY, S_STEP_Q1, S_STEP_Q2, S_STEP_ALPHA,
 S_ADAM_M_LOG_ALPHA, S_ADAM_V_LOG_ALPHA, S_GRAD_LOG_ALPHA, S_PER_FRAME,
 S_NOISE_COUNTER, S_KEEP_GRADS, S_GRAPH_COUNT) = range(14)


class SacmiConfig(ctypes.Structure):
    _fields_ = [
        ("state_dim", ctypes.c_int32), ("action_dim", ctypes.c_int32),
        ("hidden_dim", ctypes.c_int32), ("max_batch", ctypes.c_int32),
        ("gamma", ctypes.c_double), ("tau", ctypes.c_double), ("lr", ctypes.c_double),
        ("alpha", ctypes.c_double), ("auto_entropy", ctypes.c_int32),
        ("replay_kind", ctypes.c_int32), ("action_low", ctypes.c_double),
        ("action_high", ctypes.c_double), ("capacity", ctypes.c_int64),
        ("per_alpha", ctypes.c_double), ("per_beta_start", ctypes.c_double),
        ("per_beta_frames", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("n_hidden", ctypes.c_int32), ("compute_dtype", ctypes.c_int32),
    ]


# name -> (argtypes)   every function returns int status except the two noted
_PROTOS = {
    "sacmi_device_count": [c_i32p],
    "sacmi_create": [ctypes.POINTER(SacmiConfig), ctypes.c_int, ctypes.POINTER(c_vp)],
    "sacmi_destroy": [c_vp],
    "sacmi_set_stream": [c_vp, c_vp],
    "sacmi_synchronize": [c_vp],
    "sacmi_tensor_numel": [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i64p],
    "sacmi_set_tensor": [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_f32p,
                         ctypes.c_int64],
    "sacmi_get_tensor": [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_f32p,
                         ctypes.c_int64],
    "sacmi_set_scalar": [c_vp, ctypes.c_int, ctypes.c_double],
    "sacmi_get_scalar": [c_vp, ctypes.c_int, c_f64p],
    "sacmi_push": [c_vp, c_f32p, c_f32p, c_f32p, c_f32p, c_u8p, ctypes.c_int64],
    "sacmi_push_packed": [c_vp, c_vp, ctypes.c_int64],
    "sacmi_len": [c_vp, c_i64p],
    "sacmi_replay_clear": [c_vp],
    "sacmi_get_rows": [c_vp, c_i64p, ctypes.c_int64, c_f32p, c_f32p, c_f32p, c_f32p, c_u8p],
    "sacmi_get_slots": [c_vp, c_i64p, ctypes.c_int64, c_f32p, c_f32p, c_f32p, c_f32p, c_u8p],
    "sacmi_rng_set_mt": [c_vp, ctypes.c_int, c_u32p, ctypes.c_int32],
    "sacmi_rng_get_mt": [c_vp, ctypes.c_int, c_u32p, c_i32p],
    "sacmi_rng_seed_device": [c_vp, ctypes.c_uint64, ctypes.c_uint64],
    "sacmi_sample_indices": [c_vp, ctypes.c_int32, c_i64p],
    "sacmi_step": [c_vp, ctypes.c_int32, c_i64p, c_f32p, c_f32p, c_f32p],
    "sacmi_step_async": [c_vp, ctypes.c_int32],
    "sacmi_step_launch": [c_vp, ctypes.c_int32],
    "sacmi_step_wait": [c_vp, c_f32p],
    "sacmi_step_many_async": [c_vp, ctypes.c_int32, ctypes.c_int32],
    "sacmi_step_phase_ex": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_int32,
                            ctypes.c_int32, ctypes.c_int32],
    "sacmi_step_ride_possible": [c_vp, ctypes.c_int32, c_i32p],
    "sacmi_step_act16": [c_vp, ctypes.c_int32, c_i32p],
    "sacmi_read_activation": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_f32p, ctypes.c_int64],
    "sacmi_read_batch": [c_vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), c_f32p, ctypes.c_int64],
    "sacmi_fetch_losses": [c_vp, c_f32p, ctypes.c_int32, c_i32p],
    "sacmi_step_phase": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_float],
    "sacmi_grad_buffer": [c_vp, ctypes.c_int, ctypes.POINTER(c_vp), c_i64p],
    "sacmi_grad_arena_numel": [c_vp, c_i64p],
    "sacmi_attach_grad_arena": [c_vp, c_vp, ctypes.c_int64],
    "sacmi_per_sample": [c_vp, ctypes.c_int32, c_f64p, c_i64p, c_f32p],
    "sacmi_per_update": [c_vp, c_i64p, c_f32p, ctypes.c_int64],
    "sacmi_per_get_priorities": [c_vp, c_f32p, ctypes.c_int64],
    "sacmi_per_set_priorities": [c_vp, c_f32p, ctypes.c_int64],
    "sacmi_act": [c_vp, c_f32p, ctypes.c_int32, ctypes.c_int32, c_f32p, c_f32p],
    "sacmi_allreduce_unique_id": [ctypes.c_char_p, ctypes.c_int32],
    "sacmi_allreduce_init": [c_vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32],
    "sacmi_step_dp": [c_vp, ctypes.c_int32, ctypes.c_int32],
    "sacmi_dp_loopback_init": [c_vp, ctypes.c_int32],
    "sacmi_dp_set_sharded": [c_vp, ctypes.c_int32],
    "sacmi_dp_sync_state": [c_vp],
    "sacmi_dp_sharded": [c_vp, ctypes.POINTER(ctypes.c_int32)],
    "sacmi_profile_step": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, c_f32p, c_f64p,
                           ctypes.c_int32, c_i32p],
    "sacmi_profile_sites": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, c_f32p, c_f64p,
                            c_f64p, ctypes.c_int32, c_i32p],
    "sacmi_selftest_span_checker": [c_i32p, c_i32p],
    "sacmi_profile_timeline": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                               c_i32p, c_i32p, c_i32p, c_f64p, c_f64p, c_f64p, c_f64p, c_i32p,
                               c_f64p],
    "sacmi_profile_timeline_dp": [c_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                  c_i32p, c_i32p, c_i32p, c_f64p, c_f64p, c_f64p, c_f64p, c_i32p,
                                  c_f64p],
}
# kernel kinds of the launch timeline (TlKind, csrc/sacmi_internal.h)
TL_KINDS = {1: "k_gemm", 2: "k_fwd_x6", 3: "k_fwd16", 4: "k_axk16", 5: "k_axk_x6", 6: "k_dw_part16",
            7: "k_dw_fin", 8: "k_heads_sample", 9: "k_gemm_sample_bwd", 10: "k_mt_sample",
            11: "k_gather", 12: "k_per_f1", 13: "k_per_f2", 14: "k_per_f2b", 15: "k_per_f3",
            16: "k_per_f4", 17: "per_unfused", 18: "k_adam", 19: "k_sample_bwd_tail",
            20: "k_fwd16p", 21: "k_dw_part_x6"}
EXPORTS = tuple(_PROTOS) + ("sacmi_abi_version", "sacmi_last_error")

_lib = None


class SacmiError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and type the library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsacmi.so not found at {LIB_PATH}; build it with "
            f"`make -C humanoid-walking-with-sac_amd` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    lib.sacmi_abi_version.restype = ctypes.c_int
    lib.sacmi_abi_version.argtypes = []
    lib.sacmi_last_error.restype = ctypes.c_char_p
    lib.sacmi_last_error.argtypes = []
    for name, args in _PROTOS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    v = lib.sacmi_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"libsacmi ABI {v} != expected {ABI_VERSION}; rebuild")
    _lib = lib
    return lib


def check(status: int) -> None:
    """Map a status code to the reference's exception types."""
    if status == SACMI_OK:
        return
    msg = load().sacmi_last_error().decode(errors="replace")
    if status in (SACMI_EVALUE, SACMI_ENAN):
        raise ValueError(msg)
    raise SacmiError(f"sacmi error {status}: {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args))


def fptr(a):
    return a.ctypes.data_as(c_f32p) if a is not None else None


def dptr(a):
    return a.ctypes.data_as(c_f64p) if a is not None else None


def i64ptr(a):
    return a.ctypes.data_as(c_i64p) if a is not None else None


def i32ptr(a):
    return a.ctypes.data_as(c_i32p) if a is not None else None


def u8ptr(a):
    return a.ctypes.data_as(c_u8p) if a is not None else None


def u32ptr(a):
    return a.ctypes.data_as(c_u32p) if a is not None else None


def device_count() -> int:
    n = ctypes.c_int32(0)
    call("sacmi_device_count", ctypes.byref(n))
    return n.value
