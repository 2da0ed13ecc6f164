"""ctypes binding of libdpt.so (include/dpt.h).

The product path has NO CPU fallback: if the HIP library is missing or no GPU is
visible, every call raises ``DptError``.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPT_LIB") or os.path.join(HERE, "libdpt.so")

DPT_OK = 0
DPT_E_CAP = -4
DPT_E_RCCL = -6
DPT_RCCL_ID_BYTES = 128
DPT_MODE_RAW = 0
DPT_MODE_PRESPLIT = 1
DPT_MODE_ATOMS = 2
DPT_FLAG_UNCAPPED = 0x10
DPT_FLAG_LEN_ONLY = 0x20
STATUS_OK, STATUS_NO_TOKENIZATION, STATUS_EMPTY_WORD, STATUS_TOO_LONG, STATUS_INTERNAL = range(5)


class DptError(RuntimeError):
    pass


class VocabStats(ctypes.Structure):
    _fields_ = [("n_tokens", ctypes.c_uint32), ("n_nodes", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("max_bytes", ctypes.c_uint32), ("max_cp", ctypes.c_uint32), ("device_bytes", ctypes.c_uint64),
                ("hash_max_probe", ctypes.c_uint32), ("hash_buckets", ctypes.c_uint32)]


_lib = None
P = ctypes.c_void_p
U64 = ctypes.c_uint64
I32 = ctypes.c_int


def lib():
    """Load libdpt.so (raises DptError when the HIP extension is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("DPT_NO_TORCH", "0") != "1":
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7. Loading it
        # first makes libdpt.so bind to that copy (same SONAME) instead of /opt/rocm's, so device
        # pointers and streams from torch are valid for the engine.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise DptError(f"HIP extension not built: {LIB_PATH} missing (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    L.dpt_last_error.restype = ctypes.c_char_p
    L.dpt_abi_version.restype = I32
    L.dpt_vocab_create.argtypes = [P, P, P, ctypes.c_uint32, I32, ctypes.POINTER(P)]
    L.dpt_vocab_destroy.argtypes = [P]
    L.dpt_vocab_stats_get.argtypes = [P, ctypes.POINTER(VocabStats)]
    L.dpt_ctx_create.argtypes = [I32, ctypes.POINTER(P)]
    L.dpt_ctx_destroy.argtypes = [P]
    L.dpt_ctx_reserve.argtypes = [P, U64, U64]
    L.dpt_ctx_reserve_vocab.argtypes = [P, P, U64, U64, U64]
    L.dpt_ctx_workspace_bytes.argtypes = [P, ctypes.POINTER(U64), ctypes.POINTER(U64)]
    L.dpt_ctx_long_need.argtypes = [P, ctypes.POINTER(U64), ctypes.POINTER(U64)]
    L.dpt_encode.argtypes = [P, P, I32, P, U64, P, P, U64, P, U64, P, P, P, P]
    L.dpt_encode_host.argtypes = [P, P, I32, P, U64, P, P, U64, P, U64, P, P, P]
    L.dpt_encode_padded.argtypes = [P, P, I32, P, U64, P, P, U64, P, U64, P, P, P, P]
    L.dpt_dp_host.argtypes = [P, P, I32, P, U64, P, P, U64, P, P, P]
    L.dpt_dp_host_far.argtypes = [P, P, I32, P, U64, P, P, U64, P, P, P, P, U64, P]
    L.dpt_token_histogram.argtypes = [P, P, U64, P, ctypes.c_uint32, P]
    L.dpt_ctx_set_histogram.argtypes = [P, P, ctypes.c_uint32]
    L.dpt_ctx_set_histogram_ex.argtypes = [P, P, ctypes.c_uint32, I32]
    L.dpt_ctx_profile.argtypes = [P, I32]
    L.dpt_ctx_profile_read.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64)]
    L.dpt_ctx_debug_counter_bias.argtypes = [P, U64]
    L.dpt_rccl_get_unique_id.argtypes = [P]
    L.dpt_rccl_comm_create.argtypes = [P, I32, I32, I32, ctypes.POINTER(P)]
    L.dpt_rccl_comm_destroy.argtypes = [P]
    L.dpt_hist_allreduce.argtypes = [P, ctypes.c_size_t, P, P]
    for name in ("dpt_vocab_create", "dpt_vocab_destroy", "dpt_vocab_stats_get", "dpt_ctx_create", "dpt_ctx_destroy",
                 "dpt_ctx_reserve", "dpt_ctx_reserve_vocab", "dpt_ctx_workspace_bytes", "dpt_ctx_long_need", "dpt_encode", "dpt_encode_padded", "dpt_encode_host", "dpt_dp_host", "dpt_dp_host_far", "dpt_token_histogram",
                 "dpt_ctx_set_histogram", "dpt_ctx_set_histogram_ex", "dpt_ctx_profile", "dpt_ctx_profile_read", "dpt_ctx_debug_counter_bias",
                 "dpt_rccl_get_unique_id", "dpt_rccl_comm_create", "dpt_rccl_comm_destroy", "dpt_hist_allreduce"):
        getattr(L, name).restype = I32
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != DPT_OK:
        msg = lib().dpt_last_error().decode("utf-8", "replace")
        raise DptError(f"{what} failed ({rc}): {msg}")


EXPORTED = ["dpt_last_error", "dpt_abi_version", "dpt_vocab_create", "dpt_vocab_destroy", "dpt_vocab_stats_get",
            "dpt_ctx_create", "dpt_ctx_destroy", "dpt_ctx_reserve", "dpt_ctx_reserve_vocab", "dpt_ctx_workspace_bytes",
            "dpt_ctx_long_need",
            "dpt_encode", "dpt_encode_padded", "dpt_encode_host",
            "dpt_dp_host", "dpt_dp_host_far", "dpt_token_histogram", "dpt_ctx_set_histogram", "dpt_ctx_set_histogram_ex",
            "dpt_ctx_profile", "dpt_ctx_profile_read", "dpt_ctx_debug_counter_bias",
            "dpt_rccl_get_unique_id", "dpt_rccl_comm_create", "dpt_rccl_comm_destroy", "dpt_hist_allreduce"]
