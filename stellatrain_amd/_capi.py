"""ctypes binding of ``libstg_codec.so`` (the C-ABI in include/stg/codec.h).

The HIP library is the product: there is no CPU fallback.  Importing the
symbols of a missing or stale library raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# STG_CODEC_LIB: an alternative in-tree build of the same sources (tuning
# experiments, tools/gpu_run.sh); the default is the product library.
LIB_PATH = os.environ.get("STG_CODEC_LIB") or os.path.join(_HERE, "libstg_codec.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "stg", "codec.h")

STG_OK = 0
ERRORS = {-1: "STG_ERR_INVALID", -2: "STG_ERR_UNKNOWN", -3: "STG_ERR_HIP", -4: "STG_ERR_UNSUPPORTED",
          -5: "STG_ERR_DEVICE"}


class CodecError(RuntimeError):
    """Raised for a non-zero status; mirrors the reference's std::runtime_error."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class StgBucket(C.Structure):
    """``stg_bucket_t`` (include/stg/codec.h): one bucket of a batched call."""
    _fields_ = [("key", C.c_char_p), ("d_src", C.c_void_p), ("n", C.c_size_t), ("k", C.c_uint32),
                ("d_idx", C.c_void_p), ("idx_cap", C.c_size_t), ("d_val", C.c_void_p), ("val_cap", C.c_size_t),
                ("idx_offset", C.c_int32), ("d_count", C.c_void_p)]


_lib: C.CDLL | None = None

_SIGS = {
    "stg_codec_create": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    "stg_codec_destroy": (C.c_int, [C.c_void_p]),
    "stg_codec_name": (C.c_char_p, [C.c_void_p]),
    "stg_codec_compress_host": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p,
                                          C.c_size_t, C.c_void_p, C.c_size_t, C.c_int32, C.POINTER(C.c_size_t)]),
    "stg_codec_compress_device": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p,
                                            C.c_size_t, C.c_void_p, C.c_size_t, C.c_int32, C.c_void_p, C.c_void_p]),
    "stg_codec_compress_batch_device": (C.c_int, [C.c_void_p, C.POINTER(StgBucket), C.c_size_t, C.c_void_p]),
    "stg_codec_get_state": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.POINTER(C.c_float),
                                      C.POINTER(C.c_float), C.c_void_p]),
    "stg_codec_check": (C.c_int, [C.c_void_p]),
    "stg_codec_debug_words": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "stg_codec_set_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "stg_codec_get_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "stg_scatter_merge_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_size_t, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "stg_scatter_merge_check": (C.c_int, [C.c_void_p]),
    "stg_scatter_merge_release": (C.c_int, [C.c_void_p]),
    "stg_error_feedback_device": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "stg_sgd_create": (C.c_int, [C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int,
                                 C.POINTER(C.c_void_p)]),
    "stg_sgd_destroy": (C.c_int, [C.c_void_p]),
    "stg_sgd_optimize_raw_device": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                              C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "stg_sgd_get_momentum": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "stg_merge_optimize_sgd_device": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                                C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "stg_merge_optimize_adam_device": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                                 C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p,
                                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "stg_adam_create": (C.c_int, [C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int,
                                  C.POINTER(C.c_void_p)]),
    "stg_adam_destroy": (C.c_int, [C.c_void_p]),
    "stg_adam_optimize_raw_device": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                               C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "stg_adam_get_state": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.c_void_p]),
    "stg_adam_check": (C.c_int, [C.c_void_p, C.c_void_p]),
    "stg_merge_compress_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "stg_codec_compress_wire_batch_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                                       C.c_void_p]),
    "stg_merge_gather_compress_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                   C.c_void_p]),
    "stg_gather_slice": (C.c_int, [C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "stg_gather_add_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_uint64, C.c_int,
                                        C.c_void_p]),
    "stg_wire_flag": (C.c_int, [C.c_uint64, C.c_int]),
    "stg_wire_encode_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p]),
    "stg_wire_decode_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p]),
    "stg_wire_encode_batch_device": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
    "stg_synth_fill_device": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p]),
    "stg_last_error": (C.c_char_p, []),
}


def header_symbols(path: str = HEADER) -> list[str]:
    """Every function declared in include/stg/codec.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(stg_\w+)\s*\(", txt, re.M)))


def lib() -> C.CDLL:
    """Load libstg_codec.so (HIP runtime resolved through torch's when loaded)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"stellatrain_amd: HIP codec library missing at {LIB_PATH}; "
                          "run __graft_entry__.build() (make -C stellatrain_amd/csrc)")
    try:  # share torch's HIP runtime (same soname) when torch is present
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
        pass
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)  # AttributeError = stale library: fail loudly
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != STG_OK:
        msg = lib().stg_last_error().decode(errors="replace")
        raise CodecError(rc, f"{ERRORS.get(rc, rc)}: {msg}")
