"""TEST INFRASTRUCTURE ONLY -- ctypes wrappers for the CPU checker libraries.

* ``Oracle``    wraps ``oracle/liboracle.so`` (clean-room restatement,
                oracle/stg_oracle.cpp); travels to the GPU box.
* ``Reference`` wraps ``oracle/_ref/libstg_ref.so`` (the reference's own
                backend/src/compress sources compiled in place; this container only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (stellatrain_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libstg_ref.so")
REF_SRC = "/root/reference/backend/src"

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")


def build(ref: bool | None = None) -> None:
    """Compile liboracle.so (and oracle/_ref when the reference is present)."""
    targets = ["all"]
    if ref is None:
        ref = os.path.isdir(REF_SRC)
    if ref:
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE, *targets], check=True)


def _load(path: str) -> C.CDLL:
    if not os.path.exists(path):
        build(ref=path == REF_SO)
    return C.CDLL(path)


class _Codecs:
    """Common numpy-facing surface of the oracle and the reference driver."""

    prefix = ""

    def __init__(self, lib: C.CDLL):
        self.lib = lib
        p = self.prefix
        f = getattr(lib, f"{p}_tv16_new"); f.restype = C.c_void_p; f.argtypes = []
        f = getattr(lib, f"{p}_tv16_free"); f.restype = None; f.argtypes = [C.c_void_p]
        f = getattr(lib, f"{p}_tv16_compress"); f.restype = C.c_size_t
        f.argtypes = [C.c_void_p, C.c_char_p, _f32p, C.c_size_t, C.c_uint32, _u32p, C.c_size_t, _f32p, C.c_int32]
        f = getattr(lib, f"{p}_tv16_state"); f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        f = getattr(lib, f"{p}_tv_new"); f.restype = C.c_void_p; f.argtypes = []
        f = getattr(lib, f"{p}_tv_free"); f.restype = None; f.argtypes = [C.c_void_p]
        f = getattr(lib, f"{p}_tv_compress"); f.restype = C.c_size_t
        f.argtypes = [C.c_void_p, C.c_uint64, _f32p, C.c_size_t, C.c_uint32, _u32p, C.c_size_t, _f32p]
        f = getattr(lib, f"{p}_tv_state"); f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_float)]

    # -- thresholdv16 -------------------------------------------------------
    def tv16_new(self):
        return getattr(self.lib, f"{self.prefix}_tv16_new")()

    def tv16_free(self, h):
        getattr(self.lib, f"{self.prefix}_tv16_free")(h)

    def tv16_compress(self, h, name: str, src: np.ndarray, k: int, cap: int | None = None, idx_offset: int = 0):
        cap = k if cap is None else cap
        idx = np.zeros(cap, np.uint32)
        val = np.zeros(cap, np.float32)
        src = np.ascontiguousarray(src, np.float32)
        cnt = getattr(self.lib, f"{self.prefix}_tv16_compress")(
            h, name.encode(), src, src.size, k, idx, cap, val, idx_offset)
        return int(cnt), idx, val

    def tv16_state(self, h, name: str):
        t, inc = C.c_float(), C.c_float()
        rc = getattr(self.lib, f"{self.prefix}_tv16_state")(h, name.encode(), C.byref(t), C.byref(inc))
        return None if rc else (t.value, inc.value)

    # -- threshold-v --------------------------------------------------------
    def tv_new(self):
        return getattr(self.lib, f"{self.prefix}_tv_new")()

    def tv_free(self, h):
        getattr(self.lib, f"{self.prefix}_tv_free")(h)

    def tv_compress(self, h, key: int, src: np.ndarray, k: int, cap: int | None = None):
        cap = k if cap is None else cap
        idx = np.zeros(cap, np.uint32)
        val = np.zeros(cap, np.float32)
        src = np.ascontiguousarray(src, np.float32)
        cnt = getattr(self.lib, f"{self.prefix}_tv_compress")(h, key, src, src.size, k, idx, cap, val)
        return int(cnt), idx, val

    def tv_state(self, h, key: int):
        t = C.c_float()
        rc = getattr(self.lib, f"{self.prefix}_tv_state")(h, key, C.byref(t))
        return None if rc else t.value


class Oracle(_Codecs):
    prefix = "orc"

    def __init__(self, path: str = ORACLE_SO):
        lib = _load(path)
        super().__init__(lib)
        lib.orc_synth_fill.restype = None
        lib.orc_synth_fill.argtypes = [_f32p, C.c_size_t, C.c_uint64, C.c_int, C.c_uint32]
        lib.orc_tv16_first_threshold.restype = C.c_float
        lib.orc_tv16_first_threshold.argtypes = [_f32p, C.c_size_t, C.c_uint32]
        lib.orc_tv_first_threshold.restype = C.c_float
        lib.orc_tv_first_threshold.argtypes = [_f32p, C.c_size_t, C.c_uint32]
        lib.orc_tv16_block_sums.restype = None
        lib.orc_tv16_block_sums.argtypes = [_f32p, C.c_size_t, _f32p]
        lib.orc_topk_compress.restype = C.c_int64
        lib.orc_topk_compress.argtypes = [_f32p, C.c_size_t, C.c_uint32, _u32p, C.c_size_t, _f32p, C.c_int32, C.c_int]
        lib.orc_merge_numel.restype = C.c_int64
        lib.orc_merge_numel.argtypes = [C.c_int64, C.c_double, C.c_int]
        lib.orc_api_numel.restype = C.c_int64
        lib.orc_api_numel.argtypes = [C.c_int64, C.c_float]
        lib.orc_merge_decompress.restype = C.c_size_t
        lib.orc_merge_decompress.argtypes = [_u32p, _f32p, C.c_size_t, C.c_int, C.c_size_t, _u32p, _f32p]
        lib.orc_sgd_new.restype = C.c_void_p
        lib.orc_sgd_new.argtypes = [C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int]
        lib.orc_sgd_free.restype = None
        lib.orc_sgd_free.argtypes = [C.c_void_p]
        lib.orc_sgd_apply.restype = None
        lib.orc_sgd_apply.argtypes = [C.c_void_p, C.c_char_p, _f32p, C.c_uint32, _f32p, _u32p, C.c_uint32]
        lib.orc_sgd_momentum.restype = C.c_int
        lib.orc_sgd_momentum.argtypes = [C.c_void_p, C.c_char_p, _f32p, C.c_uint32]
        lib.orc_adam_new.restype = C.c_void_p
        lib.orc_adam_new.argtypes = [C.c_float] * 5 + [C.c_int, C.c_int]
        lib.orc_adam_free.restype = None
        lib.orc_adam_free.argtypes = [C.c_void_p]
        lib.orc_adam_apply.restype = None
        lib.orc_adam_apply.argtypes = [C.c_void_p, C.c_char_p, _f32p, C.c_uint32, _f32p, _u32p, C.c_uint32]
        lib.orc_adam_state.restype = C.c_int
        lib.orc_adam_state.argtypes = [C.c_void_p, C.c_char_p, _f32p, _f32p, C.c_uint32, C.POINTER(C.c_float)]
        lib.orc_wire_flag.restype = C.c_uint8
        lib.orc_wire_flag.argtypes = [C.c_uint64, C.c_int]
        lib.orc_wire_encode.restype = None
        lib.orc_wire_encode.argtypes = [_u32p, _f32p, C.c_size_t, C.c_uint8, C.c_void_p, C.c_void_p]
        lib.orc_wire_decode.restype = None
        lib.orc_wire_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint8, _u32p, _f32p]
        lib.orc_gather_slice.restype = None
        lib.orc_gather_slice.argtypes = [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        lib.orc_gather_add.restype = None
        lib.orc_gather_add.argtypes = [_f32p, _f32p, C.POINTER(C.c_void_p), C.c_int, C.c_int64, C.c_int]
        lib.orc_last_error.restype = C.c_char_p

    def synth(self, n: int, seed: int, dist: int = 0, param: int = 0) -> np.ndarray:
        out = np.empty(n, np.float32)
        self.lib.orc_synth_fill(out, n, seed, dist, param)
        return out

    def tv16_first_threshold(self, src, k):
        src = np.ascontiguousarray(src, np.float32)
        return float(self.lib.orc_tv16_first_threshold(src, src.size, k))

    def tv_first_threshold(self, src, k):
        src = np.ascontiguousarray(src, np.float32)
        return float(self.lib.orc_tv_first_threshold(src, src.size, k))

    def tv16_block_sums(self, src):
        src = np.ascontiguousarray(src, np.float32)
        out = np.empty(src.size // 16, np.float32)
        self.lib.orc_tv16_block_sums(src, src.size, out)
        return out

    def topk_compress(self, src, k, cap=None, idx_offset=0, bug_compat=True):
        cap = k if cap is None else cap
        idx = np.zeros(max(cap, 1), np.uint32)
        val = np.zeros(max(cap, 1), np.float32)
        src = np.ascontiguousarray(src, np.float32)
        rc = self.lib.orc_topk_compress(src, src.size, k, idx, cap, val, idx_offset, int(bug_compat))
        if rc < 0:
            raise RuntimeError(self.lib.orc_last_error().decode())
        return int(rc), idx[:cap], val[:cap]

    def merge_numel(self, n, ratio, world=1):
        return int(self.lib.orc_merge_numel(n, ratio, world))

    def api_numel(self, n, ratio):
        return int(self.lib.orc_api_numel(n, ratio))

    def merge_decompress(self, idx, val, per_rank, world, n):
        out_idx = np.zeros(per_rank * world, np.uint32)
        out_val = np.zeros(per_rank * world, np.float32)
        m = self.lib.orc_merge_decompress(np.ascontiguousarray(idx, np.uint32), np.ascontiguousarray(val, np.float32),
                                          per_rank, world, n, out_idx, out_val)
        return out_idx[:m], out_val[:m]

    def sgd_new(self, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, maximize=False):
        return self.lib.orc_sgd_new(lr, momentum, dampening, weight_decay, int(nesterov), int(maximize))

    def sgd_free(self, h):
        self.lib.orc_sgd_free(h)

    def sgd_apply(self, h, name, param, g, gidx):
        self.lib.orc_sgd_apply(h, name.encode(), param, param.size, np.ascontiguousarray(g, np.float32),
                               np.ascontiguousarray(gidx, np.uint32), len(g))

    def sgd_momentum(self, h, name, n):
        out = np.zeros(n, np.float32)
        rc = self.lib.orc_sgd_momentum(h, name.encode(), out, n)
        return None if rc else out

    def wire_flag(self, tensor_numel: int, fp16_values: bool = False) -> int:
        return int(self.lib.orc_wire_flag(tensor_numel, int(fp16_values)))

    def wire_encode(self, idx, val, flag):
        """comm_manager.cpp queueTx casts: (idx bytes as u16/u32 array, val as u16/f32 array)."""
        idx = np.ascontiguousarray(idx, np.uint32)
        val = np.ascontiguousarray(val, np.float32)
        n = idx.size
        oi = np.zeros(n, np.uint16 if flag & 1 else np.uint32)
        ov = np.zeros(n, np.uint16 if flag & 2 else np.float32)
        self.lib.orc_wire_encode(idx, val, n, flag, oi.ctypes.data, ov.ctypes.data)
        return oi, ov

    def wire_decode(self, widx, wval, flag):
        widx, wval = np.ascontiguousarray(widx), np.ascontiguousarray(wval)
        n = widx.size
        idx, val = np.zeros(n, np.uint32), np.zeros(n, np.float32)
        self.lib.orc_wire_decode(widx.ctypes.data, wval.ctypes.data, n, flag, idx, val)
        return idx, val

    def gather_slice(self, n: int, local_rank: int, num_gpus: int):
        a, b = C.c_int64(), C.c_int64()
        self.lib.orc_gather_slice(n, local_rank, num_gpus, C.byref(a), C.byref(b))
        return a.value, b.value

    def gather_add(self, grads, resid, local_rank: int):
        """cpu_gather.cpp:59-87 for one local rank: grads[0] (in place) +=
        resid, grads[1], ... over the rank's slice."""
        ptrs = (C.c_void_p * len(grads))(*[g.ctypes.data for g in grads])
        self.lib.orc_gather_add(grads[0], resid, ptrs, len(grads), grads[0].size, local_rank)

    def adam_new(self, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, weight_decay=0.0, amsgrad=False, maximize=False):
        return self.lib.orc_adam_new(lr, b1, b2, eps, weight_decay, int(amsgrad), int(maximize))

    def adam_free(self, h):
        self.lib.orc_adam_free(h)

    def adam_apply(self, h, name, param, g, gidx):
        self.lib.orc_adam_apply(h, name.encode(), param, param.size, np.ascontiguousarray(g, np.float32),
                                np.ascontiguousarray(gidx, np.uint32), len(g))

    def adam_state(self, h, name, n):
        """(m, v, vmax, tick) of a name, or None before its first call."""
        m, v, vmax = np.zeros(n, np.float32), np.zeros(n, np.float32), C.c_float()
        tick = self.lib.orc_adam_state(h, name.encode(), m, v, n, C.byref(vmax))
        return None if tick < 0 else (m, v, np.float32(vmax.value), tick)


class Reference(_Codecs):
    """The reference's own compress/*.cpp (this container only)."""

    prefix = "ref"

    def __init__(self, path: str = REF_SO):
        lib = _load(path)
        super().__init__(lib)
        lib.ref_topk_compress.restype = C.c_longlong
        lib.ref_topk_compress.argtypes = [_f32p, C.c_size_t, C.c_uint32, _u32p, C.c_size_t, _f32p]

    def topk_compress(self, src, k, cap=None):
        cap = k if cap is None else cap
        idx = np.zeros(max(cap, 1), np.uint32)
        val = np.zeros(max(cap, 1), np.float32)
        src = np.ascontiguousarray(src, np.float32)
        rc = self.lib.ref_topk_compress(src, src.size, k, idx, cap, val)
        if rc < 0:
            raise RuntimeError("Invalid parameter k")
        return int(rc), idx[:cap], val[:cap]


def reference_available() -> bool:
    return os.path.isdir(REF_SRC) or os.path.exists(REF_SO)
