"""The codec-facing surface of ``FasterDpEngine`` and its MERGE call site.

Mirrors (``/root/reference/backend/src``):

* ``FasterDpEngine::configure_compression``        engine/core.cpp:185-195
* ``FasterDpEngine::configure_compression_ratio``  engine/core.cpp:197-200
* ``FasterDpEngine::compress(name, tensor, ratio)`` engine/core.cpp:1210-1245
  (pybind ``fasterdp.compress``, python/pybind.cpp:80-82)
* ``ModuleCompress::run`` MERGE path                engine/modules/compress.cpp:36-70,139-142,172-186
* ``ModuleCpuOptimize::run`` MERGE decompress       engine/modules/cpu_optimize.cpp:40-72
* ``SGD::optimize_raw``                             optim/sgd.cpp:34-263

The rest of the engine (shm, ZMQ ring, scheduler, telemetry) is out of scope
(SURVEY.md section 2).  All compute runs on the HIP library; this module only
computes sizes, owns buffers and orders launches on torch's current stream.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import CodecError, check, lib
from .compressor import Compressor, make_compressor

__all__ = ["CodecEngine", "SparseSGD", "merge_numel", "api_numel", "scatter_merge", "owner_of"]


def merge_numel(n: int, ratio: float, world: int = 1) -> int:
    """Pairs per rank on the MERGE path (compress.cpp:44,52): the kept fraction is
    stored in a float, ``n * k`` is a float product, truncated to int64."""
    kf = np.float32((1.0 - float(ratio)) / float(np.float32(world)))
    return max(min(int(n), 1), int(np.float32(np.float32(n) * kf)))


def api_numel(n: int, ratio: float) -> int:
    """``numel_to_select = (1. - ratio) * numel`` with a float ratio (core.cpp:1216)."""
    return int((1.0 - float(np.float32(ratio))) * n)


def owner_of(sizes, world: int) -> list[int]:
    """Key-affine bucket placement for multi-GPU runs: greedy
    longest-first bytes balancing (largest bucket to the least-loaded rank,
    ties by rank and bucket order); deterministic, so a key always lands on the
    same rank and its AIMD state stays resident there."""
    load = [0] * world
    out = [0] * len(sizes)
    order = sorted(range(len(sizes)), key=lambda i: (-int(sizes[i]), i))
    for i in order:
        g = min(range(world), key=lambda r: (load[r], r))
        load[g] += int(sizes[i])
        out[i] = g
    return out


class CodecEngine:
    """Codec part of ``FasterDpEngine``: default method thresholdv16
    (core.cpp:23-26), ratio 0.99, ``compress(name, tensor, ratio)``."""

    def __init__(self, device: int = 0):
        self.device = device
        self.compression_ratio_ = 0.99
        self.compressor_: Compressor | None = None
        self.configure_compression("thresholdv16")

    def configure_compression(self, method: str) -> None:
        # core.cpp:185-195 accepts only these two; "topk" only via configure()
        if method not in ("thresholdv", "thresholdv16"):
            raise CodecError(-2, f"Unknown compression method {method}.")
        self.compressor_ = make_compressor(method, device=self.device)

    def configure(self, method: str) -> None:
        """The factory inside FasterDpEngine::configure (core.cpp:110-118)."""
        self.compressor_ = make_compressor(method, device=self.device)

    def configure_compression_ratio(self, ratio: float) -> None:
        assert 0 < ratio <= 1
        self.compression_ratio_ = float(ratio)

    def compression_ratio(self) -> float:
        return self.compression_ratio_

    def compressor(self) -> Compressor:
        return self.compressor_

    def compress(self, name: str, tensor, ratio: float):
        """core.cpp:1210-1245: returns (idx int32, val float32), narrowed to the count."""
        import torch
        if ratio < 0 or ratio > 1:
            raise CodecError(-1, "Ratio must be in range [0, 1].")
        k = api_numel(tensor.numel(), ratio)
        dev = tensor.device
        idx = torch.empty(k, dtype=torch.int32, device=dev)
        val = torch.empty(k, dtype=torch.float32, device=dev)
        if k == 0:
            return idx, val
        total = self.compressor_.compress(name, tensor.reshape(-1), k, idx, val)
        if total != k:
            idx, val = idx.narrow(0, 0, total), val.narrow(0, 0, total)
        return idx, val

    def compress_bucket(self, key: str, grad, world: int = 1, residual=None):
        """MERGE path of ModuleCompress::run (compress.cpp:38-70,139-186), device
        resident and asynchronous.  Returns (idx, val, count) where idx/val have
        ``numel * world`` zeroed slots (compress.cpp:60-64) and the first
        ``numel`` are this node's pairs.  With ``residual`` given, applies the
        error feedback: zero the selected entries of ``grad`` (all ``numel``
        slots, including unwritten zero indices, compress.cpp:178-179) and copy
        the bucket into ``residual`` (compress.cpp:185)."""
        import torch
        n = grad.numel()
        numel = merge_numel(n, self.compression_ratio_, world)
        idx = torch.zeros(numel * world, dtype=torch.int32, device=grad.device)
        val = torch.zeros(numel * world, dtype=torch.float32, device=grad.device)
        if not grad.is_contiguous():
            raise ValueError("grad must be contiguous")
        if residual is not None and (residual.numel() != n or residual.dtype != torch.float32
                                     or not residual.is_contiguous()):
            raise ValueError("residual must be a contiguous float32 tensor of the bucket's size")
        g = grad.reshape(-1)
        if residual is None:
            cnt = self.compressor_.compress_async(key, g, numel, idx[:numel], val[:numel], 0)
        else:
            # stg_merge_compress_batch_device: codec + error feedback, the
            # residual copy fused into thresholdv16's streaming pass
            cnt = self.compressor_.compress_batch_async([(key, g, numel, idx[:numel], val[:numel], 0)],
                                                        residuals=[residual.reshape(-1)])
        return idx, val, cnt


def scatter_merge(idx, val, per_rank: int, world: int, n: int, dense=None, mark=None, out_idx=None, out_val=None,
                  count=None):
    """MERGE decompress on the device (cpu_optimize.cpp:40-72).  ``dense``
    (float32[n]) and ``mark`` (uint8[n]) must be zero and are left zero.  Per
    rank, the last occurrence of a duplicated index wins (index_put_ without
    accumulate); the output holds each index once (unique1d)."""
    import torch
    dev = idx.device
    if out_idx is None:
        out_idx = torch.empty(per_rank * world, dtype=torch.int32, device=dev)
    if out_val is None:
        out_val = torch.empty(per_rank * world, dtype=torch.float32, device=dev)
    if count is None:
        count = torch.empty(1, dtype=torch.int32, device=dev)
    if world > 1:
        if dense is None:
            dense = torch.zeros(n, dtype=torch.float32, device=dev)
        if mark is None:
            mark = torch.zeros(n, dtype=torch.uint8, device=dev)
    dp = C.c_void_p(dense.data_ptr()) if dense is not None else None
    mp = C.c_void_p(mark.data_ptr()) if mark is not None else None
    check(lib().stg_scatter_merge_device(C.c_void_p(idx.data_ptr()), C.c_void_p(val.data_ptr()), per_rank, world, n,
                                         dp, mp, C.c_void_p(out_idx.data_ptr()), C.c_void_p(out_val.data_ptr()),
                                         C.c_void_p(count.data_ptr()),
                                         C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))
    return out_idx, out_val, count


def scatter_merge_check(device=None) -> None:
    """Raises CodecError when a MERGE decompress on the current stream of
    ``device`` hit a device failure (a look-back that gave up; the count of
    that call reads 0xffffffff).  Syncs the stream."""
    import torch
    dev = _cuda_device(device)
    with torch.cuda.device(dev):  # the C side keys the scratch on the current device
        check(lib().stg_scatter_merge_check(C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))


def scatter_merge_release(device=None) -> None:
    """Frees the MERGE decompress scratch kept for the current stream of
    ``device`` (call before dropping a stream that merged)."""
    import torch
    dev = _cuda_device(device)
    with torch.cuda.device(dev):
        check(lib().stg_scatter_merge_release(C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))


def _cuda_device(device):
    """torch.device of `device` (None or a bare "cuda": the current device)."""
    import torch
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    return torch.device("cuda", torch.cuda.current_device() if d.index is None else d.index)


def gather_slice(n: int, local_rank: int, num_gpus: int):
    """Local rank's slice [n*r/N, n*(r+1)/N) of the gather-add (cpu_gather.cpp:59-61)."""
    a, b = C.c_uint64(), C.c_uint64()
    check(lib().stg_gather_slice(n, local_rank, num_gpus, C.byref(a), C.byref(b)))
    return a.value, b.value


def gather_add(grads, residual, local_rank: int) -> None:
    """ModuleCpuGather::run on the device (cpu_gather.cpp:59-87): over this
    local rank's slice, ``grads[0] += residual + grads[1] + ... + grads[N-1]``
    left to right, in one pass.  ``grads`` are float32 device tensors of one
    size (peers' buffers where P2P is enabled); ``residual`` may be None."""
    import torch
    g0 = grads[0]
    n = g0.numel()
    for t in list(grads) + ([residual] if residual is not None else []):
        if t.numel() != n or t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("gather_add: contiguous float32 device tensors of one size")
    ptrs = (C.c_void_p * len(grads))(*[t.data_ptr() for t in grads])
    check(lib().stg_gather_add_device(C.c_void_p(g0.data_ptr()),
                                      C.c_void_p(residual.data_ptr()) if residual is not None else None,
                                      ptrs, len(grads), n, local_rank,
                                      C.c_void_p(torch.cuda.current_stream(g0.device.index).cuda_stream)))


WIRE_U16_IDX = 0x01  # COMM_FLAG_UINT16_IDX (comm_manager.h:24)
WIRE_F16_VAL = 0x02  # COMM_FLAG_FP16_VAL (comm_manager.h:25)


def wire_flag(tensor_numel: int, fp16_values: bool = False) -> int:
    """The flag byte CommManager::queueTx sends (comm_manager.cpp:573-590)."""
    return int(lib().stg_wire_flag(tensor_numel, int(fp16_values)))


def wire_encode(idx, val, flag: int, idx_out=None, val_out=None):
    """Pack a (idx, val) stream into the ring's wire layout on the device
    (comm_manager.cpp:509-548): int16-typed u16 indices when ``flag & 1``,
    fp16 bits (as int16) when ``flag & 2``; otherwise the 32-bit arrays."""
    import torch
    dev, n = idx.device, idx.numel()
    if idx_out is None:
        idx_out = torch.empty(n, dtype=torch.int16 if flag & WIRE_U16_IDX else torch.int32, device=dev)
    if val_out is None:
        val_out = torch.empty(n, dtype=torch.int16 if flag & WIRE_F16_VAL else torch.float32, device=dev)
    check(lib().stg_wire_encode_device(C.c_void_p(idx.data_ptr()), C.c_void_p(val.data_ptr()), n, flag,
                                       C.c_void_p(idx_out.data_ptr()), C.c_void_p(val_out.data_ptr()),
                                       C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))
    return idx_out, val_out


class StgWireStream(C.Structure):
    _fields_ = [("d_idx", C.c_void_p), ("d_val", C.c_void_p), ("numel", C.c_size_t), ("flag", C.c_int),
                ("d_idx_out", C.c_void_p), ("d_val_out", C.c_void_p)]


def wire_encode_batch(items):
    """Batched wire encode (``stg_wire_encode_batch_device``): items of
    (idx, val, flag, idx_out, val_out) device tensors; the same bytes as
    ``wire_encode`` on each, in launches of up to 16 streams."""
    import torch
    if not items:
        return
    arr = (StgWireStream * len(items))()
    for j, (idx, val, flag, io, vo) in enumerate(items):
        arr[j] = StgWireStream(idx.data_ptr(), val.data_ptr(), idx.numel(), int(flag), io.data_ptr(), vo.data_ptr())
    dev = items[0][0].device
    check(lib().stg_wire_encode_batch_device(arr, len(items),
                                             C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))


def wire_decode(widx, wval, flag: int, idx=None, val=None):
    """Unpack a received stream (comm_manager.cpp:877-906) into int32 indices
    and float32 values on the device."""
    import torch
    dev, n = widx.device, widx.numel()
    if idx is None:
        idx = torch.empty(n, dtype=torch.int32, device=dev)
    if val is None:
        val = torch.empty(n, dtype=torch.float32, device=dev)
    check(lib().stg_wire_decode_device(C.c_void_p(widx.data_ptr()), C.c_void_p(wval.data_ptr()), n, flag,
                                       C.c_void_p(idx.data_ptr()), C.c_void_p(val.data_ptr()),
                                       C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))
    return idx, val


def _merge_optimize(fn, h, param, name, idx, val, per_rank, world, dense, mark, out_idx, out_val, count):
    """ModuleCpuOptimize::run through one C call (``fn``): the MERGE decompress
    of ``world`` rank streams into the merged stream (returned), then the
    optimizer's step on it."""
    import torch
    dev, n = param.device, param.numel()
    if out_idx is None:
        out_idx = torch.empty(per_rank * world, dtype=torch.int32, device=dev)
    if out_val is None:
        out_val = torch.empty(per_rank * world, dtype=torch.float32, device=dev)
    if count is None:
        count = torch.empty(1, dtype=torch.int32, device=dev)
    if world > 1:
        if dense is None:
            dense = torch.zeros(n, dtype=torch.float32, device=dev)
        if mark is None:
            mark = torch.zeros(n, dtype=torch.uint8, device=dev)
    dp = C.c_void_p(dense.data_ptr()) if dense is not None else None
    mp = C.c_void_p(mark.data_ptr()) if mark is not None else None
    check(fn(h, name.encode(), C.c_void_p(param.data_ptr()), n, C.c_void_p(idx.data_ptr()), C.c_void_p(val.data_ptr()),
             per_rank, world, dp, mp, C.c_void_p(out_idx.data_ptr()), C.c_void_p(out_val.data_ptr()),
             C.c_void_p(count.data_ptr()), C.c_void_p(torch.cuda.current_stream(dev.index).cuda_stream)))
    return out_idx, out_val, count


class SparseSGD:
    """``SGD`` sparse optimizer (optim/sgd.h:10-50) on the device.  Options as
    SGD::configure (sgd.cpp:265-300); ``optimize_raw`` as sgd.cpp:34-263."""

    def __init__(self, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
                 nesterov: bool = False, maximize: bool = False, device: int = 0):
        h = C.c_void_p()
        check(lib().stg_sgd_create(device, lr, momentum, dampening, weight_decay, int(nesterov), int(maximize),
                                   C.byref(h)))
        self._h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().stg_sgd_destroy(h)
            except Exception:
                pass
            self._h = None

    def name(self) -> str:
        return "SGD"

    def optimize_raw(self, param, name: str, grad, gidx, grad_len: int | None = None, d_grad_len=None) -> None:
        import torch
        n = int(grad_len if grad_len is not None else grad.numel())
        check(lib().stg_sgd_optimize_raw_device(
            self._h, name.encode(), C.c_void_p(param.data_ptr()), param.numel(), C.c_void_p(grad.data_ptr()),
            C.c_void_p(gidx.data_ptr()), n, C.c_void_p(d_grad_len.data_ptr()) if d_grad_len is not None else None,
            C.c_void_p(torch.cuda.current_stream(param.device.index).cuda_stream)))

    def merge_optimize(self, param, name: str, idx, val, per_rank: int, world: int = 1, dense=None, mark=None,
                       out_idx=None, out_val=None, count=None):
        """ModuleCpuOptimize::run (cpu_optimize.cpp:26-100): the MERGE
        decompress, then optimize_raw on its output; at world 1 the step runs
        inside the decompress's emission launch."""
        return _merge_optimize(lib().stg_merge_optimize_sgd_device, self._h, param, name, idx, val, per_rank, world,
                               dense, mark, out_idx, out_val, count)

    def momentum_buffer(self, name: str, n: int):
        import torch
        out = np.zeros(n, np.float32)
        rc = lib().stg_sgd_get_momentum(self._h, name.encode(), C.c_void_p(out.ctypes.data), n,
                                        C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        return None if rc else out


class SparseAdam:
    """``Adam`` sparse optimizer (optim/adam.h:10-55) on the device.  Options as
    Adam::configure (adam.cpp:90-122; defaults adam.h:21-23, lr
    sparse_optimizer.h:30); ``optimize_raw`` as adam.cpp:19-86."""

    def __init__(self, lr: float = 1e-3, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, maximize: bool = False, device: int = 0):
        h = C.c_void_p()
        check(lib().stg_adam_create(device, lr, b1, b2, eps, weight_decay, int(amsgrad), int(maximize), C.byref(h)))
        self._h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().stg_adam_destroy(h)
            except Exception:
                pass
            self._h = None

    def name(self) -> str:
        return "Adam"

    def optimize_raw(self, param, name: str, grad, gidx, grad_len: int | None = None, d_grad_len=None) -> None:
        import torch
        n = int(grad_len if grad_len is not None else grad.numel())
        check(lib().stg_adam_optimize_raw_device(
            self._h, name.encode(), C.c_void_p(param.data_ptr()), param.numel(), C.c_void_p(grad.data_ptr()),
            C.c_void_p(gidx.data_ptr()), n, C.c_void_p(d_grad_len.data_ptr()) if d_grad_len is not None else None,
            C.c_void_p(torch.cuda.current_stream(param.device.index).cuda_stream)))

    def merge_optimize(self, param, name: str, idx, val, per_rank: int, world: int = 1, dense=None, mark=None,
                       out_idx=None, out_val=None, count=None):
        """ModuleCpuOptimize::run with Adam: the step inside the decompress's
        emission at world 1 without amsgrad, else the two calls."""
        return _merge_optimize(lib().stg_merge_optimize_adam_device, self._h, param, name, idx, val, per_rank, world,
                               dense, mark, out_idx, out_val, count)

    def check_device(self) -> None:
        """Raise if a device-side failure was flagged (amsgrad look-back timeout)."""
        import torch
        check(lib().stg_adam_check(self._h, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))

    def state(self, name: str, n: int):
        """(m, v, vmax, tick) of a name, or None before its first call."""
        import torch
        m, v = np.zeros(n, np.float32), np.zeros(n, np.float32)
        vmax, tick = C.c_float(), C.c_uint32()
        rc = lib().stg_adam_get_state(self._h, name.encode(), C.c_void_p(m.ctypes.data), C.c_void_p(v.ctypes.data),
                                      n, C.byref(vmax), C.byref(tick),
                                      C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        return None if rc else (m, v, np.float32(vmax.value), int(tick.value))
