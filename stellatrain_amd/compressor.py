"""Host-side mirror of the reference codec interface, over the HIP C-ABI.

Reference interface (``/root/reference/backend/src/compress/compressor.h:12-31``)::

    class Compressor {
        Compressor(std::unique_ptr<ThreadPool> &thread_pool, std::string name);
        const std::string &name();
        virtual size_t compress(const std::string &name, ConstSegment<float> src, uint32_t k,
                                Segment<uint32_t> dst_idx, Segment<float> dst_val,
                                int32_t idx_offset = 0) = 0;
    };

``ConstSegment``/``Segment`` (pointer, length) pairs become 1-D tensors or
arrays whose length is the segment length.  Device tensors run the
device-resident path on torch's current HIP stream; host tensors/arrays run
the host path (copy in, compress on the GPU, copy out).  ``compress`` returns
the reference's ``size_t`` (so it synchronises for device inputs);
``compress_async`` returns the count as a device tensor and never syncs.
Errors raise ``RuntimeError`` (``CodecError``), as the reference throws
``std::runtime_error`` (topk.cpp:34, core.cpp:117,193).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import CodecError, StgBucket, check, lib

__all__ = ["Compressor", "ThresholdvCompressor16", "ThresholdvCompressor", "TopkCompressor", "make_compressor",
           "CodecError"]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _stream_ptr(device: int) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


class Compressor:
    """Base class: one C-ABI codec handle (``stg_codec_create``)."""

    _method = ""

    def __init__(self, thread_pool=None, *, device: int = 0, method: str | None = None):
        # thread_pool: accepted for signature parity (compressor.h:26); the GPU
        # codec needs no host pool.
        self.thread_pool_ = thread_pool
        self.device = device
        self._method = method or self._method
        h = C.c_void_p()
        check(lib().stg_codec_create(self._method.encode(), device, C.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().stg_codec_destroy(h)
            except Exception:
                pass
            self._h = None

    def name(self) -> str:
        """``Compressor::name()`` (compressor.h:28)."""
        return lib().stg_codec_name(self._h).decode()

    # -- compress ----------------------------------------------------------
    def compress(self, name: str, src, k: int, dst_idx, dst_val, idx_offset: int = 0) -> int:
        """``Compressor::compress`` (compressor.h:30); returns the pair count."""
        if _is_torch(src) and src.is_cuda:
            cnt = self.compress_async(name, src, k, dst_idx, dst_val, idx_offset)
            c = int(cnt.item())
            self.check_device()  # the synchronous form surfaces device-side failures as errors
            return c
        return self._compress_host(name, src, k, dst_idx, dst_val, idx_offset)

    def compress_async(self, name: str, src, k: int, dst_idx, dst_val, idx_offset: int = 0, count=None):
        """Device-resident compress on torch's current stream; returns a 1-element
        uint32-valued int32 tensor holding the count (no host sync)."""
        import torch
        assert src.is_cuda and dst_idx.is_cuda and dst_val.is_cuda, "device path needs device tensors"
        assert src.dtype == torch.float32 and dst_val.dtype == torch.float32
        assert dst_idx.dtype in (torch.int32, torch.uint32)
        assert src.is_contiguous() and dst_idx.is_contiguous() and dst_val.is_contiguous()
        if count is None:
            count = torch.empty(1, dtype=torch.int32, device=src.device)
        check(lib().stg_codec_compress_device(
            self._h, name.encode(), C.c_void_p(src.data_ptr()), src.numel(), int(k),
            C.c_void_p(dst_idx.data_ptr()), dst_idx.numel(), C.c_void_p(dst_val.data_ptr()), dst_val.numel(),
            int(idx_offset), C.c_void_p(count.data_ptr()), C.c_void_p(_stream_ptr(src.device.index))))
        return count

    def compress_raw(self, key: bytes, src_ptr: int, n: int, k: int, idx_ptr: int, cap: int, val_ptr: int,
                     count_ptr: int, stream_ptr: int, idx_offset: int = 0) -> None:
        """Lowest-overhead device call: raw device pointers, no validation
        beyond the C-ABI's own (for tight host loops such as bench.py)."""
        rc = self._fn_dev(self._h, key, src_ptr, n, k, idx_ptr, cap, val_ptr, cap, idx_offset, count_ptr, stream_ptr)
        if rc:
            check(rc)

    def compress_batch_async(self, items, stream=None, counts=None, residuals=None, wire_flags=None):
        """Batched device compress (``stg_codec_compress_batch_device``): the
        same results as ``compress_async`` on each (name, src, k, dst_idx,
        dst_val[, idx_offset]) in order, on one stream.  Returns a
        (len(items),) int32 tensor of counts (no host sync).  With
        ``residuals`` (one float32 tensor per item) it is the MERGE compress
        with error feedback (``stg_merge_compress_batch_device``,
        compress.cpp:139-186): every src is zeroed at its dst_idx slots and its
        residual receives the zeroed bucket.  With ``wire_flags`` (one STG_WIRE_*
        flag per item; thresholdv16) the emission writes each stream's wire form
        (``stg_codec_compress_wire_batch_device``, comm_manager.cpp:486-590):
        dst_idx is int16 under flag 1, dst_val float16-sized under flag 2, their
        numel the pair capacity."""
        import torch
        if not items:
            return None
        dev = items[0][1].device
        if counts is None:
            counts = torch.zeros(len(items), dtype=torch.int32, device=dev)
        arr = (StgBucket * len(items))()
        keep = []
        for j, it in enumerate(items):
            name, src, k, di, dv = it[:5]
            off = it[5] if len(it) > 5 else 0
            assert src.is_cuda and di.is_cuda and dv.is_cuda and src.dtype == torch.float32
            assert src.is_contiguous() and di.is_contiguous() and dv.is_contiguous()
            kb = name.encode()
            keep.append(kb)
            arr[j] = StgBucket(kb, src.data_ptr(), src.numel(), int(k), di.data_ptr(), di.numel(), dv.data_ptr(),
                               dv.numel(), int(off), counts.data_ptr() + 4 * j)
        sp = stream if stream is not None else _stream_ptr(dev.index)
        if wire_flags is not None:
            if residuals is not None or len(wire_flags) != len(items):
                raise ValueError("wire_flags: one flag per bucket, no residuals")
            fl = (C.c_int * len(items))(*[int(f) for f in wire_flags])
            check(lib().stg_codec_compress_wire_batch_device(self._h, arr, fl, len(items), C.c_void_p(sp)))
            return counts
        if residuals is None:
            check(lib().stg_codec_compress_batch_device(self._h, arr, len(items), C.c_void_p(sp)))
            return counts
        if len(residuals) != len(items):
            raise ValueError("one residual per bucket")
        rp = (C.c_void_p * len(items))()
        for j, (it, r) in enumerate(zip(items, residuals)):
            if r.numel() != it[1].numel() or r.dtype != torch.float32 or not r.is_contiguous() or not r.is_cuda:
                raise ValueError("residual must be a contiguous float32 device tensor of the bucket's size")
            rp[j] = r.data_ptr()
        check(lib().stg_merge_compress_batch_device(self._h, arr, rp, len(items), C.c_void_p(sp)))
        return counts

    def merge_gather_compress_async(self, name: str, grads, k: int, dst_idx, dst_val, residual=None,
                                    idx_offset: int = 0, count=None, stream=None):
        """One MERGE task with the intra-node gather ahead of it
        (``stg_merge_gather_compress_device``; cpu_gather.cpp:59-87, then
        compress.cpp:139-186): ``grads[0] += residual + grads[1] + ... +
        grads[N-1]`` (this rank's slices, left to right), compress grads[0]
        under ``name``, and with ``residual`` its error feedback.  thresholdv16
        sums the sources inside its streaming pass.  Returns the int32 count
        tensor (no host sync)."""
        import torch
        g0 = grads[0]
        n = g0.numel()
        for t in list(grads) + ([residual] if residual is not None else []) + [dst_idx, dst_val]:
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("merge_gather_compress: contiguous device tensors")
        for t in list(grads) + ([residual] if residual is not None else []):
            if t.numel() != n or t.dtype != torch.float32:
                raise ValueError("merge_gather_compress: float32 sources of one size")
        if count is None:
            count = torch.zeros(1, dtype=torch.int32, device=g0.device)
        kb = name.encode()
        b = StgBucket(kb, g0.data_ptr(), n, int(k), dst_idx.data_ptr(), dst_idx.numel(), dst_val.data_ptr(),
                      dst_val.numel(), int(idx_offset), count.data_ptr())
        ptrs = (C.c_void_p * len(grads))(*[t.data_ptr() for t in grads])
        sp = stream if stream is not None else _stream_ptr(g0.device.index)
        check(lib().stg_merge_gather_compress_device(
            self._h, C.byref(b), C.c_void_p(residual.data_ptr()) if residual is not None else None, ptrs,
            len(grads), C.c_void_p(sp)))
        return count

    @staticmethod
    def bucket_array(rows):
        """Prebuilt ``stg_bucket_t`` array from raw tuples (key bytes, src_ptr,
        n, k, idx_ptr, cap, val_ptr, count_ptr[, idx_offset]) for tight loops."""
        arr = (StgBucket * len(rows))()
        for j, r in enumerate(rows):
            arr[j] = StgBucket(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[5], r[8] if len(r) > 8 else 0, r[7])
        return arr

    def compress_batch_raw(self, arr, nb: int, stream_ptr: int) -> None:
        """Batched call on a prebuilt ``bucket_array`` (no per-call marshalling)."""
        f = getattr(self, "_fn_batch_cache", None)
        if f is None:
            f = self._fn_batch_cache = lib().stg_codec_compress_batch_device
        rc = f(self._h, arr, nb, stream_ptr)
        if rc:
            check(rc)

    @property
    def _fn_dev(self):
        f = getattr(self, "_fn_dev_cache", None)
        if f is None:
            f = self._fn_dev_cache = lib().stg_codec_compress_device
        return f

    def _compress_host(self, name, src, k, dst_idx, dst_val, idx_offset) -> int:
        s = src.numpy() if _is_torch(src) else src
        di = dst_idx.numpy() if _is_torch(dst_idx) else dst_idx
        dv = dst_val.numpy() if _is_torch(dst_val) else dst_val
        if not (isinstance(s, np.ndarray) and s.dtype == np.float32 and s.flags.c_contiguous):
            raise TypeError("src must be a contiguous float32 array/tensor")
        if di.dtype.itemsize != 4 or dv.dtype != np.float32 or not di.flags.c_contiguous or not dv.flags.c_contiguous:
            raise TypeError("dst_idx must be contiguous (u)int32 and dst_val contiguous float32")
        out = C.c_size_t()
        check(lib().stg_codec_compress_host(
            self._h, name.encode(), C.c_void_p(s.ctypes.data), s.size, int(k), C.c_void_p(di.ctypes.data),
            di.size, C.c_void_p(dv.ctypes.data), dv.size, int(idx_offset), C.byref(out)))
        return int(out.value)

    # -- introspection (tests) ----------------------------------------------
    def state(self, name: str = "", key_ptr: int = 0, stream=None):
        """Per-key AIMD state (threshold, threshold_inc) or None if never seen."""
        t, inc = C.c_float(), C.c_float()
        sp = stream if stream is not None else 0
        rc = lib().stg_codec_get_state(self._h, name.encode(), C.c_void_p(key_ptr), C.byref(t), C.byref(inc),
                                       C.c_void_p(sp))
        if rc != 0:
            return None
        return t.value, inc.value

    def set_timing(self, enable: bool) -> None:
        check(lib().stg_codec_set_timing(self._h, int(enable)))

    def get_timing(self):
        """(scan_ms, fill_ms, call_ms) accumulated since the last read, and calls."""
        ms = (C.c_double * 3)()
        calls = C.c_uint64()
        check(lib().stg_codec_get_timing(self._h, ms, C.byref(calls)))
        return (ms[0], ms[1], ms[2]), int(calls.value)

    def check_device(self) -> None:
        check(lib().stg_codec_check(self._h))


class ThresholdvCompressor16(Compressor):
    """``ThresholdvCompressor16(std::unique_ptr<ThreadPool>&, bool multicore=true)``
    (thresholdv16.h:33-34); per-name AIMD state (thresholdv16.cpp:81-97)."""

    _method = "thresholdv16"

    def __init__(self, thread_pool=None, multicore: bool = True, *, device: int = 0):
        self.multicore_ = multicore  # never read by the reference either
        super().__init__(thread_pool, device=device)


class ThresholdvCompressor(Compressor):
    """``ThresholdvCompressor(std::unique_ptr<ThreadPool>&, bool multicore=true)``
    (thresholdv.h:24-25); AIMD state keyed by the src pointer (thresholdv.cpp:44)."""

    _method = "thresholdv"

    def __init__(self, thread_pool=None, multicore: bool = True, *, device: int = 0):
        self.multicore_ = multicore
        super().__init__(thread_pool, device=device)


class TopkCompressor(Compressor):
    """``TopkCompressor(std::unique_ptr<ThreadPool>&)`` (topk.h:28-29).  ``exact=False``
    keeps the shipped behaviour (byte-count memcpy, idx 0..k-1: topk.cpp:31,42);
    ``exact=True`` is the intended top-k by |x| with real indices."""

    _method = "topk"

    def __init__(self, thread_pool=None, *, exact: bool = False, device: int = 0):
        super().__init__(thread_pool, device=device, method="topk_exact" if exact else "topk")


def make_compressor(method: str, thread_pool=None, *, device: int = 0) -> Compressor:
    """Factory of FasterDpEngine::configure (core.cpp:110-118)."""
    if method == "thresholdv":
        return ThresholdvCompressor(thread_pool, True, device=device)
    if method == "thresholdv16":
        return ThresholdvCompressor16(thread_pool, True, device=device)
    if method == "topk":
        return TopkCompressor(thread_pool, device=device)
    if method == "topk_exact":
        return TopkCompressor(thread_pool, exact=True, device=device)
    raise CodecError(-2, f"Unknown compression method {method}.")
