"""The reference's threading contract on one codec handle.

The engine calls ``compressor()->compress()`` from up to 32 ThreadPool workers
at once, each on a different key (engine/config.h:6-7,
engine/core_module_api.cpp:7-24, engine/modules/compress.cpp:140-142);
thresholdv16 guards its threshold maps with a mutex
(compress/thresholdv16.cpp:84,256).  Here:

* ``tests/cpp/concurrency`` -- 16 ``std::thread``s on ONE handle through the
  drop-in header ``include/stg/compressor.h``: per thread one key through
  ``compress()`` (host memory, the handle's per-thread stream) and one through
  ``compress_device()`` (device memory, a HIP stream the thread created),
  interleaved, several AIMD calls each;
* a Python ``threading`` variant through ctypes (which drops the GIL for the
  call): 16 threads, one torch stream each, ``compress_device`` on their own
  keys;

and every call's whole (idx, val) stream, count and threshold / increment
bits are compared with the oracle replaying each key's sequence alone.
"""
from __future__ import annotations

import os
import subprocess
import threading

import numpy as np
import pytest

from parity import assert_same_stream, assert_topk_values, fbits

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binary():
    exe = os.path.join(ROOT, "tests", "cpp", "concurrency")
    if not os.path.exists(exe):  # normally built by __graft_entry__.build()
        from stellatrain_amd.build import build_concurrency
        build_concurrency()
    return exe


def _read(path, calls):
    data = open(path, "rb").read()
    out, p = [], 0
    for _ in range(2 * calls):
        tag = int(np.frombuffer(data, np.uint32, 1, p)[0])
        cnt = int(np.frombuffer(data, np.uint64, 1, p + 4)[0])
        p += 12
        idx = np.frombuffer(data, np.uint32, cnt, p).copy()
        p += 4 * cnt
        val = np.frombuffer(data, np.float32, cnt, p).copy()
        p += 4 * cnt
        t, inc = np.frombuffer(data, np.float32, 2, p)
        p += 8
        out.append((tag, cnt, idx, val, t, inc))
    assert p == len(data)
    return out


def _check_thread(oracle, method, t, n0, calls, recs):
    n = n0 + 5 * (t % 4)
    k = n // 100
    hs = {}
    for path in (0, 1):
        hs[path] = oracle.tv16_new() if method == "thresholdv16" else oracle.tv_new() if method == "thresholdv" else None
    for c in range(calls):
        for path in (0, 1):
            tag, cnt, idx, val, tg, ig = recs[2 * c + path]
            assert tag == path
            src = oracle.synth(n, 1000 * t + (500 if path else 0) + c)
            if method == "thresholdv16":
                co, io, vo = oracle.tv16_compress(hs[path], f"{t}@{'dev' if path else 'host'}", src, k)
                st = oracle.tv16_state(hs[path], f"{t}@{'dev' if path else 'host'}")
                assert (fbits(tg), fbits(ig)) == (fbits(st[0]), fbits(st[1])), (t, c, path)
            elif method == "thresholdv":
                co, io, vo = oracle.tv_compress(hs[path], 1, src, k)
                assert fbits(tg) == fbits(oracle.tv_state(hs[path], 1)), (t, c, path)
            else:
                co, io, vo = oracle.topk_compress(src, k, bug_compat=True)
            assert cnt == co, (t, c, path, cnt, co)
            if method == "topk":
                assert_topk_values(val, vo[:co])
            else:
                assert_same_stream(idx, val, io, vo, co)
    for h in hs.values():
        if h is not None:
            (oracle.tv16_free if method == "thresholdv16" else oracle.tv_free)(h)


@pytest.mark.parametrize("method,threads,calls,n", [("thresholdv16", 16, 6, 1 << 20), ("thresholdv", 16, 4, 1 << 19),
                                                    ("topk", 8, 2, 1 << 18)])
def test_cpp_threads_share_one_handle(gpu, oracle, method, threads, calls, n, tmp_path):
    out = str(tmp_path / "c")
    r = subprocess.run([_binary(), method, str(threads), str(calls), str(n), out], capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr + r.stdout
    for t in range(threads):
        _check_thread(oracle, method, t, n, calls, _read(f"{out}.{t}", calls))


def test_python_threads_device_streams(gpu, oracle):
    """16 Python threads, one torch stream each, compress_device on one shared
    thresholdv16 handle (ctypes releases the GIL for the call)."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    from stellatrain_amd._capi import check, lib
    import ctypes as C
    comp = ThresholdvCompressor16()
    T, calls, n0 = 16, 5, (1 << 20) + 7
    results, errors = {}, []
    barrier = threading.Barrier(T)

    def worker(t):
        try:
            n = n0 + 3 * t
            k = n // 100
            s = torch.cuda.Stream(device=gpu)
            src = torch.empty(n, dtype=torch.float32, device=gpu)
            outs = []
            barrier.wait()
            for c in range(calls):
                # the outputs are zeroed on the thread's stream too: torch's
                # streams do not wait for the default stream, so zeros issued
                # there could land after the call's writes
                with torch.cuda.stream(s):
                    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
                    val = torch.zeros(k, dtype=torch.float32, device=gpu)
                    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
                    check(lib().stg_synth_fill_device(C.c_void_p(src.data_ptr()), n, 7000 * (t + 1) + c, 0, 0,
                                                      C.c_void_p(s.cuda_stream)))
                    comp.compress_raw(f"py{t}@w".encode(), src.data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(),
                                      cnt.data_ptr(), s.cuda_stream)
                outs.append((idx, val, cnt))
            s.synchronize()
            results[t] = [(int(c.item()), i.cpu().numpy().view(np.uint32), v.cpu().numpy()) for i, v, c in outs]
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    assert not errors, errors
    comp.check_device()
    for t in range(T):
        n = n0 + 3 * t
        k = n // 100
        h = oracle.tv16_new()
        for c in range(calls):
            co, io, vo = oracle.tv16_compress(h, f"py{t}@w", oracle.synth(n, 7000 * (t + 1) + c), k)
            cnt, ig, vg = results[t][c]
            assert cnt == co
            assert_same_stream(ig, vg, io, vo, co)
        st = oracle.tv16_state(h, f"py{t}@w")
        assert fbits(comp.state(f"py{t}@w")[0]) == fbits(st[0])
        oracle.tv16_free(h)
