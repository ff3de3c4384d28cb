"""GPU parity of the wire form written by the thresholdv16 emission
(``stg_codec_compress_wire_batch_device``): the reference compresses, then
queueTx packs the stream (comm_manager.cpp:486-590).  Here the codec's own
stores write the packed types.  Every byte must equal the oracle's
thresholdv16 stream (oracle/_ref-pinned) packed by the wire restatement
(tests/test_wire_oracle.py), over sequences of calls that take the ordered
scan, the regime-B fill after a scale drop (window, leader and crew), the
one-bucket path and the batched launch.
"""
from __future__ import annotations

import numpy as np
import pytest

from stellatrain_amd.synth import D1, D2, seed_for, synth

pytestmark = pytest.mark.gpu

# per-call gradient scale: 100x drops empty the window and take the crew
SCALES = [1.0, 1.0, 0.01, 0.01, 1.0, 30.0]


def _u(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint16) if a.itemsize == 2 else a.view(np.uint32)


def _bufs(torch, gpu, cap, flag):
    di = torch.full((cap,), -1, dtype=torch.int16 if flag & 1 else torch.int32, device=gpu)
    dv = torch.full((cap,), -1, dtype=torch.int16 if flag & 2 else torch.float32, device=gpu)
    return di, dv


def _run(gpu, oracle, cases, calls=len(SCALES)):
    """cases: (key, n, k, dist, flag, idx_offset); one batched call per step."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    for it in range(calls):
        items, flags, expect = [], [], []
        for j, (key, n, k, dist, flag, off) in enumerate(cases):
            src = (synth(n, seed_for(900 + j, it), dist) * np.float32(SCALES[it % len(SCALES)])).astype(np.float32)
            co, io, vo = oracle.tv16_compress(ho, key, src, k, idx_offset=off)
            expect.append((co, oracle.wire_encode(io[:co], vo[:co], flag)))
            di, dv = _bufs(torch, gpu, k, flag)
            items.append((key, torch.from_numpy(src).to(gpu), k, di, dv, off))
            flags.append(flag)
        counts = comp.compress_batch_async(items, wire_flags=flags)
        torch.cuda.synchronize()
        got = counts.cpu().numpy().tolist()
        for (key, src, k, di, dv, off), flag, (co, (oi, ov)), cg in zip(items, flags, expect, got):
            assert cg == co, (it, key)
            assert np.array_equal(_u(di.cpu().numpy())[:co], _u(oi)), (it, key, flag)
            assert np.array_equal(_u(dv.cpu().numpy())[:co], _u(ov)), (it, key, flag)
    comp.check_device()
    oracle.tv16_free(ho)


@pytest.mark.parametrize("n,k,dist,flag,off", [
    (60000, 600, D1, 1, 0),          # u16 indices as queueTx picks them (numel < 65536)
    (60000, 600, D1, 1, 70000),      # offsets past 32767: blocks saturate, the tail truncates
    (4099, 41, D2, 3, 30000),        # ragged tail, fp16 values, count % 8 != 0
    ((1 << 22) + 5, 41943, D1, 2, 0),  # one-bucket path at size, fp16 values
    ((1 << 22) + 5, 41943, D1, 3, 12345),
])
def test_wire_fused_one_bucket(gpu, oracle, n, k, dist, flag, off):
    _run(gpu, oracle, [("w@b", n, k, dist, flag, off)])


def test_wire_fused_batched(gpu, oracle):
    """Four keys in one launch (the batched scan and fill), every flag."""
    _run(gpu, oracle, [("b0@w", 60000, 600, D1, 1, 70000), ("b1@w", 1 << 20, 10485, D1, 2, 0),
                       ("b2@w", 300007, 3000, D2, 3, 100), ("b3@w", 1 << 20, 10485, D1, 0, 5)])


def test_wire_fused_unsupported_codec(gpu):
    """Only thresholdv16 fuses the packing: the other codecs refuse the call."""
    import torch
    from stellatrain_amd import TopkCompressor
    from stellatrain_amd._capi import CodecError
    comp = TopkCompressor()
    src = torch.ones(1024, dtype=torch.float32, device=gpu)
    di, dv = _bufs(torch, gpu, 16, 1)
    with pytest.raises(CodecError):
        comp.compress_batch_async([("t@w", src, 16, di, dv)], wire_flags=[1])
