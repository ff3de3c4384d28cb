"""GPU parity of the wire format (engine/comm_manager.cpp:486-590) through the
C-ABI (``stg_wire_encode_device`` / ``stg_wire_decode_device``) against the
oracle restatement, which tests/test_wire_oracle.py pins to the x86
instruction semantics of the reference's casts.  Bit-exact on every byte.
"""
from __future__ import annotations

import numpy as np
import pytest

from stellatrain_amd.synth import D1, seed_for, synth

pytestmark = pytest.mark.gpu


def _stream(n, seed, idx_hi):
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, idx_hi, n, dtype=np.uint32)
    val = (rng.standard_normal(n) * 10.0 ** rng.integers(-9, 6, n)).astype(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 65504.0, 65520.0, 6.0e-8, 2.98e-8, -1.7, 3e9, -0.5],
                  np.float32)
    if n >= sp.size:
        val[rng.choice(n, sp.size, replace=False)] = sp
    return idx, val


def _u(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint16) if a.itemsize == 2 else a.view(np.uint32)


@pytest.mark.parametrize("n", [1, 8, 9, 17, 655, 4099, 167772])
@pytest.mark.parametrize("flag", [0, 1, 2, 3])
def test_wire_encode_decode_parity(gpu, oracle, n, flag):
    import torch
    from stellatrain_amd import wire_decode, wire_encode
    idx, val = _stream(n, 100 * n + flag, 65536 if flag & 1 else 1 << 30)
    oi, ov = oracle.wire_encode(idx, val, flag)
    gi, gv = wire_encode(torch.from_numpy(idx.view(np.int32)).to(gpu), torch.from_numpy(val).to(gpu), flag)
    assert np.array_equal(_u(gi.cpu().numpy()), _u(oi))
    assert np.array_equal(_u(gv.cpu().numpy()), _u(ov))
    # decode the oracle's bytes on the device (a reference peer's stream)
    di, dv = oracle.wire_decode(oi, ov, flag)
    wi = torch.from_numpy(oi.view(np.int16 if flag & 1 else np.int32)).to(gpu)
    wv = torch.from_numpy(ov.view(np.int16) if flag & 2 else ov).to(gpu)
    hi, hv = wire_decode(wi, wv, flag)
    assert np.array_equal(_u(hi.cpu().numpy()), di)
    assert np.array_equal(_u(hv.cpu().numpy()), _u(dv))


def test_wire_codec_round_trip(gpu, oracle):
    """thresholdv16 stream of a < 65536-element bucket (u16 flag, as queueTx
    picks it) through encode -> decode on the device equals the oracle's
    reference-path bytes; indices below 32768 survive exactly."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel, wire_decode, wire_encode, wire_flag
    n = 60000
    k = merge_numel(n, 0.99)
    flag = wire_flag(n)
    assert flag == oracle.wire_flag(n) == 1
    comp = ThresholdvCompressor16()
    for it in range(3):
        src = synth(n, seed_for(53, it), D1)
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        comp.compress("wire@w", torch.from_numpy(src).to(gpu), k, idx, val)
        hi, hv = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        oi, ov = oracle.wire_encode(hi, hv, flag)
        di, dv = oracle.wire_decode(oi, ov, flag)
        wi, wv = wire_encode(idx, val, flag)
        ri, rv = wire_decode(wi, wv, flag)
        assert np.array_equal(_u(ri.cpu().numpy()), di) and np.array_equal(_u(rv.cpu().numpy()), _u(dv))
        low = hi < 32768
        assert np.array_equal(di[low], hi[low])


def test_wire_encode_batch_matches_single(gpu, oracle):
    """stg_wire_encode_batch_device: 37 streams (three launches of <= 16),
    mixed flags and lengths incl. 0 and < 8, byte-identical to the oracle."""
    import torch
    from stellatrain_amd import wire_encode_batch
    rng = np.random.default_rng(7)
    lens = [0, 1, 7, 9, 655, 4099, 65535] + [int(x) for x in rng.integers(1, 20000, 30)]
    items, expect = [], []
    for j, n in enumerate(lens):
        flag = j % 4
        idx, val = _stream(n, 500 + j, 65536 if flag & 1 else 1 << 30)
        di = torch.from_numpy(idx.view(np.int32)).to(gpu)
        dv = torch.from_numpy(val).to(gpu)
        io = torch.full((max(n, 1),), -1, dtype=torch.int16 if flag & 1 else torch.int32, device=gpu)[:n]
        vo = torch.full((max(n, 1),), -1, dtype=torch.int16 if flag & 2 else torch.float32, device=gpu)[:n]
        items.append((di, dv, flag, io, vo))
        expect.append(oracle.wire_encode(idx, val, flag))
    wire_encode_batch(items)
    torch.cuda.synchronize()
    for (di, dv, flag, io, vo), (oi, ov) in zip(items, expect):
        assert np.array_equal(_u(io.cpu().numpy()), _u(oi))
        assert np.array_equal(_u(vo.cpu().numpy()), _u(ov))
