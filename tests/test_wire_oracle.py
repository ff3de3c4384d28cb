"""Pin the wire-format oracle (oracle/stg_oracle.cpp orc_wire_*, restating
engine/comm_manager.cpp:486-590) on the CPU.

The reference's casts cannot be built here (comm_manager.cpp needs libzmq /
cppzmq, absent from the image), so the restatement is pinned to the x86
instruction semantics its SIMD blocks use, modelled independently in numpy:
_mm_packs_epi32 = int32 -> int16 signed saturation, _mm256_cvtepi16_epi32 =
sign extension, _mm256_cvtps_ph(v, 0) = IEEE binary16 round-to-nearest-even
(numpy's float16 cast), _mm256_cvtph_ps = exact widening; and to the scalar
tails' C conversions (the float -> uint16_t tail is GCC's vcvttss2si r32 + a
16-bit store, read from the -O3 -march=broadwell object code of the same
construct).  Parity of the wire format is therefore pinned by ISA semantics,
not by reference output.
"""
from __future__ import annotations

import numpy as np
import pytest


def _simd_end(n):
    return 8 * ((n - 1) // 8) if n else 0


def _model_encode(idx, val, flag):
    n, se = idx.size, _simd_end(idx.size)
    if flag & 1:
        wi = idx.astype(np.uint16)  # tail: (uint16_t) truncation
        wi[:se] = np.clip(idx[:se].view(np.int32), -32768, 32767).astype(np.int16).view(np.uint16)
    else:
        wi = idx.copy()
    if flag & 2:
        with np.errstate(invalid="ignore", over="ignore"):
            wv = val.astype(np.float16).view(np.uint16).copy()
            t = np.full(n, np.int32(-2**31), np.int32)
            ok = np.isfinite(val) & (val > -2147483904.0) & (val < 2147483648.0)
            t[ok] = np.trunc(val[ok]).astype(np.int64).astype(np.int32)
        tail = (t.view(np.uint32) & 0xFFFF).astype(np.uint16)
        wv[se:] = tail[se:]
    else:
        wv = val.copy()
    return wi, wv


def _model_decode(wi, wv, flag):
    n, se = wi.size, _simd_end(wi.size)
    if flag & 1:
        idx = wi.astype(np.uint32)
        idx[:se] = wi[:se].view(np.int16).astype(np.int32).view(np.uint32)
    else:
        idx = wi.copy()
    if flag & 2:
        val = wv.view(np.float16).astype(np.float32)
        val[se:] = wv[se:].astype(np.float32)
    else:
        val = wv.copy()
    return idx, val


def _inputs(n, seed, idx_hi):
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, idx_hi, n, dtype=np.uint32)
    val = (rng.standard_normal(n) * 10.0 ** rng.integers(-9, 6, n)).astype(np.float32)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 65504.0, 65520.0, 6.0e-8, 2.98e-8, -1.7, 3e9, -0.5],
                        np.float32)
    m = min(n, specials.size)
    pos = rng.choice(n, m, replace=False) if n else np.zeros(0, np.int64)
    val[pos] = specials[:m]
    return idx, val


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 16, 17, 100, 4099, 65535])
@pytest.mark.parametrize("flag", [0, 1, 2, 3])
def test_wire_oracle_matches_isa_model(oracle, n, flag):
    idx, val = _inputs(n, n * 7 + flag, 65536)
    wi, wv = oracle.wire_encode(idx, val, flag)
    mi, mv = _model_encode(idx, val, flag)
    assert np.array_equal(wi, mi)
    assert np.array_equal(wv.view(np.uint32 if wv.dtype == np.float32 else np.uint16),
                          mv.view(np.uint32 if mv.dtype == np.float32 else np.uint16))
    di, dv = oracle.wire_decode(wi, wv, flag)
    ei, ev = _model_decode(mi, mv, flag)
    assert np.array_equal(di, ei)
    assert np.array_equal(dv.view(np.uint32), ev.view(np.uint32))


def test_wire_flag_rule(oracle):
    """comm_manager.cpp:578-590: u16 indices below 65536 elements; fp16 values
    only when asked (FP16_COMPRESSION, config.h:64)."""
    assert oracle.wire_flag(65535) == 1 and oracle.wire_flag(65536) == 0
    assert oracle.wire_flag(100, True) == 3 and oracle.wire_flag(1 << 24, True) == 2


def test_wire_u16_round_trip_quirk(oracle):
    """The shipped u16 index path: exact below 32768, saturated to 32767 in the
    SIMD blocks at or above it, exact again in the scalar tail."""
    n = 40  # blocks cover 0..31, tail 32..39
    idx = np.full(n, 40000, np.uint32)
    idx[:4] = [0, 1, 32767, 12345]
    val = np.arange(n, dtype=np.float32)
    wi, wv = oracle.wire_encode(idx, val, 1)
    di, dv = oracle.wire_decode(wi, wv, 1)
    assert list(di[:4]) == [0, 1, 32767, 12345]
    assert np.all(di[4:32] == 32767) and np.all(di[32:] == 40000)
    assert np.array_equal(dv, val)
