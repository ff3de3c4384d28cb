"""Synthetic fp32 gradient buckets, integer-only.

``numpy`` twin of ``stg_synth_fill_device`` (csrc/synth.hip): splitmix64,
Irwin-Hall(4) of 24-bit uniforms, centred, * 2^-24 * 1e-3 in double, rounded
once to float32.  D2 scales by 2^-e (e = U{0..8}); D3 zeroes an element with
probability param/1e4.  Bit-identical on CPU and GPU (tests/test_synth.py).
"""
from __future__ import annotations

import numpy as np

D1, D2, D3 = 0, 1, 2
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def synth(n: int, seed: int, dist: int = D1, param: int = 0, chunk: int = 1 << 22) -> np.ndarray:
    out = np.empty(n, np.float32)
    scale = 1e-3 / 16777216.0
    m24 = np.uint64(0xFFFFFF)
    with np.errstate(over="ignore"):
        sb = np.uint64(seed) * np.uint64(0x100000001B3)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        i = np.arange(lo, hi, dtype=np.uint64)
        with np.errstate(over="ignore"):
            base = sb + i * np.uint64(4)
            r0 = _splitmix64(base)
            r1 = _splitmix64(base + np.uint64(1))
        v = ((r0 & m24).astype(np.int64) + ((r0 >> np.uint64(24)) & m24).astype(np.int64) +
             (r1 & m24).astype(np.int64) + ((r1 >> np.uint64(24)) & m24).astype(np.int64) - (1 << 25))
        x = v.astype(np.float64) * scale
        if dist == D2:
            e = ((r1 >> np.uint64(48)) % np.uint64(9)).astype(np.int64)
            x = x * (1.0 / np.exp2(e.astype(np.float64)))
        elif dist == D3:
            z = ((r0 >> np.uint64(48)) % np.uint64(10000)).astype(np.int64)
            x = np.where(z < param, 0.0, x)
        out[lo:hi] = x.astype(np.float32)
    return out


def seed_for(bucket: int, it: int) -> int:
    """Seed schedule of SURVEY 8(d): 0x5EED0000 + bucket*1000 + iter."""
    return 0x5EED0000 + bucket * 1000 + it
