"""Comparison helpers shared by the parity tests (test infrastructure)."""
from __future__ import annotations

import numpy as np


def bits(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def fbits(x) -> int:
    """Bit pattern of one float32 scalar."""
    return int(np.float32(x).view(np.uint32))


def assert_same_pairs(idx_a, val_a, idx_b, val_b, n: int):
    """Bit-exact equality of the first n (idx, val) pairs as sets (order-free)."""
    ia, ib = np.asarray(idx_a[:n], np.uint32), np.asarray(idx_b[:n], np.uint32)
    oa, ob = np.argsort(ia, kind="stable"), np.argsort(ib, kind="stable")
    np.testing.assert_array_equal(ia[oa], ib[ob])
    np.testing.assert_array_equal(bits(val_a[:n])[oa], bits(val_b[:n])[ob])


def assert_same_stream(idx_a, val_a, idx_b, val_b, n: int, what: str = ""):
    """Bit-exact equality of the first n pairs in order.  On a mismatch the
    message names `what` (side, call, regime ...), the first differing
    position, the number of differing entries and the last indices of both."""
    ia, ib = np.asarray(idx_a[:n], np.uint32), np.asarray(idx_b[:n], np.uint32)
    va, vb = bits(val_a[:n]), bits(val_b[:n])
    bad = np.flatnonzero((ia != ib) | (va != vb)) if ia.size == ib.size else np.arange(n)
    if bad.size:
        f = int(bad[0])
        raise AssertionError(
            f"{what}: {bad.size} of {n} pairs differ, first at {f} "
            f"(idx {ia[f:f + 4].tolist()} vs {ib[f:f + 4].tolist()}); "
            f"stream ends {ia[-3:].tolist()} vs {ib[-3:].tolist()}")


def canonical_heap_order(idx, val, head: int, count: int, src: np.ndarray, oracle):
    """Re-order the heap-fill segment [head, count) by (line sum desc, index asc).

    The reference pops equal sums in libstdc++ heap order, the GPU in position
    order; with this canonical form both streams must be bit-identical."""
    idx = np.asarray(idx[:count], np.uint32).copy()
    val = np.ascontiguousarray(val[:count], np.float32).copy()
    sums = oracle.tv16_block_sums(src)
    nb = sums.size
    seg_i = idx[head:].astype(np.int64)
    line = seg_i // 16
    tl = src.size % 16
    key = np.empty(seg_i.size, np.float64)
    full = line < nb
    key[full] = sums[line[full]]
    if (~full).any():  # ragged tail line: signed sum * 16 / tl (thresholdv16.cpp:232)
        s = np.float32(0)
        for x in src[nb * 16:]:
            s = np.float32(s + x)
        key[~full] = np.float32(np.float32(s * np.float32(16)) / np.float32(tl))
    order = np.lexsort((seg_i, -key))
    idx[head:] = idx[head:][order]
    val[head:] = val[head:][order]
    return idx, val


def line_keys(src: np.ndarray, idx: np.ndarray, oracle) -> np.ndarray:
    """Tree-order 16-float line sums of the lines the indices start."""
    sums = oracle.tv16_block_sums(src)
    lines = np.asarray(idx, np.int64) // 16
    keep = lines < sums.size
    return np.sort(sums[lines[keep]])


def assert_topk_values(vg, vo):
    """Same-cardinality top-k values (topk.cpp:28-46 partition order is free):
    the SIGNED bit patterns agree as a multiset, except that among exact |x|
    ties at the k-th magnitude either sign may have been kept."""
    vg, vo = np.asarray(vg, np.float32), np.asarray(vo, np.float32)
    assert vg.size == vo.size
    cut = np.abs(vo).min() if vo.size else np.float32(0)
    assert np.abs(vg).min() == cut if vg.size else True
    above_g, above_o = vg[np.abs(vg) > cut], vo[np.abs(vo) > cut]
    np.testing.assert_array_equal(np.sort(bits(above_g)), np.sort(bits(above_o)))
    assert np.count_nonzero(np.abs(vg) == cut) == np.count_nonzero(np.abs(vo) == cut)
