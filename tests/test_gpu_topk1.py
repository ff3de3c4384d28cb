"""Top-k in one pass over the bucket, steered by the key's last k-th magnitude (topk1.hip).

A key's first call takes the select's launches (topk.hip); later calls stream
the bucket once against a band around the last k-th magnitude and resolve T
inside it; a band that misses (the magnitudes jump) falls back to the select
inside the emission launch and widens.  Every call is checked against the oracle:
the whole stream for the corrected mode, the signed value multiset (freedom
only at the k-th magnitude) for the shipped mode.  Debug words 38 / 39 count
calls resolved in the band / by the select.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from parity import assert_same_stream, assert_topk_values
from stellatrain_amd.synth import D1, D3, seed_for, synth

pytestmark = pytest.mark.gpu


def _words(comp):
    import torch
    from stellatrain_amd._capi import check, lib
    w = (C.c_uint32 * 64)()
    check(lib().stg_codec_debug_words(comp._h, C.c_void_p(torch.cuda.current_stream().cuda_stream), w, 64))
    return list(w)


def _check(gpu, oracle, comp, key, src, k, bug_compat, off=0):
    import torch
    co, io, vo = oracle.topk_compress(src, k, idx_offset=off, bug_compat=bug_compat)
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    assert comp.compress(key, torch.from_numpy(src).to(gpu), k, idx, val, off) == co
    if bug_compat:
        np.testing.assert_array_equal(idx.cpu().numpy(), np.arange(k))
        assert_topk_values(val.cpu().numpy(), vo)
    else:
        assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, k)


@pytest.mark.parametrize("bug_compat", [False, True])
def test_hint_sequence(gpu, oracle, bug_compat):
    """First call, steady calls (band hits), a 10x jump (miss, widen), steady
    again, a 10x drop (miss), steady; ragged n, idx_offset."""
    from stellatrain_amd import TopkCompressor
    comp = TopkCompressor(exact=not bug_compat)
    n, k = (1 << 21) + 17, 20971
    scales = [1, 1, 1, 1, 10, 10, 10, 1, 1]
    for c, sc in enumerate(scales):
        src = synth(n, seed_for(310, c), D1) * np.float32(sc)
        _check(gpu, oracle, comp, "w", src, k, bug_compat, off=0 if bug_compat else 33)
    comp.check_device()
    w = _words(comp)
    hits, sel = w[38], w[39]
    assert sel == 3 and hits == 6, (hits, sel)  # the first call and the two jumps: the select's way


@pytest.mark.parametrize("case", ["ties_listed", "ties_crowded", "zeros_t0", "sorted"])
@pytest.mark.parametrize("bug_compat", [False, True])
def test_hint_ties(gpu, oracle, case, bug_compat):
    """test_gpu_codecs.test_topk_ties's inputs, each compressed three times
    under one key (the later calls with the hint)."""
    n = 1 << 20
    if case == "ties_listed":
        x = synth(n, seed_for(13, 0)).astype(np.float64)
        src, k = (np.round(x / 5e-6) * 5e-6).astype(np.float32), 10485
    elif case == "ties_crowded":
        x = synth(n, seed_for(13, 1)).astype(np.float64)
        src, k = (np.round(x / 1e-4) * 1e-4).astype(np.float32), 10485
    elif case == "zeros_t0":
        src, k = synth(n, seed_for(13, 2), D3, 9000), 200000
    else:
        x = synth(n, seed_for(13, 3))
        src, k = x[np.argsort(np.abs(x), kind="stable")], 10485
    if bug_compat:
        k = min(k, n // 8) if case != "zeros_t0" else n // 4 + 5000
    from stellatrain_amd import TopkCompressor
    comp = TopkCompressor(exact=not bug_compat)
    for _ in range(3):
        _check(gpu, oracle, comp, "t", src, k, bug_compat)
    comp.check_device()


def test_c2_steady_64mib(gpu, oracle):
    """C2's bucket (64 MiB, k = 1 %): four calls on fresh data under one key,
    both modes."""
    from stellatrain_amd import TopkCompressor
    n, k = 16 << 20, 167772
    for bug_compat in (False, True):
        comp = TopkCompressor(exact=not bug_compat)
        for c in range(4):
            _check(gpu, oracle, comp, "c2", synth(n, seed_for(320, c), D1), k, bug_compat)
        comp.check_device()
        w = _words(comp)
        assert w[38] >= 3 and w[39] == 1, w[36:40]


@pytest.mark.parametrize("bug_compat", [False, True])
def test_interleaved_keys(gpu, oracle, bug_compat):
    """Keys appearing between hinted calls on one workspace: A, B, A, C, B, C,
    D, A, ...  A key's first call runs the select's launches (no emission
    launch), so the control block's call parity must move only with hinted
    calls; every call against the oracle."""
    from stellatrain_amd import TopkCompressor
    comp = TopkCompressor(exact=not bug_compat)
    n, k = (1 << 20) + 5, 10485
    order = ["A", "B", "A", "C", "B", "C", "D", "A", "E", "B", "D", "E", "A", "F", "A"]
    calls = {}
    for key in order:
        c = calls.get(key, 0)
        calls[key] = c + 1
        src = synth(n, seed_for(330 + ord(key), c), D1)
        _check(gpu, oracle, comp, key, src, k, bug_compat)
    comp.check_device()
    w = _words(comp)
    # every first call takes the select's way; hinted calls mostly hit (at
    # this size a fresh bucket's k-th magnitude can land outside the band)
    assert w[39] >= len(calls) and w[38] >= len(order) - 2 * len(calls), w[36:40]


@pytest.mark.parametrize("bug_compat", [False, True])
def test_k_zero(gpu, oracle, bug_compat):
    """k = 0 on a bucket the one-pass path covers (topk.cpp accepts it: the
    count is the capacity, nothing written), first and hinted calls, and a
    hinted call after it still exact."""
    import torch
    from stellatrain_amd import TopkCompressor
    comp = TopkCompressor(exact=not bug_compat)
    n, k = 1 << 20, 10485
    src = synth(n, seed_for(340, 0), D1)
    _check(gpu, oracle, comp, "z", src, k, bug_compat)
    for key in ("z", "fresh"):
        idx = torch.zeros(4, dtype=torch.int32, device=gpu)
        val = torch.zeros(4, dtype=torch.float32, device=gpu)
        d = torch.from_numpy(src).to(gpu)
        assert comp.compress(key, d, 0, idx, val, 0) == 4  # count = dst_idx.second (topk.cpp:25)
        assert not idx.any() and not val.any()
    _check(gpu, oracle, comp, "z", synth(n, seed_for(340, 1), D1), k, bug_compat)
    _check(gpu, oracle, comp, "fresh", synth(n, seed_for(340, 2), D1), k, bug_compat)
    comp.check_device()
