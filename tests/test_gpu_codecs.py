"""GPU parity: the HIP codecs (through the C-ABI) against the CPU oracle.

The oracle (oracle/stg_oracle.cpp) is itself pinned bit-exactly to the
reference build (tests/test_oracle_golden.py).  Every case runs a multi-call
AIMD sequence per key so both thresholdv16 regimes (A: filled by the ordered
scan, B: heap fill) and the device-resident state updates are exercised.
"""
from __future__ import annotations

import numpy as np
import pytest

from parity import assert_same_stream, assert_topk_values, bits
from stellatrain_amd.synth import D1, D2, D3, seed_for, synth

pytestmark = pytest.mark.gpu

# (n, k) pairs: whole lines, ragged tails (n % 16 != 0), k % 16 in {0, 7, 15},
# tiny buckets and a multi-tile bucket.
TV16_CASES = [
    (65536, 655, D1, 0),
    (100013, 1007, D1, 0),
    (100013, 1007, D2, 0),
    (1000003, 10000, D1, 0),
    (1000000, 9999, D1, 0),
    (4096 + 7, 40, D1, 0),
    (1000, 7, D1, 0),
    (33, 3, D1, 0),
    (17, 16, D1, 0),
    (262144, 2621, D2, 0),
]


def _regime_split(oracle, src, k, t_before, cnt):
    """Number of leading output slots filled by the ordered scan (regime A part)."""
    sums = oracle.tv16_block_sums(src)
    q = int(np.count_nonzero(sums >= np.float32(t_before)))
    kb = k // 16
    return min(q, kb) * 16


@pytest.mark.parametrize("n,k,dist,param", TV16_CASES)
def test_thresholdv16_parity(gpu, oracle, n, k, dist, param):
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    regimes = set()
    for it in range(10):
        src = synth(n, seed_for(7, it), dist, param)
        t_before = oracle.tv16_state(ho, "3@weight")
        co, io, vo = oracle.tv16_compress(ho, "3@weight", src, k)
        d = torch.from_numpy(src).to(gpu)
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        cg = comp.compress("3@weight", d, k, idx, val)
        assert cg == co
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        # the whole stream, heap fill included (libstdc++ pop order, tv16fill.hip)
        assert_same_stream(ig, vg, io, vo, co)
        so, sg = oracle.tv16_state(ho, "3@weight"), comp.state("3@weight")
        assert bits(np.array(so, np.float32)).tolist() == bits(np.array(sg, np.float32)).tolist()
        if t_before is not None:
            regimes.add("B" if so[0] < t_before[0] else "A")
        head = _regime_split(oracle, src, k, t_before[0], co) if t_before is not None else 0
        assert_same_stream(ig, vg, io, vo, head)
    comp.check_device()
    oracle.tv16_free(ho)


@pytest.mark.parametrize("n,k,dist", [(1 << 20, 10485, D1), (100013, 1007, D1), (262144, 2621, D2)])
def test_thresholdv16_stream_order(gpu, oracle, n, k, dist):
    """Whole output stream in order, bit-exact: the ordered-scan prefix and the
    heap fill in libstdc++ priority_queue pop order (equal line sums occur in
    most regime-B calls of D1 data)."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    tied_fills = 0
    for it in range(8):
        src = synth(n, seed_for(1, it), dist)
        t_before = oracle.tv16_state(ho, "k")
        co, io, vo = oracle.tv16_compress(ho, "k", src, k)
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        assert comp.compress("k", torch.from_numpy(src).to(gpu), k, idx, val) == co
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        head = _regime_split(oracle, src, k, t_before[0], co) if t_before is not None else 0
        assert_same_stream(ig, vg, io, vo, co)
        sums = oracle.tv16_block_sums(src)
        if t_before is not None and head < co:
            ties = np.unique(sums[np.asarray(io[head:co:16], np.int64) // 16 % sums.size], return_counts=True)[1]
            tied_fills += int((ties > 1).any())
    if n == 1 << 20:
        assert tied_fills  # equal line sums inside the heap fill were exercised


@pytest.mark.parametrize("n,k,zp", [(100013, 1007, 9000), (65536, 655, 9995), (1000, 16, 9995), (1 << 20, 10485, 9995)])
def test_thresholdv16_ties_sparse(gpu, oracle, n, k, zp):
    """D3: exact-zero lines tie at sum 0 (99.95 % zeros: the fill reaches
    into them, so the tie sits at the cut and decides the index SET).  The
    whole stream equals the reference's: libstdc++ heap order among ties."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    for it in range(6):
        src = synth(n, seed_for(3, it), D3, zp)
        t_before = oracle.tv16_state(ho, "z")
        co, io, vo = oracle.tv16_compress(ho, "z", src, k)
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        assert comp.compress("z", torch.from_numpy(src).to(gpu), k, idx, val) == co
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        so, sg = oracle.tv16_state(ho, "z"), comp.state("z")
        assert np.float32(so[0]) == np.float32(sg[0]) and np.float32(so[1]) == np.float32(sg[1])
        assert_same_stream(ig, vg, io, vo, co)
        assert np.all(vg[:co] == src[ig[:co]])
        assert len(np.unique(ig[:co])) == co
    comp.check_device()


# (1 << 22) + 3, k = n / 2: about half the elements qualify, so most workgroups'
# LDS lists overflow (csrc/tv.hip tv_steal reads those units again) and the
# ragged tail is non-empty
@pytest.mark.parametrize("n,k,dist", [(100013, 100, D1), (1 << 20, 1048, D1), (1 << 20, 1048, D2), (5000, 4999, D1),
                                      ((1 << 22) + 3, 1 << 21, D1)])
def test_thresholdv_parity(gpu, oracle, n, k, dist):
    import torch
    from stellatrain_amd import ThresholdvCompressor
    comp = ThresholdvCompressor()
    ho = oracle.tv_new()
    d = torch.empty(n, dtype=torch.float32, device=gpu)  # one stable buffer: pointer-keyed state
    for it in range(10):
        src = synth(n, seed_for(5, it), dist)
        co, io, vo = oracle.tv_compress(ho, 1, src, k)
        d.copy_(torch.from_numpy(src))
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        cg = comp.compress("ignored", d, k, idx, val)
        assert cg == co
        assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
        st = comp.state("", key_ptr=d.data_ptr())
        assert np.float32(st[0]) == np.float32(oracle.tv_state(ho, 1))
    comp.check_device()


@pytest.mark.parametrize("n,k", [(100013, 1000), (1 << 20, 10485), (4099, 41), (64, 64)])
def test_topk_bug_compat(gpu, oracle, n, k):
    import torch
    from stellatrain_amd import TopkCompressor
    src = synth(n, seed_for(9, 0))
    co, io, vo = oracle.topk_compress(src, k, bug_compat=True)
    comp = TopkCompressor()
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    assert comp.compress("x", torch.from_numpy(src).to(gpu), k, idx, val) == co
    np.testing.assert_array_equal(idx.cpu().numpy(), np.arange(k))
    assert_topk_values(val.cpu().numpy(), vo)


@pytest.mark.parametrize("n,k,off", [(100013, 1000, 0), (1 << 20, 10485, 77), (4099, 41, 0)])
def test_topk_exact(gpu, oracle, n, k, off):
    import torch
    from stellatrain_amd import TopkCompressor
    src = synth(n, seed_for(11, 0), D2)
    co, io, vo = oracle.topk_compress(src, k, idx_offset=off, bug_compat=False)
    comp = TopkCompressor(exact=True)
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    assert comp.compress("x", torch.from_numpy(src).to(gpu), k, idx, val, off) == co
    assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, k)


def _quantized(n, seed, step):
    """D1 values rounded to multiples of `step`: few distinct magnitudes, so the
    k-th magnitude is tied many times over."""
    x = synth(n, seed).astype(np.float64)
    return (np.round(x / step) * step).astype(np.float32)


# Ties at T: (a) ~1.3k equal keys in T's level-2 bin (the listed select);
# (b) ~26k equal keys (more than the list holds: the level-3 histogram and the
# one-workgroup recount); (c) 90 % zeros with k past the nonzeros (T = 0, every
# tile past its superset capacity); (d) magnitudes in ascending order: every
# key of the top k sits in the last tiles (each of them overflows its
# superset and is re-read).
@pytest.mark.parametrize("case", ["ties_listed", "ties_crowded", "zeros_t0", "sorted"])
@pytest.mark.parametrize("bug_compat", [False, True])
def test_topk_ties(gpu, oracle, case, bug_compat):
    import torch
    from stellatrain_amd import TopkCompressor
    n = 1 << 20
    if case == "ties_listed":
        src, k = _quantized(n, seed_for(13, 0), 5e-6), 10485
    elif case == "ties_crowded":
        src, k = _quantized(n, seed_for(13, 1), 1e-4), 10485
    elif case == "zeros_t0":
        src, k = synth(n, seed_for(13, 2), D3, 9000), 200000
    else:
        x = synth(n, seed_for(13, 3))
        src, k = x[np.argsort(np.abs(x), kind="stable")], 10485
    if bug_compat:
        k = min(k, n // 8) if case != "zeros_t0" else n // 4 + 5000  # past the copied floats: T = 0
    co, io, vo = oracle.topk_compress(src, k, bug_compat=bug_compat)
    comp = TopkCompressor(exact=not bug_compat)
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    assert comp.compress("x", torch.from_numpy(src).to(gpu), k, idx, val) == co
    if bug_compat:
        np.testing.assert_array_equal(idx.cpu().numpy(), np.arange(k))
        assert_topk_values(val.cpu().numpy(), vo)
    else:
        assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, k)
    comp.check_device()


def test_topk_capacity_error(gpu):
    import torch
    from stellatrain_amd import CodecError, TopkCompressor
    comp = TopkCompressor()
    src = torch.zeros(100, device=gpu)
    with pytest.raises(CodecError, match="Invalid parameter k"):
        comp.compress("x", src, 10, torch.zeros(5, dtype=torch.int32, device=gpu), torch.zeros(5, device=gpu))


def test_synth_device_matches_numpy(gpu):
    import ctypes as C

    import torch
    from stellatrain_amd._capi import check, lib
    for dist, param in [(D1, 0), (D2, 0), (D3, 9000)]:
        n = 100003
        d = torch.empty(n, dtype=torch.float32, device=gpu)
        check(lib().stg_synth_fill_device(C.c_void_p(d.data_ptr()), n, 1234 + dist, dist, param, None))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(bits(d.cpu().numpy()), bits(synth(n, 1234 + dist, dist, param)))


def test_host_path_matches_device(gpu, oracle):
    """stg_codec_compress_host (host in/out, H2D + kernels + D2H) == oracle."""
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    n, k = 200003, 2000
    for it in range(4):
        src = synth(n, seed_for(2, it))
        co, io, vo = oracle.tv16_compress(ho, "h", src, k, idx_offset=5)
        idx = np.zeros(k, np.uint32)
        val = np.zeros(k, np.float32)
        assert comp.compress("h", src, k, idx, val, 5) == co
        assert_same_stream(idx, val, io, vo, co)


# Batched launches: several buckets (distinct keys, mixed sizes incl. buckets
# with fewer lines than workgroups, ragged tails, idx offsets) per persistent
# launch, and a repeated key that must split the batch (its second call sees
# the threshold the first call wrote).
BATCH = [
    ("b0@weight", 1000003, 10000, D1, 0),
    ("b1@weight", 65536, 655, D2, 1 << 20),
    ("b2@bias", 1000, 7, D1, 0),
    ("b0@weight", 1000003, 10000, D1, 0),
    ("b3@weight", 4096 + 7, 40, D1, 5),
    ("b4@weight", 262144, 2621, D1, 0),
    ("b5@weight", 33, 3, D1, 0),
]


@pytest.mark.parametrize("layout", ["mixed", "full_batch", "short_chunks"])
def test_thresholdv16_batch(gpu, oracle, layout):
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    iters = 7
    if layout == "mixed":
        spec = BATCH
    elif layout == "full_batch":  # a full batch of 32 distinct keys (MAX_BATCH), then one more: two launches
        spec = [(f"s{i}@w", 131072 + 16 * i + (i % 3), 1311 + i, D1 if i % 2 else D2, 0) for i in range(33)]
    else:
        # more chunks than two per workgroup (dynamic chunk takes) and every
        # bucket ending in a short chunk: streaming waves with no lines there
        # must not take chunks out of order (the C4 layout's failure mode)
        spec = [(f"c{i}@w", (65 << 15) + 16 * 37 * i + 5 + 16 * (i % 4), 21300 + i, D1, 0) for i in range(16)]
        iters = 4
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    for it in range(iters):
        items, ref = [], []
        for j, (key, n, k, dist, off) in enumerate(spec):
            src = synth(n, seed_for(40 + j, it), dist)
            t_before = oracle.tv16_state(ho, key)
            co, io, vo = oracle.tv16_compress(ho, key, src, k, idx_offset=off)
            ref.append((src, co, io, vo, t_before, oracle.tv16_state(ho, key)))
            items.append((key, torch.from_numpy(src).to(gpu), k, torch.zeros(k, dtype=torch.int32, device=gpu),
                          torch.zeros(k, dtype=torch.float32, device=gpu), off))
        counts = comp.compress_batch_async(items).cpu().numpy()
        torch.cuda.synchronize()
        for j, ((key, _, k, idx, val, off), (src, co, io, vo, t_before, _)) in enumerate(zip(items, ref)):
            assert counts[j] == co, (it, j)
            ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
            assert_same_stream(ig, vg, io, vo, co)
        # final state of every key equals the oracle's after its last call
        last = {}
        for (key, *_), r in zip(spec, ref):
            last[key] = r[5]
        for key, so in last.items():
            sg = comp.state(key)
            assert bits(np.array(so, np.float32)).tolist() == bits(np.array(sg, np.float32)).tolist(), key
    comp.check_device()
    oracle.tv16_free(ho)


def test_thresholdv16_batch_64mib(gpu, oracle):
    """The bench workload: 8 x 64 MiB buckets per launch, k = 1%, against the
    oracle for two keys of the batch over an AIMD sequence (both regimes)."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd.synth import seed_for as sf
    n = 16 << 20
    k = merge_numel(n, 0.99)
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    keys = [f"{i}@weight" for i in range(8)]
    outs = [(torch.zeros(k, dtype=torch.int32, device=gpu), torch.zeros(k, dtype=torch.float32, device=gpu))
            for _ in keys]
    regimes = set()
    for it in range(6):
        srcs = [synth(n, sf(i, it)) if i in (0, 5) else None for i in range(8)]
        dev = []
        for i in range(8):
            t = torch.empty(n, dtype=torch.float32, device=gpu)
            if srcs[i] is not None:
                t.copy_(torch.from_numpy(srcs[i]))
            else:
                from stellatrain_amd._capi import lib
                import ctypes as C
                lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, sf(i, it), 0, 0,
                                            C.c_void_p(torch.cuda.current_stream().cuda_stream))
            dev.append(t)
        counts = comp.compress_batch_async(
            [(keys[i], dev[i], k, outs[i][0], outs[i][1]) for i in range(8)]).cpu().numpy()
        assert (counts == k).all()
        for i in (0, 5):
            t_before = oracle.tv16_state(ho, keys[i])
            co, io, vo = oracle.tv16_compress(ho, keys[i], srcs[i], k)
            ig, vg = outs[i][0].cpu().numpy().view(np.uint32), outs[i][1].cpu().numpy()
            assert_same_stream(ig, vg, io, vo, co)
            so = oracle.tv16_state(ho, keys[i])
            assert bits(np.array(so, np.float32)).tolist() == bits(np.array(comp.state(keys[i]), np.float32)).tolist()
            if t_before is not None:
                regimes.add("B" if so[0] < t_before[0] else "A")
    comp.check_device()
    oracle.tv16_free(ho)
    assert regimes  # at least one steady-state call compared


@pytest.mark.parametrize("n,k,dist,param", [((1 << 21) + 5, 209715, D1, 0), (1 << 20, 1 << 17, D3, 9000)])
def test_thresholdv16_large_fill(gpu, oracle, n, k, dist, param):
    """Regime B far from the window: the inputs' scale drops 100x between
    calls, so the ordered scan finds almost nothing above the threshold and
    the heap fill (tv16fill.hip full path: the literal make_heap / pop_heap)
    emits up to k/16 lines.  D3 adds exact-zero ties at the cut."""
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    big = 0
    for it, scale in enumerate([1.0, 1.0, 0.01, 1.0, 0.3, 0.003, 0.003]):
        src = (synth(n, seed_for(11, it), dist, param) * np.float32(scale)).astype(np.float32)
        t_before = oracle.tv16_state(ho, "f")
        co, io, vo = oracle.tv16_compress(ho, "f", src, k)
        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        assert comp.compress("f", torch.from_numpy(src).to(gpu), k, idx, val) == co
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        so, sg = oracle.tv16_state(ho, "f"), comp.state("f")
        assert bits(np.array(so, np.float32)).tolist() == bits(np.array(sg, np.float32)).tolist(), it
        head = _regime_split(oracle, src, k, t_before[0], co) if t_before is not None else 0
        if t_before is not None and (co - head) // 16 > 4095:  # more than the window path could hold
            big += 1
        assert_same_stream(ig, vg, io, vo, co)
    comp.check_device()
    oracle.tv16_free(ho)
    assert big  # at least one call filled more than one piece
