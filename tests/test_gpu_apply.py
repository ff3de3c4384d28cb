"""GPU parity of the config-5 inverse path: MERGE decompress + sparse SGD.

* ``stg_scatter_merge_device`` against the oracle restatement of
  ``ModuleCpuOptimize::run`` MERGE (engine/modules/cpu_optimize.cpp:40-72):
  rank-ordered index_put_ into a dense zero tensor, sum, / world, gathered at
  the union of the indices (output index-ascending on both sides).
* ``stg_sgd_optimize_raw_device`` against the oracle restatement of
  ``SGD::optimize_raw`` (optim/sgd.cpp:34-263) -- the oracle's SGD is itself
  pinned bit-exactly to the reference build (tests/test_oracle_golden.py).
* The whole C5 round trip (compress -> decompress -> SGD apply, 3 steps) and
  the error-feedback residual of ``ModuleCompress::run``
  (engine/modules/compress.cpp:172-186).

All comparisons are bit-exact (integer indices and fp32 bit patterns).
"""
from __future__ import annotations

import numpy as np
import pytest

from parity import assert_same_stream
from stellatrain_amd.synth import D1, D2, seed_for, synth

pytestmark = pytest.mark.gpu


def _sorted_pairs(idx, val):
    idx = np.asarray(idx).view(np.uint32)
    o = np.argsort(idx, kind="stable")
    return idx[o], np.asarray(val, np.float32)[o]


def _rank_streams(n, per_rank, world, seed, overlap):
    """world rank streams of unique indices each; with ``overlap`` the ranks
    share half of their indices (the merge's sum path)."""
    rng = np.random.default_rng(seed)
    shared = rng.choice(n, per_rank // 2, replace=False) if overlap else np.zeros(0, np.int64)
    idx, val = [], []
    for r in range(world):
        rest = np.setdiff1d(np.arange(n), shared)
        own = rng.choice(rest, per_rank - shared.size, replace=False)
        ii = np.concatenate([shared, own]).astype(np.uint32)
        rng.shuffle(ii)
        idx.append(ii)
        val.append(synth(per_rank, seed_for(40 + r, seed)) * np.float32(1000))
    return np.concatenate(idx), np.concatenate(val)


@pytest.mark.parametrize("n,per_rank,world,overlap", [
    (65536, 655, 1, False),
    (100013, 1000, 2, True),
    (100013, 1000, 4, True),
    (1 << 20, 10485, 8, True),
    (4099, 41, 3, False),
])
def test_scatter_merge_parity(gpu, oracle, n, per_rank, world, overlap):
    import torch
    from stellatrain_amd import scatter_merge
    from stellatrain_amd.engine import scatter_merge_check
    idx, val = _rank_streams(n, per_rank, world, 5, overlap)
    oi, ov = oracle.merge_decompress(idx, val, per_rank, world, n)
    di = torch.from_numpy(idx.view(np.int32)).to(gpu)
    dv = torch.from_numpy(val).to(gpu)
    dense = torch.zeros(n, dtype=torch.float32, device=gpu)
    mark = torch.zeros(n, dtype=torch.uint8, device=gpu)
    out_i, out_v, cnt = scatter_merge(di, dv, per_rank, world, n, dense=dense, mark=mark)
    m = int(cnt.item())
    assert m == oi.size
    gi, gv = _sorted_pairs(out_i[:m].cpu().numpy(), out_v[:m].cpu().numpy())
    ei, ev = _sorted_pairs(oi, ov)
    assert np.array_equal(gi, ei)
    assert np.array_equal(gv.view(np.uint32), ev.view(np.uint32))
    # scratch is handed back zeroed (the next bucket reuses it)
    assert int(torch.count_nonzero(dense).item()) == 0
    assert int(torch.count_nonzero(mark).item()) == 0
    scatter_merge_check()  # no device failure on this stream's scratch


@pytest.mark.parametrize("case", __import__("merge_golden").MANIFEST_MERGE["merge"], ids=lambda c: c["name"])
def test_scatter_merge_torch_goldens(gpu, case):
    """The HIP MERGE decompress against torch's own CPU kernels running
    cpu_optimize.cpp:40-72 (tests/golden/make_golden_merge.py): world 1-8,
    shared and disjoint indices, -0.0 values, a rank stream with repeated
    indices, and C5's 64 MiB bucket at world 2/4/8."""
    import torch
    from merge_golden import merge_case_check, merge_case_inputs
    from stellatrain_amd import scatter_merge
    from stellatrain_amd.engine import scatter_merge_check
    idx, val = merge_case_inputs(case)
    n = case["n"]
    dense = torch.zeros(n, dtype=torch.float32, device=gpu)
    mark = torch.zeros(n, dtype=torch.uint8, device=gpu)
    out_i, out_v, cnt = scatter_merge(torch.from_numpy(idx.view(np.int32)).to(gpu), torch.from_numpy(val).to(gpu),
                                      case["per_rank"], case["world"], n, dense=dense, mark=mark)
    m = int(cnt.item())
    merge_case_check(case, out_i[:m].cpu().numpy(), out_v[:m].cpu().numpy())
    assert int(torch.count_nonzero(dense).item()) == 0
    assert int(torch.count_nonzero(mark).item()) == 0
    scatter_merge_check()


def test_scatter_merge_world1_duplicates(gpu, oracle):
    """World 1 takes a copy path when no index repeats and the election path
    when one does (csrc/apply.hip win_mark's duplicate flag): alternate
    duplicate-free and duplicated streams on one stream's scratch, each against
    the oracle (last occurrence wins, cpu_optimize.cpp:46-50), the flag cleared
    between them."""
    import torch
    from stellatrain_amd import scatter_merge
    from stellatrain_amd.engine import scatter_merge_check
    n, per_rank = 100013, 20000
    rng = np.random.default_rng(11)
    for it, dups in enumerate([False, True, False, True, True, False]):
        idx = rng.choice(n, per_rank, replace=False).astype(np.uint32)
        if dups:  # every 7th pair repeats an earlier index of the stream
            src = rng.integers(0, per_rank // 2, per_rank // 7)
            idx[per_rank // 2:per_rank // 2 + src.size] = idx[src]
        val = synth(per_rank, seed_for(61, it)) * np.float32(100)
        oi, ov = oracle.merge_decompress(idx, val, per_rank, 1, n)
        out_i, out_v, cnt = scatter_merge(torch.from_numpy(idx.view(np.int32)).to(gpu), torch.from_numpy(val).to(gpu),
                                          per_rank, 1, n)
        m = int(cnt.item())
        assert m == oi.size, (it, dups)
        gi, gv = _sorted_pairs(out_i[:m].cpu().numpy(), out_v[:m].cpu().numpy())
        ei, ev = _sorted_pairs(oi, ov)
        assert np.array_equal(gi, ei) and np.array_equal(gv.view(np.uint32), ev.view(np.uint32)), (it, dups)
        if not dups:  # the copy path keeps the stream's order
            assert np.array_equal(out_i[:m].cpu().numpy().view(np.uint32), idx)
    scatter_merge_check()


def test_scatter_merge_release_and_reuse(gpu, oracle):
    """The per-(device, stream) MERGE scratch can be released and is rebuilt
    by the next call on that stream (world 1: the one-launch look-back path)."""
    import torch
    from stellatrain_amd import scatter_merge
    from stellatrain_amd.engine import scatter_merge_check, scatter_merge_release
    n, per_rank = 100013, 5000
    idx, val = _rank_streams(n, per_rank, 1, 7, 0.3)
    oi, ov = oracle.merge_decompress(idx, val, per_rank, 1, n)
    di = torch.from_numpy(idx.view(np.int32)).to(gpu)
    dv = torch.from_numpy(val).to(gpu)
    for _ in range(2):
        out_i, out_v, cnt = scatter_merge(di, dv, per_rank, 1, n)
        m = int(cnt.item())
        assert m == oi.size
        gi, gv = _sorted_pairs(out_i[:m].cpu().numpy(), out_v[:m].cpu().numpy())
        ei, ev = _sorted_pairs(oi, ov)
        assert np.array_equal(gi, ei) and np.array_equal(gv.view(np.uint32), ev.view(np.uint32))
        scatter_merge_check()
        scatter_merge_release()
    scatter_merge_release()  # nothing left: a no-op


SGD_CASES = [
    dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0, nesterov=False),
    dict(lr=0.05, momentum=0.9, dampening=0.1, weight_decay=1e-4, nesterov=True),
    dict(lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False),
    dict(lr=0.02, momentum=0.5, dampening=0.0, weight_decay=5e-4, nesterov=False),
]


@pytest.mark.parametrize("opt", SGD_CASES, ids=lambda o: f"m{o['momentum']}_n{int(o['nesterov'])}_wd{o['weight_decay']}")
def test_sgd_apply_parity(gpu, oracle, opt):
    import torch
    from stellatrain_amd import SparseSGD
    n, k = 100013, 1000
    param0 = synth(n, seed_for(23, 99)) * np.float32(1000)
    po = param0.copy()
    pg = torch.from_numpy(param0.copy()).to(gpu)
    ho = oracle.sgd_new(**opt)
    sgd = SparseSGD(**opt)
    rng = np.random.default_rng(3)
    for step in range(4):
        # steps 0-1 hit the same index set (momentum re-use); 2-3 a fresh one
        if step % 2 == 0:
            gidx = np.sort(rng.choice(n, k, replace=False)).astype(np.uint32)
        g = synth(k, seed_for(31, step)) * np.float32(100)
        oracle.sgd_apply(ho, "fc@weight", po, g, gidx)
        sgd.optimize_raw(pg, "fc@weight", torch.from_numpy(g).to(gpu),
                         torch.from_numpy(gidx.view(np.int32)).to(gpu))
        got = pg.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), po.view(np.uint32)), f"param differs at step {step}"
    mo = oracle.sgd_momentum(ho, "fc@weight", n)
    mg = sgd.momentum_buffer("fc@weight", n)
    if mo is None:
        assert mg is None
    else:
        assert np.array_equal(mg.view(np.uint32), mo.view(np.uint32))
    oracle.sgd_free(ho)


@pytest.mark.parametrize("n,dist,param", [(1 << 20, D1, 0), (100013, D1, 0), (262144, D2, 0)])
def test_round_trip_compress_decompress_sgd(gpu, oracle, n, dist, param):
    """C5 at test size: thresholdv16 compress -> MERGE decompress (world 1) ->
    momentum SGD, three iterations, param and momentum bit-exact."""
    import torch
    from stellatrain_amd import SparseSGD, ThresholdvCompressor16, merge_numel, scatter_merge
    k = merge_numel(n, 0.99)
    opt = dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0, nesterov=False)
    comp = ThresholdvCompressor16()
    sgd = SparseSGD(**opt)
    hc, hs = oracle.tv16_new(), oracle.sgd_new(**opt)
    param0 = synth(n, seed_for(23, 99)) * np.float32(1000)
    po, pg = param0.copy(), torch.from_numpy(param0.copy()).to(gpu)
    for it in range(3):
        src = synth(n, seed_for(11, it), dist, param)
        co, io, vo = oracle.tv16_compress(hc, "rt@weight", src, k)
        mi, mv = oracle.merge_decompress(io[:co], vo[:co], co, 1, n)
        oracle.sgd_apply(hs, "rt@weight", po, mv, mi)

        idx = torch.zeros(k, dtype=torch.int32, device=gpu)
        val = torch.zeros(k, dtype=torch.float32, device=gpu)
        cg = comp.compress("rt@weight", torch.from_numpy(src).to(gpu), k, idx, val)
        assert cg == co
        oi, ov, cnt = scatter_merge(idx, val, k, 1, n)
        m = int(cnt.item())
        assert m == mi.size
        sgd.optimize_raw(pg, "rt@weight", ov[:m], oi[:m])
        got = pg.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), po.view(np.uint32)), f"param differs at iteration {it}"
    mo = oracle.sgd_momentum(hs, "rt@weight", n)
    mg = sgd.momentum_buffer("rt@weight", n)
    assert np.array_equal(mg.view(np.uint32), mo.view(np.uint32))
    oracle.tv16_free(hc)
    oracle.sgd_free(hs)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("opt", SGD_CASES[:2], ids=lambda o: f"m{o['momentum']}_n{int(o['nesterov'])}")
def test_merge_optimize_sgd_fused(gpu, oracle, world, opt):
    """ModuleCpuOptimize::run in one call (cpu_optimize.cpp:26-100): the merged
    stream, the parameters and the momentum equal the oracle's decompress +
    optimize_raw bit for bit over three iterations (world 1: the step runs in
    the emission launch; world 2: the two calls)."""
    import torch
    from stellatrain_amd import SparseSGD, ThresholdvCompressor16, merge_numel
    n = (1 << 20) + 5
    k = merge_numel(n, 0.99)
    comp = ThresholdvCompressor16()
    sgd = SparseSGD(**opt)
    hc, hs = oracle.tv16_new(), oracle.sgd_new(**opt)
    param0 = synth(n, seed_for(23, 98)) * np.float32(1000)
    po, pg = param0.copy(), torch.from_numpy(param0.copy()).to(gpu)
    for it in range(3):
        ios, vos, igs, vgs = [], [], [], []
        for r in range(world):  # each rank's stream (the same codec, one key per rank)
            src = synth(n, seed_for(17 + r, it))
            co, io, vo = oracle.tv16_compress(hc, f"m{r}@weight", src, k)
            idx = torch.zeros(k, dtype=torch.int32, device=gpu)
            val = torch.zeros(k, dtype=torch.float32, device=gpu)
            assert comp.compress(f"m{r}@weight", torch.from_numpy(src).to(gpu), k, idx, val) == co
            ios.append(io[:k]); vos.append(vo[:k]); igs.append(idx); vgs.append(val)
        mi, mv = oracle.merge_decompress(np.concatenate(ios), np.concatenate(vos), k, world, n)
        oracle.sgd_apply(hs, "m@weight", po, mv, mi)
        oi, ov, cnt = sgd.merge_optimize(pg, "m@weight", torch.cat(igs), torch.cat(vgs), k, world)
        m = int(cnt.item())
        assert m == mi.size
        gi, gv = oi[:m].cpu().numpy().view(np.uint32), ov[:m].cpu().numpy()
        ei, ev = _sorted_pairs(gi, gv)
        xi, xv = _sorted_pairs(mi.astype(np.uint32), mv)
        assert np.array_equal(ei, xi) and np.array_equal(ev.view(np.uint32), xv.view(np.uint32))
        got = pg.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), po.view(np.uint32)), f"param differs at iteration {it}"
    mo = oracle.sgd_momentum(hs, "m@weight", n)
    mg = sgd.momentum_buffer("m@weight", n)
    if mo is None:
        assert mg is None
    else:
        assert np.array_equal(mg.view(np.uint32), mo.view(np.uint32))
    oracle.tv16_free(hc)
    oracle.sgd_free(hs)


def test_merge_optimize_sgd_world1_duplicates(gpu, oracle):
    """The step fused into the world-1 emission on both of its paths: streams
    with repeated indices (the election path) and without (the copy path),
    alternating on one scratch; parameters and momentum bit-exact against the
    oracle's decompress + optimize_raw."""
    import torch
    from stellatrain_amd import SparseSGD
    n, per_rank = 100013, 20000
    opt = dict(lr=0.05, momentum=0.9, dampening=0.1, weight_decay=1e-4, nesterov=True)
    sgd = SparseSGD(**opt)
    hs = oracle.sgd_new(**opt)
    param0 = synth(n, seed_for(23, 97)) * np.float32(1000)
    po, pg = param0.copy(), torch.from_numpy(param0.copy()).to(gpu)
    rng = np.random.default_rng(12)
    for it, dups in enumerate([True, False, True, False]):
        idx = rng.choice(n, per_rank, replace=False).astype(np.uint32)
        if dups:
            src = rng.integers(0, per_rank // 2, per_rank // 7)
            idx[per_rank // 2:per_rank // 2 + src.size] = idx[src]
        val = synth(per_rank, seed_for(62, it)) * np.float32(100)
        mi, mv = oracle.merge_decompress(idx, val, per_rank, 1, n)
        oracle.sgd_apply(hs, "d@weight", po, mv, mi)
        oi, ov, cnt = sgd.merge_optimize(pg, "d@weight", torch.from_numpy(idx.view(np.int32)).to(gpu),
                                         torch.from_numpy(val).to(gpu), per_rank, 1)
        assert int(cnt.item()) == mi.size, (it, dups)
        assert np.array_equal(pg.cpu().numpy().view(np.uint32), po.view(np.uint32)), (it, dups)
    mo = oracle.sgd_momentum(hs, "d@weight", n)
    assert np.array_equal(sgd.momentum_buffer("d@weight", n).view(np.uint32), mo.view(np.uint32))
    oracle.sgd_free(hs)


@pytest.mark.parametrize("amsgrad", [False, True])
def test_merge_optimize_adam_world1(gpu, oracle, amsgrad):
    """SparseAdam.merge_optimize at world 1 (the step in the emission launch;
    amsgrad: the decompress, then the ordered step), duplicated and
    duplicate-free streams alternating: parameters, m, v and vmax bit-exact
    against the oracle's decompress + optimize_raw."""
    import torch
    from stellatrain_amd import SparseAdam
    n, per_rank = 100013, 20000
    opt = dict(lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, weight_decay=1e-4, amsgrad=amsgrad)
    adam = SparseAdam(**opt)
    ha = oracle.adam_new(**opt)
    param0 = synth(n, seed_for(23, 96)) * np.float32(10)
    po, pg = param0.copy(), torch.from_numpy(param0.copy()).to(gpu)
    rng = np.random.default_rng(13)
    for it, dups in enumerate([False, True, False, True]):
        idx = rng.choice(n, per_rank, replace=False).astype(np.uint32)
        if dups:
            src = rng.integers(0, per_rank // 2, per_rank // 7)
            idx[per_rank // 2:per_rank // 2 + src.size] = idx[src]
        val = synth(per_rank, seed_for(63, it))
        mi, mv = oracle.merge_decompress(idx, val, per_rank, 1, n)
        oi, ov, cnt = adam.merge_optimize(pg, "a@weight", torch.from_numpy(idx.view(np.int32)).to(gpu),
                                          torch.from_numpy(val).to(gpu), per_rank, 1)
        m = int(cnt.item())
        assert m == mi.size, (it, dups)
        gi, gv = oi[:m].cpu().numpy().view(np.uint32), ov[:m].cpu().numpy()
        ei, ev = _sorted_pairs(gi, gv)
        xi, xv = _sorted_pairs(mi.astype(np.uint32), mv)
        assert np.array_equal(ei, xi) and np.array_equal(ev.view(np.uint32), xv.view(np.uint32)), (it, dups)
        # amsgrad's running maximum follows the stream's order, which the
        # reference leaves to unordered_set (cpu_optimize.cpp:14-24): the step is
        # checked on the merged stream in the order it was emitted
        if amsgrad:
            oracle.adam_apply(ha, "a@weight", po, gv, gi)
        else:
            oracle.adam_apply(ha, "a@weight", po, mv, mi)
        assert np.array_equal(pg.cpu().numpy().view(np.uint32), po.view(np.uint32)), (it, dups)
    adam.check_device()
    mo, vo, vmo, _ = oracle.adam_state(ha, "a@weight", n)
    mg, vg, vmg, _ = adam.state("a@weight", n)
    assert np.array_equal(mg.view(np.uint32), mo.view(np.uint32))
    assert np.array_equal(vg.view(np.uint32), vo.view(np.uint32))
    if amsgrad:
        assert np.float32(vmg).view(np.uint32) == np.float32(vmo).view(np.uint32)
    oracle.adam_free(ha)


def test_error_feedback_residual(gpu, oracle):
    """compress.cpp:172-186: after compress, src[idx[i]] = 0 for every slot
    i < numel and the bucket is copied into the residual."""
    import torch
    from stellatrain_amd import CodecEngine
    n = 1 << 20
    eng = CodecEngine()
    eng.configure_compression("thresholdv16")
    eng.configure_compression_ratio(0.99)
    ho = oracle.tv16_new()
    k = oracle.merge_numel(n, 0.99)
    for it in range(3):
        src = synth(n, seed_for(12, it))
        co, io, vo = oracle.tv16_compress(ho, "ef@weight", src, k)
        expect = src.copy()
        expect[io[:k]] = 0.0
        g = torch.from_numpy(src.copy()).to(gpu)
        resid = torch.full((n,), 7.0, dtype=torch.float32, device=gpu)
        idx, val, cnt = eng.compress_bucket("ef@weight", g, world=1, residual=resid)
        torch.cuda.synchronize()
        assert int(cnt.item()) == co
        assert np.array_equal(resid.cpu().numpy().view(np.uint32), expect.view(np.uint32))
        assert np.array_equal(g.cpu().numpy().view(np.uint32), expect.view(np.uint32))
    oracle.tv16_free(ho)


@pytest.mark.parametrize("n,off,numel", [(1000003, 0, 10000), (4099, 1, 41), (64, 0, 0)])
def test_error_feedback_kernel(gpu, n, off, numel):
    """stg_error_feedback_device against a torch fp32 reference of
    compress.cpp:172-186: zero the bucket at every slot's index (unwritten
    slots hold index 0), copy it into the residual; ragged and unaligned
    buckets take the copy fallback."""
    import ctypes
    import torch
    from stellatrain_amd._capi import check, lib
    gen = torch.Generator().manual_seed(n + off)
    base = torch.randn(n + off, generator=gen).to(gpu)
    g = base[off:]
    idx = torch.zeros(numel, dtype=torch.int32)
    if numel:
        idx[: numel - numel // 4] = torch.randperm(n, generator=gen)[: numel - numel // 4].to(torch.int32)
    idx = idx.to(gpu)
    expect = g.clone()
    if numel:
        expect[idx.long()] = 0.0
    resid = torch.full((n,), 7.0, dtype=torch.float32, device=gpu)
    check(lib().stg_error_feedback_device(ctypes.c_void_p(g.data_ptr()), n, ctypes.c_void_p(idx.data_ptr()), numel,
                                          ctypes.c_void_p(resid.data_ptr()),
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    assert torch.equal(resid, expect)
    assert torch.equal(g, expect)


@pytest.mark.parametrize("method", ["thresholdv16", "thresholdv", "topk_exact"])
def test_merge_compress_batch_error_feedback(gpu, oracle, method):
    """stg_merge_compress_batch_device (compress.cpp:139-186) on a batch with
    ragged buckets, a repeated key and one 64 MiB bucket, against the ORACLE
    replaying the same calls in batch order: every (idx, val) stream and count
    is the oracle's, and every bucket and residual end as the bucket with the
    oracle's numel selected slots zeroed (unwritten slots hold index 0,
    compress.cpp:60-64,178-179).  thresholdv16 takes the fused residual copy."""
    import torch
    from stellatrain_amd import make_compressor
    sizes = [(1 << 20) + 5, 65536, 100013, 4099, 262144, 1 << 24]
    keys = ["a@w", "b@w", "c@w", "a@w", "d@w", "e@w"]  # a@w twice: the batch splits its launch
    comp = make_compressor(method)
    h = oracle.tv16_new() if method == "thresholdv16" else oracle.tv_new() if method == "thresholdv" else None
    keep = []  # threshold-v keys its state by src pointer: no pointer reuse across iterations
    for it in range(3):
        items, res, grads, srcs = [], [], [], []
        for j, (n, key) in enumerate(zip(sizes, keys)):
            src = synth(n, seed_for(60 + j, it), D2 if j % 2 else D1)
            k = oracle.merge_numel(n, 0.99)
            g = torch.from_numpy(src.copy()).to(gpu)
            items.append((key, g, k, torch.zeros(k, dtype=torch.int32, device=gpu),
                          torch.zeros(k, dtype=torch.float32, device=gpu)))
            res.append(torch.full((n,), 7.0, dtype=torch.float32, device=gpu))
            grads.append(g)
            srcs.append(src)
        keep.append((items, res))
        cnt = comp.compress_batch_async(items, residuals=res).cpu().numpy()
        for j, (key, _, k, di, dv) in enumerate(items):
            src = srcs[j]
            if method == "thresholdv16":
                co, io, vo = oracle.tv16_compress(h, key, src, k)
            elif method == "thresholdv":  # a fresh src pointer every call: a fresh key
                co, io, vo = oracle.tv_compress(h, 1000 * it + j, src, k)
            else:
                co, io, vo = oracle.topk_compress(src, k, bug_compat=False)
            assert int(cnt[j]) == co, (it, j)
            ig, vg = di.cpu().numpy().view(np.uint32), dv.cpu().numpy()
            assert_same_stream(ig, vg, io, vo, co)
            expect = src.copy()
            expect[io[:k]] = 0.0  # every one of the numel slots (compress.cpp:178-179)
            assert np.array_equal(res[j].cpu().numpy().view(np.uint32), expect.view(np.uint32)), (it, j)
            assert np.array_equal(grads[j].cpu().numpy().view(np.uint32), expect.view(np.uint32)), (it, j)
    comp.check_device()
    if h is not None:
        (oracle.tv16_free if method == "thresholdv16" else oracle.tv_free)(h)


def test_merge_path_python_api(gpu, oracle):
    """The whole node-side chain through the Python API, against the oracle
    chain: gather-add (cpu_gather.cpp) -> compress + error feedback
    (compress.cpp) -> wire encode/decode (comm_manager.cpp, u16 indices; a
    bucket below 32768 elements so the shipped saturation never triggers) ->
    MERGE decompress (cpu_optimize.cpp) -> sparse Adam (adam.cpp)."""
    import torch
    from stellatrain_amd import (CodecEngine, SparseAdam, gather_add, scatter_merge, wire_decode, wire_encode,
                                 wire_flag)
    n, g = 30000, 4
    eng = CodecEngine()
    eng.configure_compression("thresholdv16")
    eng.configure_compression_ratio(0.99)
    adam = SparseAdam(lr=1e-2)
    ht, ha = oracle.tv16_new(), oracle.adam_new(lr=1e-2)
    param = synth(n, seed_for(90, 9)) * np.float32(10)
    pg = torch.from_numpy(param.copy()).to(gpu)
    resid_o = np.zeros(n, np.float32)
    resid_g = torch.zeros(n, dtype=torch.float32, device=gpu)
    k = oracle.merge_numel(n, 0.99)
    flag = wire_flag(n)
    for it in range(3):
        grads = [synth(n, seed_for(91 + r, it), D1) for r in range(g)]
        dg = [torch.from_numpy(x.copy()).to(gpu) for x in grads]
        for r in range(g):
            oracle.gather_add(grads, resid_o, r)
            gather_add(dg, resid_g, r)
        co, io, vo = oracle.tv16_compress(ht, "p", grads[0], k)
        io_full = np.zeros(k, np.uint32)
        io_full[:co] = io[:co]
        grads[0][io_full] = 0.0
        resid_o = grads[0].copy()
        idx, val, cnt = eng.compress_bucket("p", dg[0], world=1, residual=resid_g)
        wi, wv = wire_encode(idx, val, flag)
        ri, rv = wire_decode(wi, wv, flag)
        oi, ov = oracle.wire_decode(*oracle.wire_encode(io_full, np.concatenate([vo[:co], np.zeros(k - co, np.float32)]),
                                                        flag), flag)
        mi, mv = oracle.merge_decompress(oi, ov, k, 1, n)
        oracle.adam_apply(ha, "p", param, mv, mi)
        gi, gv, gc = scatter_merge(ri, rv, k, 1, n)
        adam.optimize_raw(pg, "p", gv, gi, grad_len=k, d_grad_len=gc)
        assert np.array_equal(resid_g.cpu().numpy().view(np.uint32), resid_o.view(np.uint32))
        assert np.array_equal(pg.cpu().numpy().view(np.uint32), param.view(np.uint32)), it
    oracle.tv16_free(ht)
    oracle.adam_free(ha)


@pytest.mark.parametrize("world", [1, 2])
def test_saturated_wire_merge_adam(gpu, oracle, world):
    """a bucket with 32768 <= numel < 65536 travels with u16 indices
    whose 8-wide blocks saturate every index >= 32768 to 32767
    (comm_manager.cpp:509-529), so a decoded rank stream repeats 32767.  The
    MERGE decompress keeps the last occurrence per rank (index_put_ without
    accumulate) and one entry per index (unique1d), and the sparse Adam after
    it sees unique indices: parity with the oracle chain, bit-exact."""
    import torch
    from stellatrain_amd import SparseAdam, ThresholdvCompressor16, scatter_merge, wire_decode, wire_encode, wire_flag
    n = 50000
    k = oracle.merge_numel(n, 0.99, world)
    flag = wire_flag(n)
    comp = ThresholdvCompressor16()
    ht = oracle.tv16_new()
    ha = oracle.adam_new(lr=1e-2)
    adam = SparseAdam(lr=1e-2)
    param = synth(n, seed_for(70, 1)) * np.float32(10)
    pg = torch.from_numpy(param.copy()).to(gpu)
    for it in range(2):
        ri_all, rv_all, oi_all, ov_all = [], [], [], []
        for r in range(world):
            src = synth(n, seed_for(71 + r, it))
            co, io, vo = oracle.tv16_compress(ht, f"r{r}", src, k)
            idx = torch.zeros(k, dtype=torch.int32, device=gpu)
            val = torch.zeros(k, dtype=torch.float32, device=gpu)
            assert comp.compress(f"r{r}", torch.from_numpy(src).to(gpu), k, idx, val) == co
            wi, wv = wire_encode(idx, val, flag)
            ri, rv = wire_decode(wi, wv, flag)
            oi, ov = oracle.wire_decode(*oracle.wire_encode(io, vo, flag), flag)
            assert np.array_equal(ri.cpu().numpy().view(np.uint32), oi)
            ri_all.append(ri)
            rv_all.append(rv)
            oi_all.append(oi)
            ov_all.append(ov)
        ri, rv = torch.cat(ri_all), torch.cat(rv_all)
        oi, ov = np.concatenate(oi_all), np.concatenate(ov_all)
        assert np.count_nonzero(oi == 32767) > 1  # the saturation produced duplicates
        mi, mv = oracle.merge_decompress(oi, ov, k, world, n)
        dense = torch.zeros(n, dtype=torch.float32, device=gpu) if world > 1 else None
        mark = torch.zeros(n, dtype=torch.uint8, device=gpu) if world > 1 else None
        gi, gv, gc = scatter_merge(ri, rv, k, world, n, dense=dense, mark=mark)
        m = int(gc.item())
        assert m == mi.size
        a_i, a_v = _sorted_pairs(gi[:m].cpu().numpy(), gv[:m].cpu().numpy())
        assert np.array_equal(a_i, mi) and np.array_equal(a_v.view(np.uint32), mv.view(np.uint32))
        oracle.adam_apply(ha, "p", param, mv, mi)
        adam.optimize_raw(pg, "p", gv, gi, grad_len=k * world, d_grad_len=gc)
        assert np.array_equal(pg.cpu().numpy().view(np.uint32), param.view(np.uint32)), it
    adam.check_device()
    oracle.tv16_free(ht)
    oracle.adam_free(ha)
