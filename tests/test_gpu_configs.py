"""GPU parity at every BASELINE.json config's own size, against the REFERENCE.

tests/golden/golden_configs.npz + manifest_configs.json hold the outputs of
the reference's own codec / SGD build (oracle/_ref, compiled in place from
/root/reference; tests/golden/make_golden_configs.py) on inputs regenerated
here bit-exactly on the device (stg_synth_fill_device == the generator the
goldens were made from).  Each test runs the HIP path through the C-ABI at the
config's full size:

  C1  thresholdv16 4,194,304 floats, k = 41,943, 32 AIMD calls   thresholdv16.cpp:78-295
  C2  top-k 64 MiB, k = 167,772, shipped and exact modes          topk.cpp:28-46
  C3  threshold-v 256 MiB, k = 67,108, 10 calls incl. overflow,
      plus the host-inclusive entry point                         thresholdv.cpp:40-83
  C4  the 1,024-bucket stream in 16-bucket batches, 2 sweeps      core.cpp:1052-1087
  C5  64 MiB compress -> MERGE decompress -> momentum SGD, 3 steps
                                                                  cpu_optimize.cpp:40-72, sgd.cpp:221-260
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

from parity import assert_same_stream, bits, fbits
from stellatrain_amd.synth import D1, seed_for

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLD, "manifest_configs.json")))
ARR = np.load(os.path.join(GOLD, "golden_configs.npz"))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stream_sha(idx, val, cnt) -> str:
    return sha(np.asarray(idx[:cnt], np.uint32)) + ":" + sha(bits(val[:cnt]))


def set_sha(idx, val, cnt) -> str:
    i = np.asarray(idx[:cnt], np.uint32)
    o = np.argsort(i, kind="stable")
    return stream_sha(i[o], np.asarray(val[:cnt], np.float32)[o], cnt)


def fill(t, seed, scale=1.0):
    import torch
    from stellatrain_amd._capi import check, lib
    check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), t.numel(), seed, D1, 0,
                                      C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    if scale != 1.0:
        t.mul_(np.float32(scale).item())  # one fp32 multiply, as the generator's (synth * float32(scale))


def test_c1_thresholdv16_16mib_32_calls(gpu, oracle):
    import torch
    from stellatrain_amd import ThresholdvCompressor16
    c = MAN["c1"]
    n, k = c["n"], c["k"]
    comp = ThresholdvCompressor16()
    ho = oracle.tv16_new()
    src = torch.empty(n, dtype=torch.float32, device=gpu)
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    regimes = {"A": 0, "B": 0}
    t_prev = None
    for it, row in enumerate(c["rows"]):
        fill(src, seed_for(c["bucket"], it))
        cnt = comp.compress(c["key"], src, k, idx, val)
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        assert cnt == row["count"], it
        t, inc = comp.state(c["key"])
        assert (fbits(t), fbits(inc)) == (row["t_bits"], row["inc_bits"]), it
        assert set_sha(ig, vg, cnt) == row["set"], it  # the reference's exact pair set
        if t_prev is not None:
            regimes["A" if row["t_bits"] > t_prev else "B"] += 1
        assert stream_sha(ig, vg, cnt) == row["stream"], it  # the reference's stream, heap fill included
        if it < c["full_calls"]:
            np.testing.assert_array_equal(ig[:cnt], ARR[f"c1/it{it}/idx"])
        co, io, vo = oracle.tv16_compress(ho, c["key"], src.cpu().numpy(), k)  # and the live oracle
        assert co == cnt
        assert_same_stream(ig, vg, io, vo, cnt)
        t_prev = row["t_bits"]
    assert regimes["A"] and regimes["B"]
    comp.check_device()
    oracle.tv16_free(ho)


def test_c2_topk_64mib(gpu, oracle):
    import torch
    from stellatrain_amd import TopkCompressor
    c = MAN["c2"]
    n, k = c["n"], c["k"]
    src = torch.empty(n, dtype=torch.float32, device=gpu)
    fill(src, seed_for(c["bucket"], 0))
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    assert TopkCompressor().compress("x", src, k, idx, val) == c["count"]
    np.testing.assert_array_equal(idx.cpu().numpy(), np.arange(k))
    v = val.cpu().numpy()
    cut = np.abs(v).min()
    assert fbits(cut) == c["cut_bits"]
    assert sha(np.sort(bits(v[np.abs(v) > cut]))) == c["above_sorted_sha"]
    assert int((np.abs(v) == cut).sum()) == c["at_cut"]
    # the corrected mode over the whole bucket, against the oracle
    s_np = src.cpu().numpy()
    co, io, vo = oracle.topk_compress(s_np, k, idx_offset=0, bug_compat=False)
    assert TopkCompressor(exact=True).compress("x", src, k, idx, val) == co
    assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)


def test_c3_thresholdv_256mib_overflow_and_host_path(gpu, oracle):
    import torch
    from stellatrain_amd import ThresholdvCompressor
    c = MAN["c3"]
    n, k = c["n"], c["k"]
    comp = ThresholdvCompressor()
    src = torch.empty(n, dtype=torch.float32, device=gpu)  # one buffer: pointer-keyed state
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    for it, (row, sc) in enumerate(zip(c["rows"], c["scales"])):
        fill(src, seed_for(c["bucket"], it), sc)
        cnt = comp.compress("ignored", src, k, idx, val)
        ig, vg = idx.cpu().numpy().view(np.uint32), val.cpu().numpy()
        assert cnt == row["count"], it
        assert fbits(comp.state("", key_ptr=src.data_ptr())[0]) == row["t_bits"], it
        assert stream_sha(ig, vg, cnt) == row["stream"], it
        if it == 0:
            np.testing.assert_array_equal(ig[:cnt], ARR["c3/it0/idx"])
    counts = [r["count"] for r in c["rows"]]
    assert min(counts) < k and max(counts) == k  # both sides of the cap
    # host-inclusive entry point (stg_codec_compress_host): H2D + codec + D2H
    host = ThresholdvCompressor()
    buf = np.empty(n, np.float32)
    oi, ov = np.zeros(k, np.uint32), np.zeros(k, np.float32)
    for it in range(2):
        fill(src, seed_for(c["bucket"], it), c["scales"][it])
        buf[:] = src.cpu().numpy()
        cnt = host.compress("ignored", buf, k, oi, ov)
        assert cnt == c["rows"][it]["count"] and stream_sha(oi, ov, cnt) == c["rows"][it]["stream"]
    comp.check_device()


def test_c4_stream_1024_buckets(gpu):
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd.shard import ShardPlan, c4_sizes
    c = MAN["c4"]
    sizes = c4_sizes()
    assert sha(np.array(sizes, np.int64)) == c["sizes_sha"]
    plan = ShardPlan(sizes, 1)
    ks = [merge_numel(x, 0.99) for x in sizes]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    koffs = np.concatenate([[0], np.cumsum(ks)]).astype(np.int64)
    flat = torch.empty(int(offs[-1]), dtype=torch.float32, device=gpu)
    oidx = torch.zeros(int(koffs[-1]), dtype=torch.int32, device=gpu)
    oval = torch.zeros(int(koffs[-1]), dtype=torch.float32, device=gpu)
    comp = ThresholdvCompressor16()
    rows = {(r[0], r[1]): r for r in c["rows"]}
    bad = []
    for sw in range(c["sweeps"]):
        for b, n in enumerate(sizes):
            fill(flat[offs[b]:offs[b + 1]], seed_for(b, sw))
        counts = torch.zeros(len(sizes), dtype=torch.int32, device=gpu)
        for j in range(0, len(sizes), 32):  # batched launches of 32 distinct keys (MAX_BATCH)
            items = [(plan.key(b), flat[offs[b]:offs[b + 1]], ks[b], oidx[koffs[b]:koffs[b + 1]],
                      oval[koffs[b]:koffs[b + 1]]) for b in range(j, min(j + 32, len(sizes)))]
            comp.compress_batch_async(items, counts=counts[j:])
        torch.cuda.synchronize()
        cn, ih, vh = counts.cpu().numpy(), oidx.cpu().numpy().view(np.uint32), oval.cpu().numpy()
        for b in range(len(sizes)):
            _, _, cnt, tb, ss, st = rows[(sw, b)]
            t = comp.state(plan.key(b))[0]
            got = (int(cn[b]), fbits(t), set_sha(ih[koffs[b]:], vh[koffs[b]:], int(cn[b])),
                   stream_sha(ih[koffs[b]:], vh[koffs[b]:], int(cn[b])))
            if got != (cnt, tb, ss, st):  # the stream too: the heap fill's pop order (thresholdv16.cpp:261-293)
                bad.append((sw, b, got[:2], (cnt, tb), got[2] == ss, got[3] == st))
    comp.check_device()
    assert not bad, bad[:8]


def test_c5_round_trip_64mib(gpu):
    import torch
    from stellatrain_amd import SparseSGD, ThresholdvCompressor16, scatter_merge
    c = MAN["c5"]
    n, k = c["n"], c["k"]
    comp = ThresholdvCompressor16()
    sgd = SparseSGD(lr=c["lr"], momentum=c["momentum"])
    param = torch.empty(n, dtype=torch.float32, device=gpu)
    fill(param, seed_for(c["param_bucket"], 0))
    g = torch.empty(n, dtype=torch.float32, device=gpu)
    idx = torch.zeros(k, dtype=torch.int32, device=gpu)
    val = torch.zeros(k, dtype=torch.float32, device=gpu)
    for s, row in enumerate(c["rows"]):
        fill(g, seed_for(c["bucket"], s))
        cnt = comp.compress_async("c5@weight", g, k, idx, val)
        oi, ov, oc = scatter_merge(idx, val, k, 1, n)
        sgd.optimize_raw(param, "c5@weight", ov, oi, grad_len=k, d_grad_len=oc)
        assert int(cnt.item()) == row["count"] and int(oc.item()) == row["merged"]
        assert sha(bits(param.cpu().numpy())) == row["param"], s
        assert sha(bits(sgd.momentum_buffer("c5@weight", n))) == row["momentum"], s
    comp.check_device()
