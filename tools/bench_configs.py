#!/usr/bin/env python3
"""Secondary measurements for BASELINE.json configs 2-5 (GPU box).

bench.py carries the headline line (thresholdv16, 64 MiB, k=1%).  This tool
times the other configs on one GPU and prints one JSON line per measurement:

  C2  top-k k=1% on 64 MiB buckets ("topk" bug-compatible and "topk_exact"),
      device resident;
  C3  threshold-v k=0.1% on 256 MiB buckets, device resident, and host
      inclusive: src in pinned host memory (the reference's cudaHostRegister'd
      shm, shm_manager.cpp:92), H2D + codec + D2H of the (idx, val) stream,
      serial (stg_codec_compress_host) and with the H2D of bucket i+1
      overlapped with the codec on bucket i (two streams);
  C4  the 1024-bucket stream (256 KiB..64 MiB, log-uniform, seeded) through
      thresholdv16 batches of 32, device resident;
  C5  compress -> MERGE decompress -> sparse SGD (momentum 0.9) on 64 MiB,
      and the same with sparse Adam (plain and amsgrad) as the apply;
  APPLY  the optimizer applies alone on a 64 MiB param (k = 167,772 pairs
      from the codec), and WIRE encode/decode of that stream (u16 idx, fp16 val);
  E2E thresholdv16 64 MiB host-inclusive (serial and overlapped).

Every device timing rotates over >= 512 MB of distinct buckets so the 256 MB
Infinity Cache cannot serve the reads.  GB/s = dense fp32 bytes in / time.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def emit(d):
    print(json.dumps(d), flush=True)


def fill(lib, t, seed, stream):
    from stellatrain_amd._capi import check
    check(lib.stg_synth_fill_device(C.c_void_p(t.data_ptr()), t.numel(), seed, 0, 0, C.c_void_p(stream)))


def bufs_for(torch, lib, dev, n, count, stream, base_seed=0):
    from stellatrain_amd.synth import seed_for
    out = []
    for i in range(count):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        fill(lib, t, seed_for(base_seed + i, 0), stream)
        out.append(t)
    return out


def time_device(torch, comp, method, mib, ratio, calls, warmup, keys):
    """One key per buffer; rotate over >= 512 MB."""
    from stellatrain_amd import merge_numel
    from stellatrain_amd._capi import lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = mib * (1 << 20) // 4
    k = merge_numel(n, ratio)
    nbuf = max(keys, math.ceil(512 / mib) + 1)
    bufs = bufs_for(torch, lib(), dev, n, nbuf, st.cuda_stream, 100)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    keyb = [f"{i % keys}@weight".encode() for i in range(nbuf)]
    # threshold-v keys by src pointer: every buffer is its own key there
    for i in range(nbuf):
        comp.compress_raw(keyb[i], bufs[i].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(), cnt.data_ptr(),
                          st.cuda_stream)
    for i in range(warmup):
        j = i % nbuf
        comp.compress_raw(keyb[j], bufs[j].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(), cnt.data_ptr(),
                          st.cuda_stream)
    torch.cuda.synchronize()
    # timed loop: no per-call events (each event record is a packet on the
    # stream and would lengthen every call)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    h0 = time.perf_counter()
    for i in range(calls):
        j = i % nbuf
        comp.compress_raw(keyb[j], bufs[j].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(), cnt.data_ptr(),
                          st.cuda_stream)
    host_us = (time.perf_counter() - h0) * 1e6 / calls  # enqueue only: the loop never waits for the GPU
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    # a second, instrumented pass for the per-launch breakdown
    comp.set_timing(True)
    for i in range(min(calls, 16)):
        j = i % nbuf
        comp.compress_raw(keyb[j], bufs[j].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(), cnt.data_ptr(),
                          st.cuda_stream)
    torch.cuda.synchronize()
    (k0, k1, kall), launches = comp.get_timing()
    comp.set_timing(False)
    comp.check_device()
    us = ms * 1e3 / calls
    # the bug-compatible "topk" reads only the first n/4 floats (memcpy of n
    # bytes, topk.cpp:31): its roofline is priced on the bytes it moves
    read = 4.0 * ((n + 3) // 4) if method == "topk" else 4.0 * n
    alg = read + 8.0 * k
    return {"config": f"{method} {mib} MiB k={k}", "n": n, "k": k, "us_per_call": round(us, 2),
            "alg_bytes": alg, "bytes_read_note": "4 ceil(n/4) + 8k (n/4 floats read)" if method == "topk" else "4n + 8k",
            "GBps_dense_in": round(4.0 * n / us / 1e3, 1),
            "alg_GBps": round(alg / us / 1e3, 1), "frac_hbm_peak": round(alg / us / 1e3 / PEAK, 4),
            "kernel_us": {"main": round(k0 * 1e3 / max(launches, 1), 2), "second": round(k1 * 1e3 / max(launches, 1), 2),
                          "call": round(kall * 1e3 / max(launches, 1), 2)},
            "count": int(cnt.item()), "rotating_buffers": nbuf, "host_enqueue_us_per_call": round(host_us, 2)}


def host_inclusive(torch, method, mib, ratio, calls):
    """Serial compress_host from pinned memory, then the overlapped pipeline."""
    from stellatrain_amd import make_compressor, merge_numel
    from stellatrain_amd.synth import seed_for, synth
    dev = torch.device("cuda", 0)
    n = mib * (1 << 20) // 4
    k = merge_numel(n, ratio)
    nb = 4
    host = [torch.from_numpy(synth(n, seed_for(200 + i, 0))).pin_memory() for i in range(nb)]
    oi = np.zeros(k, np.uint32)
    ov = np.zeros(k, np.float32)
    comp = make_compressor(method)
    for i in range(nb):
        comp.compress(f"{i}@w", host[i].numpy(), k, oi, ov)
    t0 = time.perf_counter()
    for c in range(calls):
        comp.compress(f"{c % nb}@w", host[c % nb].numpy(), k, oi, ov)
    serial = (time.perf_counter() - t0) / calls
    # overlapped: H2D of bucket c+1 on a copy stream while the codec runs on c
    comp2 = make_compressor(method)
    cs, ks = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    dbuf = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(2)]
    didx = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in range(2)]
    dval = [torch.zeros(k, dtype=torch.float32, device=dev) for _ in range(2)]
    hidx = [torch.zeros(k, dtype=torch.int32).pin_memory() for _ in range(2)]
    hval = [torch.zeros(k, dtype=torch.float32).pin_memory() for _ in range(2)]
    copied = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]

    def run(total):
        with torch.cuda.stream(cs):
            dbuf[0].copy_(host[0], non_blocking=True)
            copied[0].record(cs)
        for c in range(total):
            p = c % 2
            if c + 1 < total:
                q = (c + 1) % 2
                with torch.cuda.stream(cs):
                    cs.wait_event(done[q])
                    dbuf[q].copy_(host[(c + 1) % nb], non_blocking=True)
                    copied[q].record(cs)
            with torch.cuda.stream(ks):
                ks.wait_event(copied[p])
                comp2.compress_async(f"{c % nb}@w", dbuf[p], k, didx[p], dval[p])
                hidx[p].copy_(didx[p], non_blocking=True)
                hval[p].copy_(dval[p], non_blocking=True)
                done[p].record(ks)
        torch.cuda.synchronize()
    run(nb)
    t0 = time.perf_counter()
    run(calls)
    ovl = (time.perf_counter() - t0) / calls
    # H2D alone (pinned -> device), the PCIe ceiling of this path
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(calls):
        dbuf[0].copy_(host[c % nb], non_blocking=True)
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t0) / calls
    return {"config": f"{method} {mib} MiB k={k} host-inclusive", "n": n, "k": k,
            "serial_us_per_call": round(serial * 1e6, 1), "serial_GBps_dense_in": round(4.0 * n / serial / 1e9, 2),
            "overlapped_us_per_call": round(ovl * 1e6, 1), "overlapped_GBps_dense_in": round(4.0 * n / ovl / 1e9, 2),
            "h2d_only_GBps": round(4.0 * n / h2d / 1e9, 2)}


def c4_stream(torch, batches_timed, streams=1):
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import lib
    from stellatrain_amd.shard import ShardPlan, c4_sizes
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sizes = c4_sizes()
    plan = ShardPlan(sizes, 1)
    ids = plan.local(0)
    total = sum(sizes)
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    for i in ids:
        seg = flat[offs[i]:offs[i + 1]]
        fill(lib(), seg, seed_for(i, 0), st.cuda_stream)
    ks = [merge_numel(n, 0.99) for n in sizes]
    kt = sum(ks)
    oidx = torch.zeros(kt, dtype=torch.int32, device=dev)
    oval = torch.zeros(kt, dtype=torch.float32, device=dev)
    koffs = np.concatenate([[0], np.cumsum(ks)]).astype(np.int64)
    counts = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    comp = ThresholdvCompressor16()
    rows = [(plan.key(i).encode(), flat[offs[i]:].data_ptr(), sizes[i], ks[i], oidx[koffs[i]:].data_ptr(), ks[i],
             oval[koffs[i]:].data_ptr(), counts.data_ptr() + 4 * i) for i in ids]
    batches = [comp.bucket_array(rows[j:j + 32]) for j in range(0, len(rows), 32)]  # (MAX_BATCH)
    nrows = [len(rows[j:j + 32]) for j in range(0, len(rows), 32)]

    # batch j on stream j % S (keys are distinct within a sweep, so batches are
    # independent; a key's next batch is a sweep later, stream-ordered after
    # the join); STG_TV16_INFLIGHT = S splits the workgroup slots between them
    sts = [st] + [torch.cuda.Stream(dev) for _ in range(streams - 1)]

    def sweep():
        ev = torch.cuda.Event()
        ev.record(st)
        for x in sts[1:]:
            x.wait_event(ev)
        for j, (arr, nb) in enumerate(zip(batches, nrows)):
            comp.compress_batch_raw(arr, nb, sts[j % streams].cuda_stream)
        for x in sts[1:]:
            st.wait_stream(x)
    sweep()  # first calls
    sweep()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(batches_timed):
        sweep()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / batches_timed
    comp.check_device()
    assert bool((counts.cpu().numpy() == np.array(ks)).all())
    return {"config": "C4 thresholdv16 k=1% stream of 1024 buckets 256 KiB-64 MiB (1 GPU)", "buckets": len(ids),
            "streams": streams, "inflight": os.environ.get("STG_TV16_INFLIGHT", "unlimited"),
            "bytes": 4 * total, "ms_per_sweep": round(el * 1e3, 3), "GBps_dense_in": round(4.0 * total / el / 1e9, 1),
            "launches": len(batches)}


def make_opt(kind):
    from stellatrain_amd import SparseAdam, SparseSGD
    if kind == "sgd":
        return SparseSGD(lr=0.1, momentum=0.9), "SGD(m=0.9)"
    if kind == "adam":
        return SparseAdam(lr=1e-3), "Adam"
    return SparseAdam(lr=1e-3, amsgrad=True), "Adam(amsgrad)"


def c5_round_trip(torch, steps, kind="sgd"):
    from stellatrain_amd import ThresholdvCompressor16, merge_numel, scatter_merge
    from stellatrain_amd._capi import lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    nb = 9
    grads = bufs_for(torch, lib(), dev, n, nb, st.cuda_stream, 300)
    params = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nb)]
    for i, p in enumerate(params):
        fill(lib(), p, 777 + i, st.cuda_stream)
    comp = ThresholdvCompressor16()
    fused = kind.endswith("_fused")
    sgd, label = make_opt(kind[:-len("_fused")] if fused else kind)
    if fused:
        label += ", one merge_optimize call (step fused into the decompress)"
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    oi = torch.empty(k, dtype=torch.int32, device=dev)
    ov = torch.empty(k, dtype=torch.float32, device=dev)
    oc = torch.empty(1, dtype=torch.int32, device=dev)

    def step(s):
        j = s % nb
        comp.compress_async(f"{j}@w", grads[j], k, idx, val, count=cnt)
        if fused:  # ModuleCpuOptimize::run in one call (SparseSGD.merge_optimize)
            sgd.merge_optimize(params[j], f"{j}@w", idx, val, k, 1, out_idx=oi, out_val=ov, count=oc)
            return
        scatter_merge(idx, val, k, 1, n, out_idx=oi, out_val=ov, count=oc)
        sgd.optimize_raw(params[j], f"{j}@w", ov, oi, grad_len=k, d_grad_len=oc)
    for s in range(2 * nb):
        step(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    t0 = time.perf_counter()
    for s in range(steps):
        step(s)
    host_us = (time.perf_counter() - t0) * 1e6 / steps  # enqueue cost of the three Python calls
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    alg = 4.0 * n + 8.0 * k + (24.0 if kind.startswith("adam") else 16.0) * k
    return {"config": f"C5 thresholdv16 compress + decompress + {label} 64 MiB k={k}", "us_per_step": round(us, 2),
            "host_enqueue_us_per_step": round(host_us, 2),
            "GBps_dense_in": round(4.0 * n / us / 1e3, 1), "alg_GBps": round(alg / us / 1e3, 1)}


def merge_world(torch, calls, world=8):
    """MERGE decompress of `world` rank streams (cpu_optimize.cpp:40-72) into a
    64 MiB bucket: k = 167,772 pairs per rank, each rank's indices a distinct
    seeded sample of the bucket (overlapping across ranks)."""
    from stellatrain_amd import merge_numel, scatter_merge
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    g = torch.Generator(device="cpu").manual_seed(7)
    idx = torch.cat([torch.sort(torch.randperm(n, generator=g)[:k]).values for _ in range(world)]).to(torch.int32)
    idx, val = idx.to(dev), torch.randn(world * k, generator=g).to(dev)
    dense = torch.zeros(n, dtype=torch.float32, device=dev)
    mark = torch.zeros(n, dtype=torch.uint8, device=dev)
    oi = torch.empty(world * k, dtype=torch.int32, device=dev)
    ov = torch.empty(world * k, dtype=torch.float32, device=dev)
    oc = torch.empty(1, dtype=torch.int32, device=dev)
    us = _time_loop(torch, st, lambda s: scatter_merge(idx, val, k, world, n, dense, mark, oi, ov, oc), calls, 8)
    alg = world * 8.0 * k + 8.0 * int(oc.item()) + 5.0 * n  # pairs in, union out, dense + marks read once
    return {"config": f"MERGE decompress world={world}, 64 MiB bucket, k={k} per rank", "us_per_call": round(us, 2),
            "union": int(oc.item()), "alg_GBps": round(alg / us / 1e3, 1)}


def _time_loop(torch, st, fn, calls, warmup):
    for s in range(warmup):
        fn(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for s in range(calls):
        fn(s)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / calls


def apply_and_wire(torch, calls):
    """Optimizer applies and wire casts alone on one codec stream of a 64 MiB
    bucket (k = 167,772), rotating over 9 params (> 512 MB with the moments)."""
    from stellatrain_amd import ThresholdvCompressor16, merge_numel, wire_decode, wire_encode
    from stellatrain_amd._capi import lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    nb = 9
    g = bufs_for(torch, lib(), dev, n, 1, st.cuda_stream, 400)[0]
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    ThresholdvCompressor16().compress("a@w", g, k, idx, val)
    params = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nb)]
    for i, p in enumerate(params):
        fill(lib(), p, 900 + i, st.cuda_stream)
    out = []
    for kind in ("sgd", "adam", "adam_ams"):
        opt, label = make_opt(kind)
        us = _time_loop(torch, st, lambda s: opt.optimize_raw(params[s % nb], f"{s % nb}@w", val, idx), calls, 2 * nb)
        alg = 8.0 * k + (16.0 if kind == "sgd" else 24.0) * k  # (idx, g) in + RMW of param and moments
        out.append({"config": f"APPLY {label} alone, 64 MiB param, k={k}", "us_per_call": round(us, 2),
                    "alg_GBps": round(alg / us / 1e3, 1)})
    for flag in (1, 3):
        wi, wv = wire_encode(idx, val, flag)
        us_e = _time_loop(torch, st, lambda s: wire_encode(idx, val, flag, wi, wv), calls, 8)
        ri, rv = torch.empty_like(idx), torch.empty_like(val)
        us_d = _time_loop(torch, st, lambda s: wire_decode(wi, wv, flag, ri, rv), calls, 8)
        wb = k * (2 + (2 if flag & 2 else 4))
        out.append({"config": f"WIRE flag={flag} k={k}", "encode_us": round(us_e, 2), "decode_us": round(us_d, 2),
                    "encode_alg_GBps": round((8.0 * k + wb) / us_e / 1e3, 1),
                    "decode_alg_GBps": round((8.0 * k + wb) / us_d / 1e3, 1)})
    # the C4 stream's 1024 (idx, val) streams: one launch each vs batched
    from stellatrain_amd import wire_encode_batch
    from stellatrain_amd.shard import c4_sizes
    ks4 = [merge_numel(x, 0.99) for x in c4_sizes()]
    flat_i = torch.zeros(sum(ks4), dtype=torch.int32, device=dev)
    flat_v = torch.zeros(sum(ks4), dtype=torch.float32, device=dev)
    out_i = torch.empty(sum(ks4), dtype=torch.int16, device=dev)
    out_v = torch.empty(sum(ks4), dtype=torch.float32, device=dev)
    o4 = np.concatenate([[0], np.cumsum(ks4)]).astype(np.int64)
    items = [(flat_i[o4[j]:o4[j + 1]], flat_v[o4[j]:o4[j + 1]], 1, out_i[o4[j]:o4[j + 1]], out_v[o4[j]:o4[j + 1]])
             for j in range(len(ks4))]
    us_one = _time_loop(torch, st, lambda s: [wire_encode(a, b, f, c, d) for a, b, f, c, d in items], 4, 1)
    us_bat = _time_loop(torch, st, lambda s: wire_encode_batch(items), 4, 1)
    out.append({"config": f"WIRE encode of the C4 stream's {len(ks4)} streams (u16 idx)",
                "one_launch_per_stream_us": round(us_one, 1), "batched_us": round(us_bat, 1)})
    return out


def merge_ef(torch, calls):
    """MERGE compress + error feedback (compress.cpp:139-186) over 16 buckets of
    64 MiB per step (2 launches of 8): the fused thresholdv16 path
    (stg_merge_compress_batch_device) against compress + the separate
    stg_error_feedback_device pass.  Alg. bytes per bucket: 4n read + 4n
    residual write + 8k stream (+ the zeroing of k slots in both arrays).
    The error feedback zeroes the bucket in place, so every step regenerates
    the 16 buckets (a fresh gradient per iteration, as in training); the fill
    alone is timed too and subtracted."""
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    nb = 16
    grads = bufs_for(torch, lib(), dev, n, nb, st.cuda_stream, 500)
    res = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nb)]
    idx = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in range(nb)]
    val = [torch.zeros(k, dtype=torch.float32, device=dev) for _ in range(nb)]
    out = []
    for fused in (True, False):
        comp = ThresholdvCompressor16()
        counts = torch.zeros(nb, dtype=torch.int32, device=dev)

        def step(s, run=True):
            from stellatrain_amd.synth import seed_for
            for h in range(2):
                sl = range(8 * h, 8 * h + 8)
                for j in sl:
                    fill(lib(), grads[j], seed_for(500 + j, s), st.cuda_stream)
                if not run:
                    continue
                items = [(f"{j}@w", grads[j], k, idx[j], val[j]) for j in sl]
                if fused:
                    comp.compress_batch_async(items, counts=counts[8 * h:], residuals=[res[j] for j in sl])
                else:
                    comp.compress_batch_async(items, counts=counts[8 * h:])
                    for j in sl:
                        check(lib().stg_error_feedback_device(C.c_void_p(grads[j].data_ptr()), n,
                                                              C.c_void_p(idx[j].data_ptr()), k,
                                                              C.c_void_p(res[j].data_ptr()), C.c_void_p(st.cuda_stream)))
        us_all = _time_loop(torch, st, step, calls, 4) / nb
        us_fill = _time_loop(torch, st, lambda s: step(s, False), calls, 2) / nb
        us = us_all - us_fill
        alg = 8.0 * n + 8.0 * k
        out.append({"config": f"MERGE compress + error feedback, thresholdv16 64 MiB k={k}, "
                              f"{'fused residual copy' if fused else 'separate EF pass'}",
                    "us_per_bucket": round(us, 2), "fill_us_per_bucket": round(us_fill, 2), "GBps_dense_in": round(4.0 * n / us / 1e3, 1),
                    "alg_GBps": round(alg / us / 1e3, 1), "frac": round(alg / us / 1e3 / PEAK, 3)})
    return out


def gather(torch, calls):
    """Intra-node gather-add (cpu_gather.cpp:59-87) of a 64 MiB bucket from N
    device-local sources (all N ranks' slices in sequence = the whole bucket).
    Alg. bytes: 4n (dst) + 4n (residual) + 4n (N - 1) read + 4n written."""
    from stellatrain_amd import gather_add
    from stellatrain_amd._capi import lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    out = []
    for g in (2, 4, 8):
        srcs = bufs_for(torch, lib(), dev, n, g + 1, st.cuda_stream, 600)
        grads, resid = srcs[:g], srcs[g]

        def step(s):
            for r in range(g):
                gather_add(grads, resid, r)
        us = _time_loop(torch, st, step, calls, 2)
        alg = 4.0 * n * (g + 2)
        out.append({"config": f"GATHER-ADD 64 MiB bucket, N={g} sources + residual", "us_per_bucket": round(us, 2),
                    "alg_GBps": round(alg / us / 1e3, 1), "frac": round(alg / us / 1e3 / PEAK, 3)})
        del srcs, grads, resid
    return out


def gather_fused(torch, calls):
    """One MERGE task with the intra-node gather ahead of it on a 64 MiB
    bucket (cpu_gather.cpp:59-87 then compress.cpp:139-186):
    stg_merge_gather_compress_device (thresholdv16 sums the N - 1 sources and
    the residual inside its streaming pass) against the gather-add pass then
    the fused MERGE compress (stg_merge_compress_batch_device).  Every step
    regenerates grad[0] and the residual (two alternating inputs); the fill
    alone is timed and subtracted.  Alg. bytes (fused): 4n (N + 1)
    read + 8n written (grad[0], residual) + 8k."""
    from stellatrain_amd import ThresholdvCompressor16, gather_add, merge_numel
    from stellatrain_amd._capi import lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    out = []
    for g in (2, 4, 8):
        srcs = bufs_for(torch, lib(), dev, n, g + 1, st.cuda_stream, 700)
        grads, resid = srcs[:g], srcs[g]
        idx = torch.zeros(k, dtype=torch.int32, device=dev)
        val = torch.zeros(k, dtype=torch.float32, device=dev)
        counts = torch.zeros(1, dtype=torch.int32, device=dev)
        row = {"config": f"GATHER + MERGE compress (EF), thresholdv16 64 MiB k={k}, N={g} sources + residual"}
        for fused in (True, False):
            comp = ThresholdvCompressor16()

            def step(s, run=True):
                # two alternating inputs (as the headline's two buffer sets): the
                # key's threshold settles as it does in training
                fill(lib(), grads[0], seed_for(700, s % 2), st.cuda_stream)
                fill(lib(), resid, seed_for(760, s % 2), st.cuda_stream)  # (no collision with grad[1..])
                if not run:
                    return
                if fused:
                    comp.merge_gather_compress_async("gf@w", grads, k, idx, val, residual=resid, count=counts)
                else:
                    for r in range(g):  # every rank's slice of the bucket: the whole bucket
                        gather_add(grads, resid, r)
                    comp.compress_batch_async([("gf@w", grads[0], k, idx, val)], counts=counts, residuals=[resid])
            us = _time_loop(torch, st, step, calls, 4) - _time_loop(torch, st, lambda s: step(s, False), calls, 2)
            row["fused_us" if fused else "separate_us"] = round(us, 2)
            if fused:
                alg = 4.0 * n * (g + 1) + 8.0 * n + 8.0 * k
                row["fused_alg_GBps"] = round(alg / us / 1e3, 1)
                row["fused_frac"] = round(alg / us / 1e3 / PEAK, 3)
        out.append(row)
        del srcs, grads, resid
    return out


def wire_fused(torch, calls):
    """The compressed stream's wire form (comm_manager.cpp:486-590; SURVEY 8f
    row 3) written by the thresholdv16 emission
    (stg_codec_compress_wire_batch_device) against compress then
    stg_wire_encode_device: a 60,000-float bucket with u16 indices (queueTx's
    flag for numel < 65536) and a 64 MiB bucket with fp16 values
    (FP16_COMPRESSION).  Inputs rotate over >= 512 MB of device-resident
    buckets, one key."""
    from stellatrain_amd import ThresholdvCompressor16, merge_numel, wire_encode
    from stellatrain_amd._capi import lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    out = []
    for n, flag in ((60000, 1), (16 << 20, 2)):
        k = merge_numel(n, 0.99)
        nbuf = max(2, math.ceil(512 / (n * 4 / (1 << 20))) + 1) if n >= (1 << 20) else 16
        bufs = bufs_for(torch, lib(), dev, n, nbuf, st.cuda_stream, 820)
        idx = torch.zeros(k, dtype=torch.int32, device=dev)
        val = torch.zeros(k, dtype=torch.float32, device=dev)
        wi = torch.zeros(k, dtype=torch.int16 if flag & 1 else torch.int32, device=dev)
        wv = torch.zeros(k, dtype=torch.int16 if flag & 2 else torch.float32, device=dev)
        counts = torch.zeros(1, dtype=torch.int32, device=dev)
        row = {"config": f"thresholdv16 {n * 4 / (1 << 20):.2f} MiB k={k}, wire flag {flag}", "buffers": nbuf}
        for fused in (True, False):
            comp = ThresholdvCompressor16()

            def step(s):
                b = bufs[s % nbuf]
                if fused:
                    comp.compress_batch_async([("wf@w", b, k, wi, wv)], counts=counts, wire_flags=[flag])
                else:
                    comp.compress_batch_async([("wf@w", b, k, idx, val)], counts=counts)
                    wire_encode(idx, val, flag, wi, wv)
            row["fused_us" if fused else "separate_us"] = round(_time_loop(torch, st, step, calls, 8), 2)
        out.append(row)
        del bufs
    return out


def cpu_codec(method, mib, ratio, seconds):
    """The reference CPU path beside its GPU row, same run, this host's cores
    (north_star): oracle/_ref/libstg_ref.so (the reference's compress/*.cpp
    built in place, -O3 -march=broadwell) when it travelled, else the
    restatement.  1 thread, then T = min(CPU share, 32) threads, each a codec
    of its own (threshold-v: its own handle, the state keyed by the src
    pointer, thresholdv.cpp:44) over 2 shared alternating synthetic buckets
    (read-only for both codecs); steady-state calls (first calls excluded)."""
    import threading
    from oracle.oracle import REF_SO, Oracle, Reference
    sys.path.insert(0, ROOT)
    from bench import cpu_model, cpu_threads
    from stellatrain_amd import merge_numel
    o = Oracle()
    kind = "reference" if os.path.exists(REF_SO) else "port"
    impl = Reference() if kind == "reference" else o
    n = mib * (1 << 20) // 4
    k = merge_numel(n, ratio)
    bufs = [o.synth(n, 0x5EED0000 + 77 * 1000 + s) for s in range(2)]
    T = cpu_threads()

    def run(nthreads, secs):
        hs = [impl.tv_new() if method == "thresholdv" else None for _ in range(nthreads)]

        def one(t, c):
            if method == "thresholdv":
                impl.tv_compress(hs[t], 1, bufs[c % 2], k)
            elif kind == "reference":
                impl.topk_compress(bufs[c % 2], k)
            else:
                impl.topk_compress(bufs[c % 2], k, bug_compat=True)
        for t in range(nthreads):  # first call (threshold-v: nth_element over n) excluded
            one(t, 1)
        calls = [0] * nthreads
        stop = time.perf_counter() + secs
        barrier = threading.Barrier(nthreads + 1)

        def worker(t):
            barrier.wait()
            c = 0
            while time.perf_counter() < stop or c == 0:
                one(t, c)
                c += 1
            calls[t] = c
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for th in ths:
            th.start()
        t0 = time.perf_counter()
        barrier.wait()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        for h in hs:
            if h is not None:
                impl.tv_free(h)
        return 4.0 * n * sum(calls) / dt / 1e9, sum(calls), dt
    v1, c1, d1 = run(1, seconds / 2)
    vT, cT, dT = run(T, seconds / 2)
    return {"config": f"CPU {method} {mib} MiB k={k} ({'reference build' if kind == 'reference' else 'restatement'})",
            "kind": kind, "cpu": cpu_model(), "GBps_dense_in_1thread": round(v1, 3), "threads": T,
            "GBps_dense_in_T": round(vT, 3),
            "sample": f"{c1} calls in {d1:.1f} s on 1 thread, {cT} calls in {dT:.1f} s on {T} threads; 2 alternating "
                      "synthetic buckets, first call excluded"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--calls", type=int, default=48)
    p.add_argument("--c4-streams", type=int, default=4)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="per CPU baseline row (0: none)")
    p.add_argument("--only", default="c2,c3,c4,c5,single,e2e,apply,merge,ef,gather,gfused,wfused")
    a = p.parse_args()
    import torch
    from stellatrain_amd import make_compressor
    only = set(a.only.split(","))
    # C4 first: after the host-inclusive runs (pinned H2D traffic) the same
    # sweep measured 3.3 ms instead of 2.6 ms in one process
    if "c4" in only:
        emit(c4_stream(torch, 3, a.c4_streams))
    for m, tag in (("topk", "c2"), ("topk_exact", "c2")):
        if tag in only or m in only:  # "topk" / "topk_exact": one mode alone (PMC passes)
            emit(time_device(torch, make_compressor(m), m, 64, 0.99, a.calls, 8, 9))
    if "c2" in only and a.cpu_seconds > 0:  # the reference CPU path beside the GPU rows
        emit(cpu_codec("topk", 64, 0.99, a.cpu_seconds))
    if "c3" in only or "c3dev" in only:
        emit(time_device(torch, make_compressor("thresholdv"), "thresholdv", 256, 0.999, a.calls, 8, 3))
    if "c3" in only and a.cpu_seconds > 0:
        emit(cpu_codec("thresholdv", 256, 0.999, a.cpu_seconds))
    if "c3" in only:
        emit(host_inclusive(torch, "thresholdv", 256, 0.999, 12))
    if "e2e" in only:
        emit(host_inclusive(torch, "thresholdv16", 64, 0.99, 24))
    if "single" in only:  # one 64 MiB bucket per call, one stream: the latency of a lone call
        emit(time_device(torch, make_compressor("thresholdv16"), "thresholdv16 single-bucket", 64, 0.99, a.calls, 8, 16))
    if "c5" in only:
        for kind in ("sgd", "sgd_fused", "adam", "adam_fused", "adam_ams"):
            emit(c5_round_trip(torch, a.calls, kind))
    if "gfused" in only:
        for r in gather_fused(torch, a.calls):
            emit(r)
    if "wfused" in only:
        for r in wire_fused(torch, a.calls):
            emit(r)
    if "gather" in only:
        for d in gather(torch, a.calls):
            emit(d)
    if "ef" in only:
        for d in merge_ef(torch, max(8, a.calls // 4)):
            emit(d)
    if "merge" in only:
        for w in (2, 8):
            emit(merge_world(torch, a.calls, w))
    if "apply" in only:
        for d in apply_and_wire(torch, a.calls):
            emit(d)


if __name__ == "__main__":
    main()
