#!/usr/bin/env python3
"""bench.py -- grad-codec GB/s (dense fp32 in) per GPU, thresholdv16 k=1% on 64 MiB buckets.

Workload (BASELINE.json metric): one *step* compresses the 16
gradient buckets of one iteration with thresholdv16: 16 keys ("<layer>@weight")
x 64 MiB fp32 (n = 16,777,216, dst_len = 167,772 = merge_numel(n, 0.99)),
device resident.  The engine issues its MERGE-compress tasks from several
pool workers at once (engine/modules/compress.cpp:141, config.h:7); here the
step is two batched C-ABI calls (stg_codec_compress_batch_device) of 8
buckets each on two streams = two concurrent persistent launches, so one
launch's exchange tail overlaps the other's streaming.  Each rank holds 2
buffer sets (the engine's iter%2 shm buffers, core.cpp:967) = 32 distinct
buckets (2 GiB >> the 256 MB Infinity Cache); step s compresses set s%2, so
every key sees fresh data each visit and its AIMD threshold runs its real
regime A/B sequence.  Keys are initialised (first-threshold call) before the
warmup.  value = 16 x 64 MiB x steps / time.

Multi-GPU: buckets are independent, so each rank compresses its
own buckets with no collective on the data path ("scaling": "weak");
value = bytes of all ranks / max-over-ranks time.

Extra fields: ``roofline`` for the dominant (only) kernel, tv16_batch, timed
live with HIP events (algorithmic bytes = 4n + 8k per bucket, over the
interval that brackets the profiled launches of all streams; the per-launch
average duration is reported beside it), ``cpu_baseline`` (the oracle port
of backend/src/compress timed on this host, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--ratio", type=float, default=0.99)
    p.add_argument("--keys", type=int, default=16)
    p.add_argument("--method", default="thresholdv16")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-steps", type=int, default=64)
    p.add_argument("--warmup-seconds", type=float, default=2.0)
    p.add_argument("--streams", type=int, default=2,
                   help="issue key i's calls on stream i %% S, like the engine's worker pool; with S > 1 each "
                        "persistent launch takes one workgroup per CU so two launches share the chip")
    return p.parse_args()


def cpu_baseline(n: int, k: int, seconds: float):
    """Oracle port of thresholdv16 (1 thread) on host copies of two buckets."""
    from oracle.oracle import Oracle
    from stellatrain_amd.synth import seed_for, synth
    o = Oracle()
    bufs = [synth(n, seed_for(0, i)) for i in range(2)]
    h = o.tv16_new()
    o.tv16_compress(h, "0@weight", bufs[0], k)  # first call (nth_element) excluded
    calls, t0 = 0, time.perf_counter()
    while True:
        o.tv16_compress(h, "0@weight", bufs[1 - calls % 2], k)
        calls += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or calls >= 2000:
            break
    o.tv16_free(h)
    return {"value": round(4.0 * n * calls / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"thresholdv16 {4 * n >> 20} MiB k={k}, {calls} steady-state calls on 2 alternating "
                      f"synthetic buckets (first call excluded), oracle/stg_oracle.cpp -O3 -march=broadwell, "
                      f"{dt:.1f} s"}


def load_traffic(buckets_per_launch: int):
    """HBM bytes per tv16_batch launch from the committed rocprofv3 PMC summary
    (profiles/pmc_tv16_batch.json, written by tools/pmc_summary.py), scaled to
    this run's buckets per launch."""
    path = os.path.join(ROOT, "profiles", "pmc_tv16_batch.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return int(d["hbm_bytes_per_bucket"] * buckets_per_launch)
    except Exception:
        return None


def main():
    args = parse()
    if args.streams > 1:
        # S concurrent persistent launches sharing the device's two workgroup
        # slots per CU: one launch's exchange tail overlaps the others' streaming
        os.environ.setdefault("STG_TV16_INFLIGHT", str(min(args.streams, 2)))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import ctypes as C

    from stellatrain_amd import make_compressor, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for

    n = args.mib * (1 << 20) // 4
    k = merge_numel(n, args.ratio, 1)
    nk = args.keys
    ns = max(1, min(args.streams, nk))
    comp = make_compressor(args.method, device=local)
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]

    bufs = []
    for b in range(2 * nk):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(rank * 64 + b % nk, b // nk), 0, 0,
                                          C.c_void_p(stream.cuda_stream)))
        bufs.append(t)
    outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev))
            for _ in range(nk)]
    counts = torch.zeros(nk, dtype=torch.int32, device=dev)
    keys = [f"{rank * 64 + i}@weight".encode() for i in range(nk)]

    # Per-step arguments resolved once: a step is one batched C-ABI call per
    # stream (keys split evenly over the streams), on buffer set s % 2.
    plans = []
    for par in range(2):
        calls = []
        for j in range(ns):
            ids = list(range(j, nk, ns))
            rows = [(keys[i], bufs[i + nk * par].data_ptr(), n, k, outs[i][0].data_ptr(), k, outs[i][1].data_ptr(),
                     counts.data_ptr() + 4 * i) for i in ids]
            calls.append((comp.bucket_array(rows), len(rows), streams[j].cuda_stream))
        plans.append(calls)

    def step(s):
        for arr, nb, sp in plans[s % 2]:
            comp.compress_batch_raw(arr, nb, sp)

    def sync_streams():
        for st in streams[1:]:
            stream.wait_stream(st)
        torch.cuda.synchronize()

    # first call per key: first threshold (reported, untimed for the metric)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step(0)
    sync_streams()
    first_ms = (time.perf_counter() - t0) * 1e3
    for s in range(args.warmup):
        step(s + 1)
    sync_streams()
    # the GPU holds low clocks for a while after going busy: keep stepping
    # until --warmup-seconds have passed before anything is timed
    t0 = time.perf_counter()
    s = args.warmup + 1
    while time.perf_counter() - t0 < args.warmup_seconds:
        for _ in range(16):
            step(s)
            s += 1
        sync_streams()

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(s)
    t_enq = time.perf_counter() - t0
    sync_streams()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    tt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el = float(tt.item())
    comp.check_device()
    if not os.environ.get("STG_DEBUG_TV16_STAGE"):
        assert int(counts.min().item()) == k

    # ---- live kernel timing (HIP events) ----
    # per launch: the events the codec records around every tv16_batch launch
    # on its stream (stg_codec_set_timing); chip level: events on stream 0
    # bracketing the profile steps of all streams (with S streams, S launches
    # overlap, so bytes / interval is the chip's rate, and S x interval /
    # launches is the per-launch duration rocprofv3 reports).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record(stream)
    for st in streams[1:]:
        st.wait_event(ev0)
    for s in range(args.profile_steps):
        step(s)
    for st in streams[1:]:
        stream.wait_stream(st)
    ev1.record(stream)
    torch.cuda.synchronize()
    chip_ms = ev0.elapsed_time(ev1)
    comp.set_timing(True)  # a second pass: per-launch events (they cost a little themselves)
    for s in range(args.profile_steps):
        step(s)
    (kern_ms, _fill_ms, call_ms), launches = comp.get_timing()
    comp.set_timing(False)
    launches = args.profile_steps * ns  # launches in the chip interval (one per stream and step)
    kern_us = kern_ms * 1e3 / max(launches, 1)
    per_launch = nk // ns

    bucket_bytes = 4.0 * n
    total_bytes = bucket_bytes * nk * args.steps * world
    value = total_bytes / el / 1e9
    if rank == 0:
        alg = per_launch * (4.0 * n + 8.0 * k)  # 4n + 8k per bucket
        # algorithmic bytes of every launch in the profiled interval / the
        # interval (= alg per launch / (avg launch duration / S) when the S
        # streams' launches overlap fully)
        achieved = alg * launches / (chip_ms * 1e-3) / 1e9
        out = {
            "metric": "grad-codec GB/s (dense fp32 in) per GPU; thresholdv16 k=1% on 64 MiB bucket",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (splitmix64 Irwin-Hall D1, 2 x {nk} distinct {args.mib} MiB buckets per GPU, "
                    "device resident)",
            "config": {"workload": f"{args.method} k={k} (1%) on {args.mib} MiB fp32 buckets; step = one batched "
                                   f"call over {nk} keys ({nk * args.mib} MiB)",
                       "streams": ns, "buckets_per_launch": per_launch,
                       "n": n, "dst_len": k, "parallelism": f"bucket-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(per_launch),
                         "kernel": "tv16_batch", "alg_bytes_per_launch": int(alg), "avg_us": round(kern_us, 2),
                         "concurrent_launches": ns, "launches_timed": int(launches),
                         "interval_us": round(chip_ms * 1e3, 1)},
            "per_bucket_us": round(el * 1e6 / (args.steps * nk), 3),
            "first_call_ms": round(first_ms, 3),
            "host_enqueue_us_per_step": round(t_enq * 1e6 / args.steps, 2),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n, k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
