#!/usr/bin/env python3
"""bench.py -- grad-codec GB/s (dense fp32 in) per GPU, thresholdv16 k=1% on 64 MiB buckets.

Workload (BASELINE.json metric): one *step* is one
thresholdv16 compress call on one 64 MiB fp32 bucket (n = 16,777,216,
dst_len = 167,772 = merge_numel(n, 0.99)), device resident, through the
C-ABI.  Each rank owns 8 keys ("<layer>@weight") x 2 alternating buffers
(the engine's iter%2 shm buffers, core.cpp:967) = 16 distinct buckets
(1 GiB > 2x the 256 MB Infinity Cache); step s compresses key s%8 from
buffer (s//8)%2, so every key sees fresh data each visit and the per-key
AIMD threshold runs its real regime A/B sequence.  Keys are initialised
(first-threshold call) before the warmup steps.

Multi-GPU: buckets are independent, so each rank compresses its
own buckets with no collective on the data path ("scaling": "weak");
value = bytes of all ranks / max-over-ranks time.

Extra fields: ``roofline`` for the dominant kernel (tv16_scan, timed live
with HIP events on the codec's stream), ``cpu_baseline`` (the oracle port of
backend/src/compress timed on this host, rank 0 at N=1 only).
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
    p.add_argument("--warmup", type=int, default=32)
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--ratio", type=float, default=0.99)
    p.add_argument("--keys", type=int, default=8)
    p.add_argument("--method", default="thresholdv16")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-steps", type=int, default=64)
    p.add_argument("--streams", type=int, default=1,
                   help="issue key i's calls on stream i %% S, like the engine's worker pool")
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


def load_traffic():
    """HBM bytes per tv16_scan launch from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_tv16_scan.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    args = parse()
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
    comp = make_compressor(args.method, device=local)
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(args.streams - 1)]

    bufs = []
    for b in range(2 * nk):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(rank * 64 + b % nk, b // nk), 0, 0,
                                          C.c_void_p(stream.cuda_stream)))
        bufs.append(t)
    outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev),
             torch.zeros(1, dtype=torch.int32, device=dev)) for _ in range(nk)]
    keys = [f"{rank * 64 + i}@weight" for i in range(nk)]

    # per-step arguments resolved once: the timed loop is one C-ABI call per step
    kb = [kk.encode() for kk in keys]
    sptr = [st.cuda_stream for st in streams]
    plan = []
    for s in range(2 * nk):
        i = s % nk
        src = bufs[i + nk * ((s // nk) % 2)]
        oi, ov, oc = outs[i]
        plan.append((kb[i], src.data_ptr(), n, k, oi.data_ptr(), k, ov.data_ptr(), oc.data_ptr(),
                     sptr[i % len(streams)]))

    def step(s):
        comp.compress_raw(*plan[s % (2 * nk)])

    # first call per key: first threshold (reported, untimed for the metric)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(nk):
        step(i)
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3 / nk
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(s)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    tt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el = float(tt.item())
    comp.check_device()

    # ---- live per-kernel timing (HIP events on the codec's stream) ----
    comp.set_timing(True)
    for s in range(args.profile_steps):
        step(s)
    (scan_ms, fill_ms, call_ms), calls = comp.get_timing()
    comp.set_timing(False)
    scan_us = scan_ms * 1e3 / max(calls, 1)
    fill_us = fill_ms * 1e3 / max(calls, 1)
    call_us = call_ms * 1e3 / max(calls, 1)

    total_bytes = 4.0 * n * args.steps * world
    value = total_bytes / el / 1e9
    if rank == 0:
        scan_bytes = 4.0 * n  # algorithmic bytes of the scan kernel: the dense bucket read
        achieved = scan_bytes / (scan_us * 1e-6) / 1e9
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
            "data": "synthetic (splitmix64 Irwin-Hall D1, 16 distinct 64 MiB buckets per GPU, device resident)",
            "config": {"workload": f"{args.method} k={k} (1%) on {args.mib} MiB fp32 buckets, {nk} keys x 2 buffers",
                       "streams": args.streams,
                       "n": n, "dst_len": k, "parallelism": f"bucket-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(),
                         "kernel": "tv16_scan", "bytes_per_launch": int(scan_bytes), "avg_us": round(scan_us, 2)},
            "kernels_us": {"scan": round(scan_us, 2), "fill": round(fill_us, 2), "call": round(call_us, 2),
                           "first_call_ms": round(first_ms, 3)},
            "call_gbs_alg": round((4.0 * n + 8.0 * k) / (call_us * 1e-6) / 1e9, 1),
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
