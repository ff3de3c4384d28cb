#!/usr/bin/env python3
"""Per-call kernel breakdown of the thresholdv16 bench workload (GPU box).

Runs the bench.py workload one call at a time with HIP-event timing, reads
the per-key threshold after each call to classify the call's regime (A: the
ordered scan filled the stream, t grew; B: heap fill, t shrank), and prints a
JSON summary of scan / fill / call microseconds per regime.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--keys", type=int, default=8)
    p.add_argument("--calls", type=int, default=96)
    p.add_argument("--dist", type=int, default=0)
    p.add_argument("--param", type=int, default=0)
    a = p.parse_args()
    import torch

    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    n = a.mib * (1 << 20) // 4
    k = merge_numel(n, 0.99)
    comp = ThresholdvCompressor16()
    st = torch.cuda.current_stream(dev)
    bufs = []
    for b in range(2 * a.keys):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(b % a.keys, b // a.keys), a.dist,
                                          a.param, C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    for i in range(a.keys):
        comp.compress_async(f"{i}@w", bufs[i], k, idx, val, 0, count=cnt)
    comp.set_timing(True)
    comp.get_timing()
    rows = {"A": [], "B": []}
    for s in range(a.calls):
        i = s % a.keys
        before = comp.state(f"{i}@w", stream=st.cuda_stream)[0]
        comp.compress_async(f"{i}@w", bufs[i + a.keys * ((s // a.keys) % 2)], k, idx, val, 0, count=cnt)
        (sc, fi, ca), _ = comp.get_timing()
        after = comp.state(f"{i}@w", stream=st.cuda_stream)[0]
        rows["B" if after < before else "A"].append((sc * 1e3, fi * 1e3, ca * 1e3))
    comp.check_device()
    out = {"n": n, "k": k}
    for r, v in rows.items():
        if v:
            m = np.array(v)
            out[r] = {"calls": len(v), "scan_us": round(float(np.median(m[:, 0])), 2),
                      "fill_us": round(float(np.median(m[:, 1])), 2), "call_us": round(float(np.median(m[:, 2])), 2),
                      "fill_us_max": round(float(m[:, 1].max()), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
