#!/usr/bin/env python3
"""Which way the headline's regime-B fills were ordered (diagnostic).

Runs bench.py's headline step (16 keys x 64 MiB, four batched calls of four
buckets on four streams, two buffer sets) for --steps steps and prints, per
stream workspace, the fill's path counters (debug words 56..59: no ties, ties
by start position, shadow heap, literal heap; 60..63: why the literal heap --
window miss, 2^20+ lines, > EMAX kept entries, window short of the output) and
the wide path's (40..47 when built, see tv16wide.hip)."""
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
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--keys", type=int, default=16)
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--streams", type=int, default=4)
    a = p.parse_args()
    import torch
    from stellatrain_amd import make_compressor
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.engine import merge_numel
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    comp = make_compressor("thresholdv16", device=0)
    s0 = torch.cuda.current_stream(dev)
    streams = [s0] + [torch.cuda.Stream(dev) for _ in range(a.streams - 1)]
    n = a.mib * (1 << 20) // 4
    k = merge_numel(n, 0.99, 1)
    nb = a.keys
    sets = [torch.empty(n * nb, dtype=torch.float32, device=dev) for _ in range(2)]
    for par in range(2):
        for j in range(nb):
            check(lib().stg_synth_fill_device(C.c_void_p(sets[par][j * n:].data_ptr()), n, seed_for(j, par), 0, 0,
                                              C.c_void_p(s0.cuda_stream)))
    oidx = torch.zeros(k * nb, dtype=torch.int32, device=dev)
    oval = torch.zeros(k * nb, dtype=torch.float32, device=dev)
    counts = torch.zeros(nb, dtype=torch.int32, device=dev)
    groups = [list(range(j, nb, a.streams)) for j in range(a.streams)]
    plans = []
    for par in range(2):
        calls = []
        for j, g in enumerate(groups):
            rows = [(f"{i}@weight".encode(), sets[par][i * n:].data_ptr(), n, k, oidx[i * k:].data_ptr(), k,
                     oval[i * k:].data_ptr(), counts.data_ptr() + 4 * i) for i in g]
            calls.append((comp.bucket_array(rows), len(rows), streams[j].cuda_stream))
        plans.append(calls)
    torch.cuda.synchronize()
    for s in range(a.steps):
        for arr, n_, sp in plans[s % 2]:
            comp.compress_batch_raw(arr, n_, sp)
    for st in streams[1:]:
        s0.wait_stream(st)
    torch.cuda.synchronize()
    comp.check_device()
    assert bool((counts.cpu().numpy() == k).all())
    out = []
    for st in streams:
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        w = list(w)
        out.append({"paths": w[56:60], "literal_why": w[60:64], "wide": w[32:40]})
    print(json.dumps({"steps": a.steps, "buckets": a.steps * nb, "per_stream": out}), flush=True)


if __name__ == "__main__":
    main()
