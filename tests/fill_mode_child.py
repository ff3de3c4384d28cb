"""Child process of tests/test_gpu_fill_modes.py (not a test module).

Runs thresholdv16 AIMD sequences whose regime-B calls tie inside the heap
fill -- one-bucket calls and a batched launch, each ending in a 100x drop of
the gradient scale (window misses) -- with STG_DEBUG_TV16_FILL set by the
parent (read once per process: 0 = production, 1 = always the shadow heap,
2 = always the literal heap, 3 = always the leader over the window, 4 = always
the crew), checks every call's whole stream against the oracle, and prints the
fill's path counters (debug words 56..59: the orderer's ways), the one-bucket
finish's (48..51: rankers without ties, rankers with ties, the orderer after
a violation, the orderer for a call the rankers could not take), the scan
finish's freshness check (31: workers that found a list entry without the
call's tag and left the call to the fill launch) and the wide
paths' (52..55: the orderer's leader, crew buckets, the orderer's leader
failing to the literal heap, the crew's leader failing to it) as one JSON
line.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    from oracle.oracle import Oracle
    from parity import assert_same_stream
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import D1, seed_for, synth
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    o = Oracle()
    ho = o.tv16_new()
    comp = ThresholdvCompressor16()
    literal = os.environ.get("STG_DEBUG_TV16_FILL") == "2"
    # (n, k, calls, calls at full scale): the rest are scaled by 1/100, a drop
    # of the gradient scale that leaves every line sum far below the window
    # under t (a window miss: the crew's calls, tv16wide.h)
    cases = [(1 << 20, 10485, 6, 6), (4 << 20, 41943, 5, 5), (16 << 20, 167772, 4, 4),
             ((2 << 20) + 13, 20971, 7, 3)]
    if literal:
        cases = cases[:2] + cases[3:]  # the literal heap takes milliseconds per call at 64 MiB
    calls = 0
    for ci, (n, k, iters, full) in enumerate(cases):
        key = f"fm{ci}"
        idx = torch.zeros(k, dtype=torch.int32, device=dev)
        val = torch.zeros(k, dtype=torch.float32, device=dev)
        for it in range(iters):
            x = synth(n, seed_for(700 + ci, it), D1)
            if it >= full:
                x = x * np.float32(0.01)
            cnt = comp.compress(key, torch.from_numpy(x).to(dev), k, idx, val)
            co, io, vo = o.tv16_compress(ho, key, x, k)
            assert cnt == co, (n, it)
            assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
            calls += 1
    # a batched launch of three buckets (the batched scan and its fill, with
    # the crew for the window misses after the drop)
    bsz = [(1 << 20) + 5, (3 << 20) + 9, 2 << 20]
    bks = [merge_numel(n, 0.99) for n in bsz]
    for it in range(7):
        items, ref = [], []
        for j, (n, k) in enumerate(zip(bsz, bks)):
            x = synth(n, seed_for(760 + j, it), D1)
            if it >= 4:
                x = x * np.float32(0.01)
            ref.append(o.tv16_compress(ho, f"fb{j}", x, k))
            items.append((f"fb{j}", torch.from_numpy(x).to(dev), k, torch.zeros(k, dtype=torch.int32, device=dev),
                          torch.zeros(k, dtype=torch.float32, device=dev)))
        counts = comp.compress_batch_async(items).cpu().numpy()
        torch.cuda.synchronize()
        for j, ((_, _, k, ig, vg), (co, io, vo)) in enumerate(zip(items, ref)):
            assert counts[j] == co, (it, j)
            assert_same_stream(ig.cpu().numpy().view(np.uint32), vg.cpu().numpy(), io, vo, co)
            calls += 1
    comp.check_device()
    w = (C.c_uint32 * 64)()
    check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
    print(json.dumps({"ok": True, "calls": calls, "paths": list(w)[56:60], "lfin": list(w)[48:52],
                      "scan_ranked": list(w)[44:46], "stale": w[31],
                      "wide": list(w)[52:56], "mode": os.environ.get("STG_DEBUG_TV16_FILL")}), flush=True)


if __name__ == "__main__":
    main()
