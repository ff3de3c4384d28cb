#!/usr/bin/env python3
"""Diagnostic: a tiny thresholdv16 AIMD sequence (n = 33, k = 3) call by call
against the oracle, with the fill's path counters after each call."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from oracle.oracle import Oracle
    from stellatrain_amd import ThresholdvCompressor16
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for, synth
    n, k = int(sys.argv[1]) if len(sys.argv) > 1 else 33, int(sys.argv[2]) if len(sys.argv) > 2 else 3
    o = Oracle()
    ho = o.tv16_new()
    comp = ThresholdvCompressor16()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    prev = [0] * 64
    for it in range(10):
        src = synth(n, seed_for(7, it), 0, 0)
        co, io, vo = o.tv16_compress(ho, "3@weight", src, k)
        idx = torch.zeros(k, dtype=torch.int32, device=dev)
        val = torch.zeros(k, dtype=torch.float32, device=dev)
        cg = comp.compress("3@weight", torch.from_numpy(src).to(dev), k, idx, val)
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        w = list(w)
        d = {i: w[i] - prev[i] for i in range(48, 64) if w[i] != prev[i]}
        prev = w
        ig = idx.cpu().numpy().view(np.uint32)
        ok = cg == co and np.array_equal(ig[:co], io[:co])
        print(json.dumps({"it": it, "ok": bool(ok), "got": ig.tolist(), "want": io[:co].tolist(), "dbg": d}), flush=True)


if __name__ == "__main__":
    main()
