#!/usr/bin/env python3
"""Lone thresholdv16 calls on two alternating 64 MiB buckets, without and
with the MERGE error feedback (one bucket per stg_merge_compress_batch_device
call), for a kernel trace (diagnostics)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes as C
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    bufs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(2)]
    res = torch.empty(n, dtype=torch.float32, device=dev)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    for ef in (False, True):
        comp = ThresholdvCompressor16()
        for c in range(24):
            b = bufs[c % 2]
            check(lib().stg_synth_fill_device(C.c_void_p(b.data_ptr()), n, seed_for(900 + c % 2, 0), 0, 0,
                                              C.c_void_p(st.cuda_stream)))
            if ef:
                comp.compress_batch_async([("e@w", b, k, idx, val)], residuals=[res])
            else:
                comp.compress_async("e@w", b, k, idx, val)
        torch.cuda.synchronize()
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        print("ef", ef, "lfin paths", list(w)[48:52], "wide", list(w)[52:56], "fill paths", list(w)[56:60], flush=True)


if __name__ == "__main__":
    main()
