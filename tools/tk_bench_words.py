#!/usr/bin/env python3
"""bench_configs' C2 rows (time_device), then the compressor's debug words:
whether the hinted calls finished inside the stream launch (38 hits, 39
selects, 49 in-stream, 56 units done in the stream, 57 tk_one workgroups that
ran, 58 picker misses, 59 finisher poll timeouts)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from bench_configs import time_device
    from stellatrain_amd import make_compressor
    from stellatrain_amd._capi import check, lib
    st = torch.cuda.current_stream()
    for m in ("topk", "topk_exact"):
        comp = make_compressor(m)
        r = time_device(torch, comp, m, 64, 0.99, 48, 8, 9)
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        print(json.dumps({"mode": m, "us_per_call": r["us_per_call"], "kernel_us": r["kernel_us"],
                          "words": {i: w[i] for i in (38, 39, 49, 56, 57, 58, 59)},
                          "stamps_us_from_40": {i: round(((w[i] - w[40]) & 0xffffffff) / 100.0, 2) for i in range(41, 51)}}), flush=True)


if __name__ == "__main__":
    main()
