#!/usr/bin/env python3
"""Phase times of one threshold-v launch (tv_pass) on C3 (256 MiB, k = 0.1 %),
from s_memrealtime stamps (100 MHz).  Needs the stamp build:
make -C stellatrain_amd/csrc OUT=../../tools/variants/libstg_codec_tvst.so BUILD=build_tvst EXTRA=-DSTG_TV_STAMPS=1,
selected with STG_CODEC_LIB.  Times are microseconds after the start of the
workgroup that drew ticket 0: the last workgroup start, the last ticket in,
range 0's streaming end, the last streaming end, the last look-back end, the
last emission issued, range G-1's streaming and look-back ends, the fold."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from stellatrain_amd import make_compressor
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 64 << 20
    k = int(n * 0.001)
    comp = make_compressor("thresholdv")
    bufs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)]
    for i, b in enumerate(bufs):
        check(lib().stg_synth_fill_device(C.c_void_p(b.data_ptr()), n, seed_for(i, 0), 0, 0, C.c_void_p(st.cuda_stream)))
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    names = {41: "last_start", 42: "last_ticket", 43: "r0_stream_end", 44: "last_stream_end", 45: "last_lookback",
             49: "last_emit", 47: "rG1_stream_end", 48: "rG1_lookback", 46: "fold"}
    rows = []
    for it in range(16):
        comp.compress("x", bufs[it % 3], k, idx, val)
        v = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), v, 64))
        if it < 2:
            continue
        d = {nm: round(((v[w] - v[40]) & 0xffffffff) / 100.0, 2) for w, nm in names.items()}
        rows.append(d)
        print(json.dumps(d), flush=True)
    print(json.dumps({"median": {nm: sorted(r[nm] for r in rows)[len(rows) // 2] for nm in names.values()}}))
    # per range (last call): start, ticket, stream end relative to ticket 0's start; by XCD (block % 8) and ticket
    G = 256
    t = idx.cpu().numpy().view("uint32")[k - 4 * G:].reshape(G, 4).astype("int64")
    base = t[0, 1]
    rel = lambda x: ((x - base) & 0xffffffff) / 100.0
    import numpy as np
    start, tk, end = rel(t[:, 1]), rel(t[:, 2]), rel(t[:, 3])
    dur = end - tk
    xcd = t[:, 0] % 8
    print(json.dumps({"per_xcd_mean_stream_us": [round(float(dur[xcd == x].mean()), 2) for x in range(8)],
                      "per_xcd_mean_end_us": [round(float(end[xcd == x].mean()), 2) for x in range(8)],
                      "ticket_octile_mean_end_us": [round(float(end[i * 32:(i + 1) * 32].mean()), 2) for i in range(8)],
                      "ticket_octile_mean_tk_us": [round(float(tk[i * 32:(i + 1) * 32].mean()), 2) for i in range(8)],
                      "stream_us_min_med_max": [round(float(np.min(dur)), 2), round(float(np.median(dur)), 2), round(float(np.max(dur)), 2)],
                      "end_us_min_med_max": [round(float(np.min(end)), 2), round(float(np.median(end)), 2), round(float(np.max(end)), 2)]}))


if __name__ == "__main__":
    main()
