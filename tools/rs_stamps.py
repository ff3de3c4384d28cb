#!/usr/bin/env python3
"""Phase times of the radix select's first level (rs_hist<20,11>) inside a
top-k call, from s_memrealtime stamps (100 MHz).  Needs the stamp build:
make -C stellatrain_amd/csrc OUT=../../tools/variants/libstg_codec_rsst.so BUILD=build_rsst EXTRA=-DSTG_RS_STAMPS=1,
selected with STG_CODEC_LIB.  Prints, per call: the spread of workgroup starts,
first start -> last streaming end, -> last flush, -> pick start, pick length."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from stellatrain_amd import TopkCompressor
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, k = 16 << 20, 167772
    comp = TopkCompressor(exact=True)
    bufs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(4)]
    for i, b in enumerate(bufs):
        check(lib().stg_synth_fill_device(C.c_void_p(b.data_ptr()), n, seed_for(i, 0), 0, 0, C.c_void_p(st.cuda_stream)))
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    for it in range(12):
        comp.compress("x", bufs[it % 4], k, idx, val)
        v = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), v, 64))
        first, last = v[32], v[33]
        us = lambda a, b: round(((b - a) & 0xffffffff) / 100.0, 2)
        print(json.dumps({"it": it, "start_spread": us(first, last), "stream_end": us(first, v[34]),
                          "flush_end": us(first, v[35]), "pick_start": us(first, v[36]),
                          "pick": us(v[36], v[37])}), flush=True)


if __name__ == "__main__":
    main()
