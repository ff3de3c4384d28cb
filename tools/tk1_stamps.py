#!/usr/bin/env python3
"""Phase times of the emission launch of the hinted top-k (topk1.hip tk_one)
from a stamp build (-DSTG_TK1_STAMPS=1, STG_CODEC_LIB): us after workgroup 0
starts of its zeroing done, its pick done, every workgroup's pick done, the
last emission unit done, the last workgroup out; plus the two launches'
event times; 10 calls per mode on the C2 bucket (64 MiB, k = 1 %)."""
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
    bufs = []
    for i in range(4):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(500 + i, 0), 0, 0, C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    for exact in (True, False):
        comp = TopkCompressor(exact=exact)
        comp.set_timing(True)
        for c in range(10):
            comp.compress("c2", bufs[c % 4], k, idx, val)
            (k0, k1, kall), launches = comp.get_timing()
            w = (C.c_uint32 * 64)()
            check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
            w = list(w)
            t0 = w[40]
            rel = {name: round(((w[i] - t0) & 0xffffffff) / 100.0, 2) for name, i in
                   (("wg0_zeroed", 41), ("wg0_pick", 42), ("all_pick", 43), ("last_taken", 48), ("last_counted", 46),
                    ("last_lookback", 47), ("last_unit", 44), ("last_out", 45))}
            print(json.dumps({"exact": exact, "call": c, "hits": w[38], "selects": w[39], "us": rel,
                              "event_us": {"stream": round(k0 * 1e3, 2), "emit": round(k1 * 1e3, 2)}}), flush=True)


if __name__ == "__main__":
    main()
