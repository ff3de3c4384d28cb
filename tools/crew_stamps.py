#!/usr/bin/env python3
"""Phase times of the regime-B crew (tv16wide.h) from a stamp build
(-DSTG_CREW_STAMPS=1, STG_CODEC_LIB): a converged 64 MiB key, then calls at
1/100 scale; per dropped call, us after the first crew ticket at which phases
Z A C D E last completed a unit, the leader's steps (select, sort,
rank tiles, ties, pops) after its start, and the call's event time."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


WARM = int(os.environ.get("CREW_WARM", "0"))


def main():
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    comp = ThresholdvCompressor16()
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    bufs = []
    for i in range(8):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(600 + i, 0), 0, 0, C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    drops = [b * 0.01 for b in bufs[:4]]
    junk = torch.empty_like(bufs[0])
    for c in range(12):
        src = bufs[c % 8] if c < 6 else drops[c % 4]
        w0 = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w0, 64))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(WARM):  # keep the clocks up: busy work queued just before the call
            junk.copy_(bufs[1])
        e0.record(st)
        comp.compress_async("sd", src, k, idx, val)
        e1.record(st)
        torch.cuda.synchronize()
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        w = list(w)
        t0 = w[22]
        ph = {name: round(((w[16 + i] - t0) & 0xffffffff) / 100.0, 2) for i, name in enumerate("ZACDE")} \
            if w[53] != w0[53] else None
        lead = [round(((w[24 + i] - w[29]) & 0xffffffff) / 100.0, 2) for i in range(5)] if ph else None
        sub = [round(((w[8 + i] - w[29]) & 0xffffffff) / 100.0, 2) for i in range(8)] if ph else None
        print(json.dumps({"call": c, "dropped": c >= 6, "event_us": round(e0.elapsed_time(e1) * 1e3, 1),
                          "crew": w[53] - w0[53], "phases_us": ph, "leader_steps_us": lead,
                          "sub_us": sub, "last_start_us": round(((w[23] - t0) & 0xffffffff) / 100.0, 2), "m": w[6], "nr": w[7], "nroot": w[5]}), flush=True)


if __name__ == "__main__":
    main()
