#!/usr/bin/env python3
"""In-scan finish diagnostics (GPU box): single-bucket thresholdv16 calls as
tools/lone_bench makes them (64 MiB, 16 keys over 16 distinct buckets), then
per call the finish's stamps from a STG_LF2_STAMPS build (debug words 0..15,
us after workgroup 0's start): last arrival, role 0 sees every shard, worker 0
decided / emitted, ranker 0 decided (5) / bins cut (2) / entries
decoded (10) / global facts (14) / ranked (15) / checked (6) / emitted (8), the last role's end,
and ranker 0's give-up site (7) with Wk / share size (12, 13); words 44/45 count
calls the scan launch ranked, 48..51 the fill launch's lfin paths."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = int(os.environ.get("LP_N", str(16 << 20)))
    k = merge_numel(n, 0.99)
    nk = 16
    comp = ThresholdvCompressor16()
    bufs = []
    for i in range(nk):
        b = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(b.data_ptr()), n, seed_for(100 + i, 0), 0, 0,
                                          C.c_void_p(st.cuda_stream)))
        bufs.append(b)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    w = (C.c_uint32 * 64)()
    for it in range(int(os.environ.get("LP_CALLS", "48"))):
        j = it % nk
        comp.compress_raw(f"{j}@weight".encode(), bufs[j].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(),
                          cnt.data_ptr(), st.cuda_stream)
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        if it < nk:
            continue
        v = list(w)
        t0 = v[0]
        rel = {i: (round(((v[i] - t0) & 0xffffffff) / 100.0, 2) if v[i] else None) for i in (1, 3, 20, 21, 4, 5, 2, 11, 10, 14, 15, 6, 8, 9)}
        print(json.dumps({"it": it, "us": rel, "giveup": v[7], "Wk_share": v[12:14], "ranked_scan": v[44:46],
                          "lfin_paths": v[48:52]}), flush=True)
    comp.check_device()


if __name__ == "__main__":
    main()
