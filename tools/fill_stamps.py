#!/usr/bin/env python3
"""Phase timing of tv16_fill (workgroup 0) from s_memrealtime stamps.

Needs the stamp build: make -C stellatrain_amd/csrc OUT=../../tools/variants/libstg_codec_stamps.so
BUILD=build_stamps EXTRA=-DSTG_FILL_STAMPS=1, selected with STG_CODEC_LIB.
Prints, per call, the phase durations in microseconds (100 MHz clock)."""
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
    n = 16 << 20
    k = merge_numel(n, 0.99)
    comp = ThresholdvCompressor16()
    nbk = int(os.environ.get("FS_BUCKETS", "8"))
    bufs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nbk)]
    outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev))
            for _ in range(nbk)]
    for it in range(10):
        for i, b in enumerate(bufs):
            check(lib().stg_synth_fill_device(C.c_void_p(b.data_ptr()), n, seed_for(i, it % 2 if os.environ.get("FS_PARITY") else it), 0, 0,
                                              C.c_void_p(st.cuda_stream)))
        comp.compress_batch_async([(f"{i}@w", bufs[i], k, outs[i][0], outs[i][1]) for i in range(nbk)])
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        v = list(w)
        print(json.dumps({"it": it, "raw": v[:14]}), flush=True)
        ts = [x for x in v[:16] if x > 1000]
        marks = [x for x in v[:16] if 0 < x <= 1000]
        print(json.dumps({"it": it, "W_Rn_nv_D1_P0_P_nU": v[40:47], "paths": v[56:60]}), flush=True)
        print(json.dumps({"it": it, "phase_us": [round((ts[j + 1] - ts[j]) / 100.0, 2) for j in range(len(ts) - 1)],
                          "marks": marks}), flush=True)
        for j in range(64):
            w[j] = 0
    comp.check_device()


if __name__ == "__main__":
    main()
