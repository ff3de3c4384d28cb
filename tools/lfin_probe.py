#!/usr/bin/env python3
"""One-bucket path diagnostics (GPU box): single-bucket thresholdv16 calls as
the bench's single row makes them (64 MiB, 16 keys over 16 distinct buckets),
then the lfin path counters (debug words 48..51: rankers without ties, with
ties, the orderer after a violation, the orderer for a call the rankers could
not take) and, with a stamps build (STG_CODEC_LIB=.../libstg_codec_stamps.so),
ranker 0's phase times of each call."""
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
        if it >= nk:  # steady state: one stamp line per call
            check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
            v = list(w)
            ts = v[32:42]
            # a phase a call did not reach keeps an earlier call's stamp: only increasing ones count
            ph = [round((ts[i + 1] - ts[i]) / 100.0, 2) if ts[i + 1] >= ts[i] > 0 else None for i in range(9)]
            ghz = None
            if ts[7] > ts[0] > 0 and v[43] > v[42]:
                ghz = round((v[43] - v[42]) / ((ts[7] - ts[0]) * 10.0), 2)  # cycles / ns
            w0 = v[16:22]
            wph = [round((w0[i + 1] - w0[i]) / 100.0, 2) if w0[i + 1] >= w0[i] > 0 else None for i in range(5)]
            t0 = min(x for x in (v[16], v[32]) if x) if (v[16] or v[32]) else 0
            arr = [round((x - t0) / 100.0, 2) if x and t0 else None for x in v[24:27]]
            ghz = round(((v[29] - v[28]) & 0xffffffff) / ((ts[9] - ts[0]) * 10.0), 2) if ts[9] > ts[0] > 0 else None
            print(json.dumps({"it": it, "paths": v[48:52], "ranker_phase_us": ph, "Wk_P_share_fl": v[44:48],
                              "worker0_phase_us": wph, "arrive_w0_r0_last_us": arr, "last_role": v[27],
                              "ranker_clock_GHz": ghz}), flush=True)
    comp.check_device()


if __name__ == "__main__":
    main()
