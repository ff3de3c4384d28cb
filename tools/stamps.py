#!/usr/bin/env python3
"""Phase timeline of the batched thresholdv16 kernel (diagnostic build).

Run with STG_DEBUG_TV16_STAGE=4: every workgroup records s_memrealtime
(100 MHz) into 128 words after the last bucket's count:
  [j*4 + 0]  finisher, slot j < 16: the streaming waves are done with the chunk
  [j*4 + 1]  finisher: prefix counts gathered
  [j*4 + 3]  finisher: qualifying lines emitted
  [j*4 + 2]  finisher: window list written, slot released
  [64 + 4b]      ranker, bucket b < 16 (regime B only): decision seen
  [64 + 4b + 1]  ranker: every chunk's window list in place
  [64 + 4b + 2]  ranker: heap fill share emitted
Prints medians / maxima over workgroups (microseconds from the earliest stamp
of the call), median over calls.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    assert os.environ.get("STG_DEBUG_TV16_STAGE") == "4"
    import torch

    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import seed_for
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("STAMPS_MIB", "64")) * (1 << 18)
    k = merge_numel(n, 0.99)
    nb = int(os.environ.get("STAMPS_BUCKETS", "8"))
    comp = ThresholdvCompressor16()
    ns = int(os.environ.get("STAMPS_STREAMS", "1"))  # concurrent launches (with STG_TV16_WGPERCU=1)
    st = torch.cuda.current_stream(dev)
    streams = [st] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
    bufs = []
    for b in range(2 * nb * ns):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(b % (nb * ns), b // (nb * ns)), 0, 0,
                                          C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev))
            for _ in range(nb * ns)]
    cnts = [torch.zeros(nb + 1024 * 128, dtype=torch.int32, device=dev) for _ in range(ns)]

    def call(s):
        for j in range(ns):
            items = [(f"{j * nb + i}@w", bufs[j * nb + i + nb * ns * (s % 2)], k, outs[j * nb + i][0],
                      outs[j * nb + i][1]) for i in range(nb)]
            comp.compress_batch_async(items, stream=streams[j].cuda_stream, counts=cnts[j][:nb])
    call(0)
    torch.cuda.synchronize()
    per_call, ctr = [], []
    for s in range(1, 21):
        for c_ in cnts:
            c_[nb:].zero_()
        torch.cuda.synchronize()
        call(s)
        torch.cuda.synchronize()
        for c_ in cnts[:1]:  # the first stream's launch
            a = c_[nb:].cpu().numpy().view(np.uint32).astype(np.int64).reshape(1024, 128)
            used = (a != 0).any(axis=1)
            a = a[used]
            ctr.append(a[:, 120:122].copy())
            a[:, 120:122] = 0
            t0 = np.where(a > 0, a, np.iinfo(np.int64).max).min()
            per_call.append(np.where(a > 0, (a - t0) / 100.0, np.nan))
    stack = np.stack(per_call)  # calls x wgs x 128

    def med(slot):
        x = stack[:, :, slot]
        return round(float(np.nanmedian(np.nanmedian(x, axis=1))), 2) if np.isfinite(x).any() else None

    def mx(slot):
        x = stack[:, :, slot]
        return round(float(np.nanmedian(np.nanmax(x, axis=1))), 2) if np.isfinite(x).any() else None

    def dur(s1, s0):
        x = stack[:, :, s1] - stack[:, :, s0]
        return round(float(np.nanmedian(x)), 2) if np.isfinite(x).any() else None

    out = {"buckets": nb, "wgs": int(stack.shape[1]), "calls": len(per_call)}
    NJ, NBK = 16, min(nb, 16)
    out["slot_ready_med"] = [med(j * 4) for j in range(NJ)]
    out["slot_ready_max"] = [mx(j * 4) for j in range(NJ)]
    out["slot_released_med"] = [med(j * 4 + 2) for j in range(NJ)]
    out["slot_released_max"] = [mx(j * 4 + 2) for j in range(NJ)]
    out["prefix_us_med"] = [dur(j * 4 + 1, j * 4) for j in range(NJ)]
    out["emit_us_med"] = [dur(j * 4 + 3, j * 4 + 1) for j in range(NJ)]
    out["list_release_us_med"] = [dur(j * 4 + 2, j * 4 + 3) for j in range(NJ)]
    out["rank_decision_med"] = [med(64 + 4 * b) for b in range(NBK)]
    out["rank_lists_in_med"] = [med(64 + 4 * b + 1) for b in range(NBK)]
    out["rank_done_med"] = [med(64 + 4 * b + 2) for b in range(NBK)]
    out["rank_done_max"] = [mx(64 + 4 * b + 2) for b in range(NBK)]
    out["rank_emit_us_med"] = [dur(64 + 4 * b + 2, 64 + 4 * b + 1) for b in range(NBK)]
    # streaming waves' wait spins per workgroup and call (s_sleep 2 / 1 each):
    # [120] buffer set not yet released by the finisher, [121] chunk id not yet known
    cc = np.stack(ctr)
    out["wait_spins_per_wg_med"] = {"fdone": float(np.median(cc[:, :, 0])), "cseq": float(np.median(cc[:, :, 1]))}
    out["wait_spins_per_wg_p90"] = {"fdone": float(np.percentile(cc[:, :, 0], 90)),
                                    "cseq": float(np.percentile(cc[:, :, 1], 90))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
