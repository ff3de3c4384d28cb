#!/usr/bin/env python3
"""Phase timeline of the batched thresholdv16 kernel (diagnostic build).

Run with STG_DEBUG_TV16_STAGE=4: every workgroup records s_memrealtime
(100 MHz) into 128 words after the last bucket's count:
  [j*8 + 0]  finisher, slot j < 8: the streaming waves are done with the chunk
  [j*8 + 1]  finisher: look-back done (prefix known, inclusive published)
  [j*8 + 2]  finisher: chunk emitted, window list written, slot released
  [64 + 4b]      ranker, bucket b < 8 (regime B only): decision seen
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
    st = torch.cuda.current_stream(dev)
    bufs = []
    for b in range(2 * nb):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(b % nb, b // nb), 0, 0,
                                          C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev))
            for _ in range(nb)]
    cnt = torch.zeros(nb + 1024 * 128, dtype=torch.int32, device=dev)
    counts = cnt[:nb]

    def call(s):
        return comp.compress_batch_async([(f"{i}@w", bufs[i + nb * (s % 2)], k, outs[i][0], outs[i][1])
                                          for i in range(nb)], counts=counts)
    call(0)
    torch.cuda.synchronize()
    per_call = []
    for s in range(1, 21):
        cnt[nb:].zero_()
        call(s)
        torch.cuda.synchronize()
        a = cnt[nb:].cpu().numpy().view(np.uint32).astype(np.int64).reshape(1024, 128)
        used = (a != 0).any(axis=1)
        a = a[used]
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
    out["slot_ready_med"] = [med(j * 8) for j in range(8)]
    out["slot_ready_max"] = [mx(j * 8) for j in range(8)]
    out["slot_released_med"] = [med(j * 8 + 2) for j in range(8)]
    out["slot_released_max"] = [mx(j * 8 + 2) for j in range(8)]
    out["lookback_us_med"] = [dur(j * 8 + 1, j * 8) for j in range(8)]
    out["emit_us_med"] = [dur(j * 8 + 2, j * 8 + 1) for j in range(8)]
    out["rank_decision_med"] = [med(64 + 4 * b) for b in range(8)]
    out["rank_lists_in_med"] = [med(64 + 4 * b + 1) for b in range(8)]
    out["rank_done_med"] = [med(64 + 4 * b + 2) for b in range(8)]
    out["rank_done_max"] = [mx(64 + 4 * b + 2) for b in range(8)]
    out["rank_emit_us_med"] = [dur(64 + 4 * b + 2, 64 + 4 * b + 1) for b in range(8)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
