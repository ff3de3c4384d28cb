#!/usr/bin/env python3
"""Phase timeline of the batched thresholdv16 kernel (diagnostic build).

Run with STG_DEBUG_TV16_STAGE=4: every workgroup writes s_memrealtime
(100 MHz) at its start (slot 15), after scan(b) (slot 2b) and after finish(b)
(slot 2b+1), b < 7, into the words after the last bucket's count.  Prints,
per bucket, the critical-path time (max over workgroups, relative to the
earliest start) of each boundary, and the median, in microseconds.
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
    n = 16 << 20
    k = merge_numel(n, 0.99)
    nb = int(os.environ.get("STAMPS_BUCKETS", "7"))
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
    cnt = torch.zeros(nb + 2 * 1024 * 16, dtype=torch.int32, device=dev)
    counts = cnt[:nb]

    def call(s):
        return comp.compress_batch_async([(f"{i}@w", bufs[i + nb * (s % 2)], k, outs[i][0], outs[i][1])
                                          for i in range(nb)], counts=counts)
    call(0)
    torch.cuda.synchronize()
    rows = []
    for s in range(1, 25):
        cnt[nb:].zero_()
        call(s)
        torch.cuda.synchronize()
        all_ = cnt[nb:].cpu().numpy().view(np.uint32).astype(np.int64)
        a = all_[:16 * 1024].reshape(1024, 16)
        p = all_[16 * 1024:].reshape(1024, 16)
        used = a[:, 15] != 0
        a, p = a[used], p[used]
        t0 = a[:, 15].min()
        rel = (a[:, :14] - t0) / 100.0
        # probe: finish(2) after scan(3): 1 start, 2 gathered, 3 emitted, 4 AIMD
        # written, 5 regime-B collected, 6 finish end, 7 rank_deferred(1) end
        base = p[:, 1]
        sub = np.where(p[:, 1:8] > 0, (p[:, 1:8] - base[:, None]) / 100.0, np.nan)
        regime_b = bool((p[:, 5] > 0).any())
        stale = p[:, 8]  # probe: lanes stale at the first gather check, max poll rounds
        polls = p[:, 9]
        xcc = a[:, 14] & 0xF
        scan0 = rel[:, 0]
        per_xcc = [float(np.median(scan0[xcc == x])) if (xcc == x).any() else np.nan for x in range(8)]
        wg_ids = np.nonzero(used)[0]
        slow = wg_ids[np.argsort(scan0)[-16:]]
        rows.append({"xcc_scan0": per_xcc, "slow_wgs": slow.tolist(), "slow_xcc": xcc[np.argsort(scan0)[-16:]].tolist(),
                     "crit": rel.max(axis=0), "med": np.median(rel, axis=0),
                     "start_spread": float((a[:, 15].max() - t0) / 100.0), "wgs": int(used.sum()),
                     "sub_med": np.nanmedian(sub, axis=0), "stale_wgs": int((stale > 0).sum()),
                     "stale_lanes_max": int(stale.max()), "polls_max": int(polls.max()), "sub_max": np.nanmax(sub, axis=0), "B": regime_b})
    crit = np.median(np.stack([r["crit"] for r in rows]), axis=0)
    med = np.median(np.stack([r["med"] for r in rows]), axis=0)
    out = {"buckets": nb, "wgs": rows[0]["wgs"],
           "start_spread_us": round(float(np.median([r["start_spread"] for r in rows])), 2),
           "scan_end_crit_us": [round(float(crit[2 * b]), 2) for b in range(min(nb, 7))],
           "finish_end_crit_us": [round(float(crit[2 * b + 1]), 2) for b in range(min(nb, 7))],
           "scan_end_median_us": [round(float(med[2 * b]), 2) for b in range(min(nb, 7))],
           "finish_end_median_us": [round(float(med[2 * b + 1]), 2) for b in range(min(nb, 7))]}
    out["scan0_median_by_xcc_us"] = [round(float(x), 2) for x in np.nanmedian(np.stack([r["xcc_scan0"] for r in rows]), 0)]
    out["slowest16_wgs_call1"] = rows[0]["slow_wgs"]
    out["slowest16_xcc_call1"] = rows[0]["slow_xcc"]
    out["slowest16_wgs_call2"] = rows[1]["slow_wgs"]
    for tag in (False, True):
        rr = [r for r in rows if r["B"] == tag]
        if rr:
            out["probe_" + ("B" if tag else "A")] = {
                "calls": len(rr), "stale_wgs": [r["stale_wgs"] for r in rr][:6],
                "stale_lanes_max": [r["stale_lanes_max"] for r in rr][:6], "polls_max": [r["polls_max"] for r in rr][:6],
                "sub_median_us": [round(float(x), 2) for x in np.nanmedian(np.stack([r["sub_med"] for r in rr]), 0)],
                "sub_max_us": [round(float(x), 2) for x in np.nanmedian(np.stack([r["sub_max"] for r in rr]), 0)]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
