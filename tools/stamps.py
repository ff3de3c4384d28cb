#!/usr/bin/env python3
"""Phase timeline of the fused thresholdv16 kernel (diagnostic build).

Run with STG_DEBUG_TV16_STAGE=4: each workgroup writes s_memrealtime (100 MHz)
at its phase boundaries into the count buffer.  Prints, per regime, the
critical-path time from the earliest kernel start to each phase boundary
(max over workgroups) in microseconds.
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
    comp = ThresholdvCompressor16()
    st = torch.cuda.current_stream(dev)
    bufs = []
    for b in range(4):
        t = torch.empty(n, dtype=torch.float32, device=dev)
        check(lib().stg_synth_fill_device(C.c_void_p(t.data_ptr()), n, seed_for(b % 2, b // 2), 0, 0,
                                          C.c_void_p(st.cuda_stream)))
        bufs.append(t)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1 + 1024 * 16, dtype=torch.int32, device=dev)
    for i in range(2):
        comp.compress_async(f"{i}@w", bufs[i], k, idx, val, 0, count=cnt)
    out = {"A": [], "B": []}
    for s in range(24):
        i = s % 2
        before = comp.state(f"{i}@w", stream=st.cuda_stream)[0]
        cnt.zero_()
        comp.compress_async(f"{i}@w", bufs[i + 2 * ((s // 2) % 2)], k, idx, val, 0, count=cnt)
        torch.cuda.synchronize()
        after = comp.state(f"{i}@w", stream=st.cuda_stream)[0]
        allst = cnt[1:].cpu().numpy().view(np.uint32).reshape(1024, 16).astype(np.int64)
        used = allst[:, 0] != 0
        xcc = allst[used, 8] & 0xF
        stamps = allst[used, :8]
        t0 = stamps[:, 0].min()
        rel = np.where(stamps > 0, stamps - t0, -1) / 100.0  # 10 ns ticks -> us
        crit = [float(rel[:, j][rel[:, j] >= 0].max()) if (rel[:, j] >= 0).any() else None for j in range(8)]
        med = [float(np.median(rel[:, j][rel[:, j] >= 0])) if (rel[:, j] >= 0).any() else None for j in range(8)]
        scan_end = rel[:, 1]
        per_xcc = [round(float(np.median(scan_end[xcc == x])), 2) if (xcc == x).any() else None for x in range(8)]
        worst = np.argsort(scan_end)[-8:].tolist()
        out["B" if after < before else "A"].append({"crit_us": crit, "median_us": med, "wgs": int(used.sum()),
                                                    "scan_end_by_xcc": per_xcc, "slowest_wgs": worst,
                                                    "start_of_slowest": rel[worst, 0].round(2).tolist()})
    summary = {}
    for r, v in out.items():
        if v:
            summary[r] = {"calls": len(v), "crit_us": np.round(np.median(np.array(
                [[x if x is not None else np.nan for x in e["crit_us"]] for e in v]), axis=0), 2).tolist(),
                "median_us": np.round(np.median(np.array(
                    [[x if x is not None else np.nan for x in e["median_us"]] for e in v]), axis=0), 2).tolist(),
                "wgs": v[0]["wgs"], "example": {kk: v[0][kk] for kk in ("scan_end_by_xcc", "slowest_wgs", "start_of_slowest")}}
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
