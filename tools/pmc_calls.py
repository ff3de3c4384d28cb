#!/usr/bin/env python3
"""HBM traffic per codec call from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE runs of the same command), summed over the kernels of a call.

A call is counted once per dispatch of --call-kernel (the call's first launch);
every dispatch whose name contains one of --kernels adds its counters.  Reads
are reported raw and with the gfx950 correction of MI355X_MICROARCH.md
(section HBM: FETCH_SIZE counts half the bytes of wide coalesced streaming
reads), writes as WRITE_SIZE x 1024.

  python tools/pmc_calls.py gpurun_out/pmc_f gpurun_out/pmc_w --call-kernel 'rs_hist<20' \
      --kernels rs_hist,tk_ --alg-bytes 68451040 -o profiles/r02_pmc_topk_exact.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def per_kernel(d: str, counter: str, kernels):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != counter or not any(k in name for k in kernels):
                    continue
                key = (f, row.get("Dispatch_Id"))
                if key not in disp:
                    disp[key] = [name, 0.0]
                disp[key][1] += float(row["Counter_Value"])
    out = {}
    for name, v in disp.values():
        s = out.setdefault(name, [0, 0.0])
        s[0] += 1
        s[1] += v
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--call-kernel", required=True)
    p.add_argument("--kernels", required=True, help="comma-separated name substrings")
    p.add_argument("--alg-bytes", type=float, required=True, help="algorithmic bytes per call")
    p.add_argument("-o", "--out", required=True)
    a = p.parse_args()
    ks = a.kernels.split(",")
    f = per_kernel(a.fetch_dir, "FETCH_SIZE", ks)
    w = per_kernel(a.write_dir, "WRITE_SIZE", ks)
    calls_f = sum(c for n, (c, _) in f.items() if a.call_kernel in n)
    calls_w = sum(c for n, (c, _) in w.items() if a.call_kernel in n)
    if not calls_f or not calls_w:
        raise SystemExit("no dispatch of the call kernel")
    kern = {}
    for n in sorted(set(f) | set(w)):
        fc, fv = f.get(n, (0, 0.0))
        wc, wv = w.get(n, (0, 0.0))
        kern[n[:80]] = {"fetch_KiB_per_call": fv / calls_f, "write_KiB_per_call": wv / calls_w,
                        "dispatches": [fc, wc]}
    rd_raw = sum(v["fetch_KiB_per_call"] for v in kern.values()) * 1024.0
    wr = sum(v["write_KiB_per_call"] for v in kern.values()) * 1024.0
    out = {"calls": [calls_f, calls_w], "kernels": kern,
           "read_bytes_raw": rd_raw, "read_bytes_x2": 2 * rd_raw, "write_bytes": wr,
           "hbm_bytes_per_call_x2": 2 * rd_raw + wr, "alg_bytes_per_call": a.alg_bytes,
           "traffic_over_alg_x2": (2 * rd_raw + wr) / a.alg_bytes,
           "correction": "x2: read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of wide streaming reads); "
                         "raw FETCH kept for the non-streaming (superset, scattered) reads"}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
