#!/usr/bin/env python3
"""HBM traffic per tv16_batch launch from two rocprofv3 --pmc passes.

Reads the counter CSVs of the FETCH_SIZE and WRITE_SIZE passes (separate runs:
FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2) made by
tools/gpu_run.sh pmc_fetch / pmc_write, averages the counter over the
dispatches of the named kernel and applies the gfx950 corrections of
MI355X_MICROARCH.md section HBM: FETCH_SIZE (KiB) reports half the bytes of
a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Writes a JSON summary
(bench.py reads hbm_bytes_per_bucket from profiles/pmc_tv16_batch.json).

  python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
      --kernel tv16_batch --buckets 8 --alg-bytes-per-bucket 68451040 -o profiles/pmc_tv16_batch.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def counter_mean(d: str, kernel: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per_dispatch = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id"))
                per_dispatch[key] = per_dispatch.get(key, 0.0) + float(row["Counter_Value"])
    if not per_dispatch:
        raise SystemExit(f"no {counter} rows for {kernel} in {d}")
    vals = sorted(per_dispatch.values())
    return sum(vals) / len(vals), len(vals), vals[0], vals[-1]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--kernel", default="tv16_batch")
    p.add_argument("--buckets", type=int, default=8, help="buckets per launch")
    p.add_argument("--alg-bytes-per-bucket", type=float, default=4.0 * 16777216 + 8.0 * 167772)
    p.add_argument("-o", "--out", default="profiles/pmc_tv16_batch.json")
    a = p.parse_args()
    fm, fn, fmin, fmax = counter_mean(a.fetch_dir, a.kernel, "FETCH_SIZE")
    wm, wn, wmin, wmax = counter_mean(a.write_dir, a.kernel, "WRITE_SIZE")
    rd = 2.0 * fm * 1024.0
    wr = wm * 1024.0
    per_launch = rd + wr
    out = {
        "kernel": a.kernel,
        "buckets_per_launch": a.buckets,
        "dispatches": {"fetch": fn, "write": wn},
        "FETCH_SIZE_KiB_mean": fm, "FETCH_SIZE_KiB_range": [fmin, fmax],
        "WRITE_SIZE_KiB_mean": wm, "WRITE_SIZE_KiB_range": [wmin, wmax],
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": per_launch,
        "hbm_bytes_per_bucket": per_launch / a.buckets,
        "alg_bytes_per_bucket": a.alg_bytes_per_bucket,
        "traffic_over_alg": per_launch / a.buckets / a.alg_bytes_per_bucket,
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of wide streaming reads); write = WRITE_SIZE x 1024",
    }
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
