#!/usr/bin/env python3
"""Print what tools/ab_lib.sh left under gpurun_out/."""
import csv
import json
import os

for f in ("new1", "alt1", "new2", "alt2"):
    p = f"gpurun_out/{f}.json"
    if os.path.exists(p) and os.path.getsize(p):
        d = json.load(open(p))
        print(f, d["value"], d["roofline"]["frac"])
for p in ("p_new", "p_alt"):
    q = f"gpurun_out/{p}/run_kernel_stats.csv"
    if os.path.exists(q):
        for r in csv.DictReader(open(q)):
            if "tv16" in r["Name"]:
                print(p, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
