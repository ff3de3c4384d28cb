#!/usr/bin/env python3
"""Print the tail of a rocprofv3 kernel trace as a per-queue timeline (us)."""
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
f = glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = []
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].split("::")[-1].split("<")[0] or name[:20]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r.get("Queue_Id", "")))
ev.sort()
t0 = ev[-n][0]
for s, e, nm, q in ev[-n:]:
    print(f"{nm:22s} q{q:>3s} start {(s - t0) / 1e3:9.1f} end {(e - t0) / 1e3:9.1f} dur {(e - s) / 1e3:7.1f}")
