#!/usr/bin/env python3
"""Per-dispatch durations from a rocprofv3 --kernel-trace CSV: for each kernel
name, the count, min / median / p90 / max duration (us), and the gaps between
consecutive dispatches on the queue (end -> next start)."""
import csv
import glob
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_single"
f = glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("stg::(anonymous namespace)::", "").split("(")[0]
    by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, d in by.items():
    d.sort()
    print(f"{n[:44]:44s} n {len(d):5d} min {d[0]:8.2f} med {statistics.median(d):8.2f} "
          f"p90 {d[int(0.9 * (len(d) - 1))]:8.2f} max {d[-1]:8.2f}")
if len(sys.argv) > 2:  # the last N dispatches in order: name, duration, gap before
    last = rows[-int(sys.argv[2]):]
    prev = None
    for r in last:
        n = r["Kernel_Name"].replace("void ", "").replace("stg::(anonymous namespace)::", "").split("(")[0]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{n[:40]:40s} dur {(e - s) / 1e3:8.2f} gap {((s - prev) / 1e3) if prev else 0:8.2f}")
        prev = e
