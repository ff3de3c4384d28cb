#!/usr/bin/env python3
"""Readable per-kernel averages from a rocprofv3 --stats kernel_stats.csv."""
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
f = glob.glob(f"{path}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("void ", "").replace("stg::(anonymous namespace)::", "")
    short = n.split("(")[0]
    print(f"{short[:48]:48s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs']) / 1e3:9.2f} "
          f"total_ms {float(r['TotalDurationNs']) / 1e6:9.2f}")
