#!/usr/bin/env python3
"""Per-launch duration percentiles of the headline's kernels from a rocprofv3
kernel trace (``--kernel-trace --output-format csv``), written as
profiles/fill_profile.json for bench.py's ``fill_profile`` field.

    python tools/fill_profile.py gpurun_out/prof_fresh "bench.py defaults (8 fresh sets)" [out.json]
"""
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else d
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/fill_profile.json"
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    durs = {}
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for k in ("tv16_fill", "tv16_batch"):
            if k in name:
                durs.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {"source": label, "trace": f, "unit": "us"}
    for k, v in durs.items():
        v.sort()
        pick = lambda q: round(v[min(len(v) - 1, int(q * len(v)))], 2)  # noqa: E731
        res[k] = {"launches": len(v), "p50": pick(0.5), "p90": pick(0.9), "p99": pick(0.99), "max": round(v[-1], 2),
                  "mean": round(sum(v) / len(v), 2)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
