"""Print one launch sequence from a rocprofv3 kernel trace: the launches from
the N-th occurrence of a kernel name (substring) on, with start/end relative
to it.  Usage: trace_seq.py TRACE.csv FIRST_NAME COUNT [OCCURRENCE]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
name, count = sys.argv[2], int(sys.argv[3])
occ = int(sys.argv[4]) if len(sys.argv) > 4 else -2
starts = [i for i, x in enumerate(rows) if name in x["Kernel_Name"]]
i0 = starts[occ]
t0 = int(rows[i0]["Start_Timestamp"])
for x in rows[i0:i0 + count]:
    s, e = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
    print(f"{x['Kernel_Name'][:60]:60s} {s / 1e3:8.2f} {e / 1e3:8.2f} {(e - s) / 1e3:7.2f}  "
          f"grid={x['Grid_Size_X']} wg={x['Workgroup_Size_X']} vgpr={x['VGPR_Count']} lds={x['LDS_Block_Size']}")
