"""Timeline of the mc:: kernels of one call in a rocprofv3 kernel_trace.csv, relative to the
n-th-from-last launch of an anchor kernel.

    python scripts/ktrace.py <kernel_trace.csv> [anchor=k_bp_count] [which=-2] [count=40]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mc::" in r["Kernel_Name"]]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_bp_count"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
count = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = idx[which]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + count]:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{n:34s} {a / 1e3:9.1f} -> {b / 1e3:9.1f}  ({(b - a) / 1e3:8.1f} us)  queue {r['Queue_Id']}")
