"""Diagnostic: the dispatch timeline of the last S1 call in a rocprofv3 kernel-trace CSV (from the
last k_grid_count on), one line per dispatch: start / end / duration in us from that call's start,
queue, kernel.

    python scripts/trace_timeline.py <kernel_trace.csv> [first-kernel substring]
"""
import csv
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_grid_count"
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        if "mc::" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if first in r[3]]
s = starts[-1]
t0 = rows[s][0]
for st, en, q, n in rows[s:]:
    print(f"{(st - t0) / 1e3:9.1f} {(en - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} q{q} {n[:70]}")
