"""Summarise one bench step from a rocprofv3 kernel trace: per-launch duration,
gap before it, grouped by kernel; finds step boundaries at k_s2_degree."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("mc::", "").replace("void ", "")
starts = [i for i, r in enumerate(rows) if "k_s2_degree" in r["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
a = starts[which]
b = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
tend = int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"step launches={len(step)} span={(tend - t0) / 1e3:.1f} us busy={busy / 1e3:.1f} us idle={(tend - t0 - busy) / 1e3:.1f} us")
agg = defaultdict(lambda: [0, 0.0, 0.0])
prev_end = t0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = short(r["Kernel_Name"]) + f" g{r['Grid_Size_X']}"
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e3
    agg[k][2] += max(0, s - prev_end) / 1e3
    prev_end = e
for k, (n, d, gap) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{d:9.1f} us  n={n:4d}  avg={d / n:7.2f}  gaps={gap:8.1f}  {k}")
if len(sys.argv) > 3:
    prev_end = t0
    for r in step[: int(sys.argv[3])]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} +{(e - s) / 1e3:7.2f} gap {(s - prev_end) / 1e3:6.2f}  {short(r['Kernel_Name'])} g{r['Grid_Size_X']}")
        prev_end = e
