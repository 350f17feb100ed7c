"""Per-batch view of the S1 groups from a rocprofv3 kernel_trace.csv (mc:: rows): for every batch
(one k_bp_count launch) the span of each group, and inside the denoise group each size class's
kernel start / end relative to the group start -- how long the chip runs only the last classes.

    python scripts/denoise_overlap.py <kernel_trace.csv> [last_n_batches]
"""
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mc::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 7
starts = [i for i, r in enumerate(rows) if "k_bp_count" in r["Kernel_Name"]]


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("mc::", "")
    return n


for i0 in starts[-last:]:
    k = starts.index(i0)
    i1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
    seg = rows[i0:i1]
    t0 = int(seg[0]["Start_Timestamp"])
    grp = {"pixels": [], "voxel": [], "denoise": [], "query": []}
    for r in seg:
        n = r["Kernel_Name"]
        g = ("pixels" if any(p in n for p in ("k_bp_count", "k_bp_frames", "k_bp_slots", "k_bp_compact")) else
             "voxel" if ("k_bp_voxel" in n or ("k_bp_vox_order" in n and not grp["voxel"])) else
             "denoise" if ("k_bp_denoise" in n or "k_bp_classify" in n or
                           ("k_bp_vox_order" in n and grp["voxel"])) else
             "query" if any(p in n for p in ("k_bp_query", "k_bp_keepflags", "k_bp_emit")) else None)
        if g:
            grp[g].append(r)
    line = []
    for g, rs in grp.items():
        if rs:
            a = min(int(r["Start_Timestamp"]) for r in rs)
            b = max(int(r["End_Timestamp"]) for r in rs)
            line.append(f"{g} {(a - t0) / 1e3:8.1f}..{(b - t0) / 1e3:8.1f} us")
    print(" | ".join(line))
    if grp["denoise"]:
        d0 = min(int(r["Start_Timestamp"]) for r in grp["denoise"])
        for r in grp["denoise"]:
            if "denoise" in r["Kernel_Name"]:
                a, b = int(r["Start_Timestamp"]) - d0, int(r["End_Timestamp"]) - d0
                print(f"    {short(r['Kernel_Name']):32s} {a / 1e3:8.1f} .. {b / 1e3:8.1f} us  ({(b - a) / 1e3:8.1f})")
