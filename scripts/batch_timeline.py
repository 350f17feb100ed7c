"""Per-batch S1 timeline from a rocprofv3 kernel_trace.csv: for each back-projection batch (one
k_bp_count launch), the span of each kernel group and the idle gaps between them.

    python scripts/batch_timeline.py <kernel_trace.csv> [last_n_batches]
"""
import csv
import sys

GROUPS = [("pixels", ("k_bp_count", "k_bp_frames", "k_bp_slots", "k_bp_compact")),
          ("voxel", ("k_bp_vox_order", "k_bp_voxel")),
          ("denoise", ("k_bp_classify", "k_bp_denoise")),
          ("query", ("k_bp_query", "k_bp_keepflags", "k_bp_emit"))]
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mc::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 8
starts = [i for i, r in enumerate(rows) if "k_bp_count" in r["Kernel_Name"]]
for bi, i0 in enumerate(starts[-last:]):
    i1 = starts[starts.index(i0) + 1] if starts.index(i0) + 1 < len(starts) else len(rows)
    seg = rows[i0:i1]
    t0 = int(seg[0]["Start_Timestamp"])
    out = []
    prev_end = t0
    for g, pref in GROUPS:
        ks = [r for r in seg if any(p in r["Kernel_Name"] for p in pref)]
        if not ks:
            continue
        a = min(int(r["Start_Timestamp"]) for r in ks)
        b = max(int(r["End_Timestamp"]) for r in ks)
        out.append(f"{g} {(b - a) / 1e3:7.1f}us (gap {(a - prev_end) / 1e3:6.1f})")
        prev_end = b
    nxt = int(rows[i1]["Start_Timestamp"]) if i1 < len(rows) else prev_end
    print(f"batch {bi}: " + " | ".join(out) + f" | tail gap {(nxt - prev_end) / 1e3:6.1f}us")
