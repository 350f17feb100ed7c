"""Print the mc:: kernels of a rocprofv3 kernel_stats.csv: calls, average and total time.

    python scripts/kstats.py <kernel_stats.csv> [filter]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else "mc::"
for r in rows:
    n = r["Name"]
    if flt in n:
        short = n.split("(")[0].replace("void ", "")
        print(f"{short:40s} calls {r['Calls']:>6} avg_us {float(r['AverageNs']) / 1e3:9.1f} "
              f"total_ms {float(r['TotalDurationNs']) / 1e6:8.2f}")
