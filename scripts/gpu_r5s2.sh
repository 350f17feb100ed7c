#!/usr/bin/env bash
# Round 5, call s2: a rocprofv3 kernel trace (every dispatch) of a short default bench, for the
# single-workgroup scans' per-call durations and neighbours.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5s2}
mkdir -p $OUT
RAW=/tmp/mc_ktrace_$$
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$RAW" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
f=$(find "$RAW" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$OUT/scan_calls.txt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = collections.defaultdict(list)
for i, r in enumerate(rows):
    if "k_scan1" in r["Kernel_Name"]:
        # the previous dispatch on the same queue
        j = i - 1
        while j >= 0 and rows[j]["Queue_Id"] != r["Queue_Id"]:
            j -= 1
        pn = rows[j]["Kernel_Name"].split("(")[0][:40] if j >= 0 else "-"
        prev[pn].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(prev.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:42s} calls {len(v):5d} total_us {sum(v):10.1f} avg_us {sum(v)/len(v):8.1f} max_us {max(v):8.1f}")
PY
cat "$OUT/scan_calls.txt"
rm -rf "$RAW"
