#!/usr/bin/env bash
# One rocprofv3 kernel trace of the C3 E2E bench (1 warm-up + 2 timed steps); the mc:: rows of the
# per-dispatch trace are kept under $OUT (default gpurun_out/kt) with the per-batch overlap summary.
set -u
OUT=${OUT:-gpurun_out/kt}
SHAPE=${SHAPE:-c3}
mkdir -p "$OUT"
raw=/tmp/kt_raw_$$
mkdir -p "$raw"
timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace -d "$raw" -o kt --output-format csv -- \
    python3 bench.py --shape "$SHAPE" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
f=$(find "$raw" -name "kt_kernel_trace.csv" | head -n 1)
if [ -z "$f" ]; then echo "no kernel trace (rocprofv3 rc=$rc)" >&2; exit 1; fi
python3 - "$f" "$OUT/kernel_trace_mc.csv" <<'EOF'
import csv, sys
rd = csv.DictReader(open(sys.argv[1]))
w = csv.DictWriter(open(sys.argv[2], "w", newline=""), fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
w.writeheader()
for r in rd:
    if "mc::" in r["Kernel_Name"]:
        w.writerow({k: r[k] for k in ("Kernel_Name", "Start_Timestamp", "End_Timestamp")})
EOF
python3 scripts/denoise_overlap.py "$OUT/kernel_trace_mc.csv" 7 > "$OUT/denoise_overlap.txt"
exit $rc
