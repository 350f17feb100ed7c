#!/usr/bin/env bash
# Round 5, call v: rocprofv3 kernel trace + stats of the default bench (10 steps) on the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5v}
mkdir -p $OUT
RAW=/tmp/mc_raw_$$
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" \
    || { tail -20 "$OUT/prof_bench.err"; exit 1; }
find "$RAW/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$RAW/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
gzip -f "$OUT/kernel_trace.csv"
python3 scripts/kstats.py "$OUT/kernel_stats.csv" | sort -t' ' -k1 | head -60
rm -rf "$RAW"
