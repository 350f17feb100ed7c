#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 bench.py --steps "${STEPS:-10}" --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "rocprof rc=$rc"
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
head -40 "$OUT/kernel_stats.csv" 2>/dev/null | cut -c1-200
exit $rc
