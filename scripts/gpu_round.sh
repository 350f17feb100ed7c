#!/usr/bin/env bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats and two PMC
# passes (FETCH_SIZE, WRITE_SIZE: they cannot share a pass on gfx950).  Each GPU
# step has its own time limit; any failure ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
STEPS=${STEPS:-20}
BENCH_ARGS=${BENCH_ARGS:-}
run() { echo "== $*" >&2; "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
fi
run timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 3 $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
RAW=/tmp/mc_raw_$$   # raw profiler output stays on the box (per-dispatch CSVs are hundreds of MB)
mkdir -p "$RAW"
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary $BENCH_ARGS > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" \
    || { tail -20 "$OUT/prof_bench.err"; exit 1; }
find "$RAW/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 scripts/kstats.py "$OUT/kernel_stats.csv" | head -25
for C in FETCH_SIZE WRITE_SIZE; do
  run timeout -s KILL 180 rocprofv3 --pmc "$C" --output-format csv -d "$RAW/pmc_$C" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary $BENCH_ARGS > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" \
      || { tail -20 "$OUT/pmc_$C.err"; exit 1; }
  find "$RAW/pmc_$C" -name "*counter_collection.csv" -exec cp {} "$RAW/pmc_$C.csv" \;
done
python3 scripts/pmc_summary.py "$RAW" "$OUT/pmc_traffic.json" && rm -rf "$RAW"
ls -la "$OUT"
exit 0
