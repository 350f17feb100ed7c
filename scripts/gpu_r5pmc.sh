#!/usr/bin/env bash
# Round 5: the HBM traffic passes of the default bench (FETCH_SIZE / WRITE_SIZE, one per run), their
# per-group summary (scripts/pmc_summary.py) and the raw CSVs kept (gzipped) beside it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5pmc}
mkdir -p "$OUT"
RAW=/tmp/mc_raw_$$
mkdir -p "$RAW"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc "$C" --output-format csv -d "$RAW/pmc_$C" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" \
      || { tail -20 "$OUT/pmc_$C.err"; exit 1; }
  find "$RAW/pmc_$C" -name "*counter_collection.csv" -exec cp {} "$RAW/pmc_$C.csv" \;
  gzip -c "$RAW/pmc_$C.csv" > "$OUT/pmc_$C.csv.gz"
done
python3 scripts/pmc_summary.py "$RAW" "$OUT/pmc_traffic.json"
rm -rf "$RAW"
