#!/usr/bin/env bash
# One rocprofv3 PMC pass (a single counter) over a python command; the per-dispatch CSV is kept
# OUTSIDE gpurun_out (it is large) as <dir>/pmc_<COUNTER>.csv for scripts/pmc_summary.py:
#   bash scripts/pmc_pass.sh <dir> <COUNTER> <python args...>
set -u
out=$1; ctr=$2; shift 2
mkdir -p "$out/raw_$ctr"
timeout -k 10 -s KILL 500 rocprofv3 --pmc "$ctr" -d "$out/raw_$ctr" -o "pmc_$ctr" --output-format csv -- python3 "$@"
rc=$?
f=$(find "$out/raw_$ctr" -name "pmc_${ctr}_counter_collection.csv" | head -n 1)
if [ -z "$f" ]; then echo "no counter CSV (rocprofv3 rc=$rc)" >&2; exit 1; fi
cp "$f" "$out/pmc_$ctr.csv"
echo "rocprofv3 rc=$rc, $(wc -l < "$out/pmc_$ctr.csv") rows" >&2
