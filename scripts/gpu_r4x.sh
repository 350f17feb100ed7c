#!/usr/bin/env bash
# Round 4, call x (extras at HEAD): the reference-API path on C3 (uint16 depth frames through the
# get_depth_raw hook, reference container orders, no post_process), the C5 312-scene sweep, C4 E2E.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4x}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -2 "$OUT/$name.out"; }
step sweep_c2 400 python -u bench.py --variant sweep --steps 1 --warmup 1 --no-cpu-baseline
step e2e_c4 300 python -u bench.py --shape c4 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
step api_c3 500 python -u bench.py --variant api --shape c3 --steps 2 --warmup 1
