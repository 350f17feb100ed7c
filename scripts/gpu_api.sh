#!/usr/bin/env bash
# The reference-API boundary (main.py:17-21 through the drop-in modules) on one box: C2 (with a cProfile
# of one extra step), C2 in replay mode, C3.  Each run has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/api}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }; cat "$OUT/$name.json"; }
run api_c2 300 python bench.py --variant api --shape c2 --steps 5 --warmup 2 --profile
run api_c2_replay 300 python bench.py --variant api --shape c2 --steps 5 --warmup 2 --replay
run api_c3 600 python bench.py --variant api --shape c3 --steps 3 --warmup 1
