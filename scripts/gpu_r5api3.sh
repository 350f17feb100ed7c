#!/usr/bin/env bash
# Reference-API C2 with post_process, three repeats of 10 steps (box-to-box spread of the host part).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5api3
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --variant api --shape c2 --steps 10 --warmup 3 --with-pp > "$OUT/api_c2_pp_$i.json" 2> "$OUT/api_c2_pp_$i.err" || { echo "run $i failed"; tail -5 "$OUT/api_c2_pp_$i.err"; exit 1; }
  cat "$OUT/api_c2_pp_$i.json"
done
