#!/usr/bin/env bash
# Final-state measurements of the other configs: the 312-scene C2 sweep (BASELINE configs[4]) and the
# post-processing row.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3i}
mkdir -p "$OUT"
echo "== sweep $(date +%T)"
timeout -k 10 480 python bench.py --variant sweep > "$OUT/sweep_c2.json" 2> "$OUT/sweep_c2.err" || { tail -5 "$OUT/sweep_c2.err"; exit 1; }
cat "$OUT/sweep_c2.json"
echo "== pp $(date +%T)"
timeout -k 10 300 python bench.py --variant pp > "$OUT/pp_c2.json" 2> "$OUT/pp_c2.err" || { tail -5 "$OUT/pp_c2.err"; exit 1; }
cat "$OUT/pp_c2.json"
