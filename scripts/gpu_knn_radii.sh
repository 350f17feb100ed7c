#!/usr/bin/env bash
# k-NN pre-selection radii sweep (MC_KNN_RADII) on one box: scripts/bp_profile.py per radii set,
# alternating REPS times over C3 frames 600-699 and the C2 scene.  Results only change speed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/radii}
mkdir -p "$OUT"
: > "$OUT/radii.jsonl"
SETS=${SETS:-"0.6,0.75,0.9 0.62,0.68,0.8 0.64,0.7,0.8 0.66,0.72,0.85 0.58,0.66,0.75"}
for r in 1 2; do
  for sh in c3:600:100 c2:0:250; do
    IFS=: read -r S F0 NF <<< "$sh"
    for set in $SETS; do
      MC_KNN_RADII=$set timeout -k 10 240 python scripts/bp_profile.py "$S" "$F0" "$NF" 3 > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/one.json')); print(json.dumps({'radii': '$set', 'window': '$sh', 'rep': $r, **d['group_ms']}))" >> "$OUT/radii.jsonl"
    done
  done
done
cat "$OUT/radii.jsonl"
