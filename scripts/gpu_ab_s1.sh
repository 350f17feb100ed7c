#!/usr/bin/env bash
# S1 A/B on one box: scripts/bp_profile.py per library build (LIBS, space-separated paths relative to
# the repo; MCGRAPH_LIB selects one per process), alternating REPS times over the SHAPES windows
# ("shape:first:count").  Each run has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
LIBS=${LIBS:-maskclustering_amd/libmcgraph_base.so maskclustering_amd/libmcgraph.so}
SHAPES=${SHAPES:-c3:600:100 c2:0:250}
REPS=${REPS:-2}
: > "$OUT/ab.jsonl"
for r in $(seq 1 "$REPS"); do
  for sh in $SHAPES; do
    IFS=: read -r S F0 NF <<< "$sh"
    for lib in $LIBS; do
      MCGRAPH_LIB=$PWD/$lib timeout -k 10 240 python scripts/bp_profile.py "$S" "$F0" "$NF" 3 > "$OUT/one.json" 2> "$OUT/one.err" \
        || { echo "bp_profile $lib $sh failed"; tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json,sys; d=json.load(open('$OUT/one.json')); print(json.dumps({'lib': '$lib', 'rep': $r, 'window': '$sh', 'wall_ms': d['wall_ms'], **d['group_ms']}))" >> "$OUT/ab.jsonl"
    done
  done
done
cat "$OUT/ab.jsonl"
