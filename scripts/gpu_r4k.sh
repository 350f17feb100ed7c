#!/usr/bin/env bash
# Round 4: launch-size A/B of the denoise group (host-side knobs, the kernels' code unchanged): the
# ring-search grid (MC_BP_RING_WGS per CU: 4 / 8 / 16) and the class-kernel grid multiplier
# (MC_BP_OVERSUB_RT: 1 / 2 / 3), C3 frames 600-699, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4k}
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for r in 1 2; do
  for cfg in "8 2" "4 2" "16 2" "8 1" "8 3"; do
    set -- $cfg
    MC_BP_RING_WGS=$1 MC_BP_OVERSUB_RT=$2 timeout -k 10 200 python scripts/bp_profile.py c3 600 100 3 > "$OUT/one.json" 2> "$OUT/one.err" \
      || { echo "bp_profile $cfg failed"; tail -5 "$OUT/one.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/one.json')); print(json.dumps({'ring_wgs': $1, 'oversub': $2, 'rep': $r, 'wall_ms': d['wall_ms'], **d['group_ms']}))" >> "$OUT/ab.jsonl"
  done
done
cat "$OUT/ab.jsonl"
