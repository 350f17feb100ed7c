#!/usr/bin/env bash
# Environment-knob A/B on one box: the C3 E2E bench (no CPU baseline, no secondary record) once per
# setting in ENVS (space-separated VAR=value items; "-" = no knob), alternating REPS times; one line
# per run with the per-scene ms and the group times.  Each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/envab}
ENVS=${ENVS:-"- MC_BP_BIG_CUS=64 MC_BP_BIG_CUS=128"}
REPS=${REPS:-2}
SHAPE=${SHAPE:-c3}
STEPS=${STEPS:-5}
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for r in $(seq 1 "$REPS"); do
  for e in $ENVS; do
    if [ "$e" = "-" ]; then set -- ; else set -- "$e"; fi
    timeout -k 10 300 env "$@" python bench.py --shape "$SHAPE" --steps "$STEPS" --warmup 1 --no-cpu-baseline \
        --no-secondary > "$OUT/one.json" 2> "$OUT/one.err" || { echo "bench $e failed"; tail -5 "$OUT/one.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/one.json')); print(json.dumps({'env': '$e', 'rep': $r, 'ms': d['ms_per_step'], **d['config']['stage_ms']}))" >> "$OUT/ab.jsonl"
    tail -1 "$OUT/ab.jsonl"
  done
done
