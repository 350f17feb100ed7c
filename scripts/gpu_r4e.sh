#!/usr/bin/env bash
# Round 4, call e: every GPU test on the release build at HEAD (the per-class denoise tails, queue
# regions sized by the classifier), the class diagnostic against the oracle, the tail A/B and the
# reference-API C2 path under cProfile.  Each step has its own limit; a failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4e}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step diag 240 python -u scripts/diag_classes.py 3
for r in 1 2; do
  for mode in 0 1; do
    MC_BP_TAIL_JOINED=$mode timeout -k 10 240 python scripts/bp_profile.py c3 600 100 3 > "$OUT/tail_$mode.json" 2> "$OUT/tail_$mode.err" \
      || { echo "bp_profile tail $mode failed"; tail -5 "$OUT/tail_$mode.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/tail_$mode.json')); print(json.dumps({'tail_joined': $mode, 'rep': $r, 'wall_ms': d['wall_ms'], **d['group_ms']}))" >> "$OUT/tail_ab.jsonl"
  done
done
cat "$OUT/tail_ab.jsonl"
step api_c2_prof 300 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 --with-pp --profile
