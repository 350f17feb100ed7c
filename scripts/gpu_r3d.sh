#!/usr/bin/env bash
# Round-3 measurement call: the full round (every GPU test, smoke, bench, rocprofv3 stats, PMC traffic)
# on the default build, then the union-walk A/B and the API path's upload-batch count.  Each step has
# its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/v5}
OUT=$OUT bash scripts/gpu_round.sh || { echo "round failed"; exit 1; }
echo "== union A/B $(date +%T)"
OUT=$OUT/ab_union LIBS="maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_uh.so" SHAPES="c3:600:100 c2:0:250" REPS=1 \
    timeout -k 10 300 bash scripts/gpu_ab_s1.sh || { echo "union A/B failed"; exit 1; }
for nb in 1 8; do
  echo "== api ub$nb $(date +%T)"
  timeout -k 10 150 env MC_BP_UPLOAD_BATCHES=$nb python bench.py --variant api --shape c2 --steps 5 --warmup 2 \
      > "$OUT/api_c2_ub$nb.json" 2> "$OUT/api_c2_ub$nb.err" || { echo "api ub$nb failed"; exit 1; }
  cat "$OUT/api_c2_ub$nb.json"
done
