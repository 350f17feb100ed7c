#!/usr/bin/env bash
# Round 5, call r2: the one-GPU C3 bench with one vs two S1 producers (MC_BENCH_S1_PRODUCERS), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5r2}
mkdir -p $OUT
for i in 1 2; do
  for P in 1 2; do
    MC_BENCH_S1_PRODUCERS=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary \
        > "$OUT/bench_p${P}_$i.json" 2> "$OUT/bench_p${P}_$i.err" || { tail -20 "$OUT/bench_p${P}_$i.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_p${P}_$i.json').read().strip().splitlines()[-1]); print('producers $P', d['ms_per_step'], d['config']['objects'], d['roofline']['avg_launch_ms'])"
  done
done
