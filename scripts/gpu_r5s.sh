#!/usr/bin/env bash
# Round 5, call s: the C3 bench at three batch sizes (MC_BP_BATCH_PIXELS: 250 / 125 / 63 frames of
# 1920x1440 per batch) -- the per-batch fixed cost of S1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5s}
mkdir -p $OUT
for fr in 250 125 63; do
  MC_BP_BATCH_PIXELS=$((fr * 1920 * 1440)) timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-secondary --no-cpu-baseline > $OUT/bench_b$fr.json 2> $OUT/bench_b$fr.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench_b$fr.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_b$fr.json').read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('batch $fr frames', d['ms_per_step'], d['config']['objects'], {k:s[k] for k in ('bp_pixels','bp_voxel','bp_denoise','bp_query')}, d['roofline']['launches_timed'])"
done
