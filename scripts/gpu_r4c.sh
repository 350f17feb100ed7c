#!/usr/bin/env bash
# Round 4, call c: where the time goes after the denoise split.  Per-phase stamps of the class
# kernels (libmcgraph_stamps.so, C3 frames 600-699), and the reference-API C2 path under cProfile
# (reference orders with post_process, then canonical) to split its host time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4c}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
export MCGRAPH_LIB_PARTIAL=1
step pytest_s1 300 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 200 --timeout-method thread -m gpu
step stamps_c3 300 env MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_stamps.so python -u scripts/bp_stamps.py c3 600 100
step api_c2_prof 300 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 --with-pp --profile
step api_c2_canonical_prof 300 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 --canonical --profile
# voxel phase shares of the current kernel (timing-only ablations: 1 = no phases 3-4, 2 = no phase 4)
L=maskclustering_amd
OUT=$OUT/ab_vx SHAPES="c3:600:100" REPS=2 \
    LIBS="$L/libmcgraph.so $L/libmcgraph_vxab1.so $L/libmcgraph_vxab2.so $L/libmcgraph_vxfr.so" \
    timeout -k 10 300 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
# denoise tails per class (default) against one joined tail (MC_BP_TAIL_JOINED=1), alternating
for r in 1 2; do
  for mode in 0 1; do
    MC_BP_TAIL_JOINED=$mode timeout -k 10 240 python scripts/bp_profile.py c3 600 100 3 > "$OUT/tail_$mode.json" 2> "$OUT/tail_$mode.err" \
      || { echo "bp_profile tail $mode failed"; tail -5 "$OUT/tail_$mode.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/tail_$mode.json')); print(json.dumps({'tail_joined': $mode, 'rep': $r, 'wall_ms': d['wall_ms'], **d['group_ms']}))" >> "$OUT/tail_ab.jsonl"
  done
done
cat "$OUT/tail_ab.jsonl"
