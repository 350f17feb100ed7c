#!/usr/bin/env bash
# Round 5, call t2: multi-workgroup S1 batch scans.  Every GPU test + smoke on the new build, the
# default C3 line A/B against the previous build (MCGRAPH_LIB), alternated twice, and the kernel trace
# of the scans (scripts/gpu_r5s2.sh) on the new build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5t2}
mkdir -p "$OUT"
run() { echo "== $* $(date +%T)" >&2; "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
run timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for i in 1 2; do
  run timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > "$OUT/bench_new_$i.json" 2> "$OUT/bench_new_$i.err" \
      || { tail -20 "$OUT/bench_new_$i.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_new_$i.json').read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('new', d['ms_per_step'], s['bp_pixels'], s['bp_query'], d['config']['objects'])"
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_head.so run timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary \
      > "$OUT/bench_head_$i.json" 2> "$OUT/bench_head_$i.err" || { tail -20 "$OUT/bench_head_$i.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_head_$i.json').read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('head', d['ms_per_step'], s['bp_pixels'], s['bp_query'], d['config']['objects'])"
done
OUT=$OUT bash scripts/gpu_r5s2.sh
