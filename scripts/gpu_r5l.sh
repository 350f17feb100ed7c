#!/usr/bin/env bash
# r5l: split eps lists (owner-packed forward run + atomic backward run).  Every GPU test + smoke on
# the new build, then the default C3 bench line A/B against the previous build (MCGRAPH_LIB), two
# alternations.  Each GPU step has its own limit; a failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5l}
mkdir -p "$OUT"
run() { echo "== $* $(date +%T)" >&2; "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  run timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
for i in 1 2; do
  run timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > "$OUT/bench_new_$i.json" 2> "$OUT/bench_new_$i.err" \
      || { tail -20 "$OUT/bench_new_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_new_$i.json').read().strip().splitlines()[-1]); print('new', d['ms_per_step'], d['config']['stage_ms']['bp_denoise'], d['config']['objects'])"
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_head.so run timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary \
      > "$OUT/bench_head_$i.json" 2> "$OUT/bench_head_$i.err" || { tail -20 "$OUT/bench_head_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_head_$i.json').read().strip().splitlines()[-1]); print('head', d['ms_per_step'], d['config']['stage_ms']['bp_denoise'], d['config']['objects'])"
done
