#!/usr/bin/env bash
# Round 5, call u: batches sized by mask pixels (the expected share learned from the previous call;
# grow-and-redo when a batch has more): S1 suite, bench, C3 and C4 end to end on every frame.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5u}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 280 --timeout-method thread -m gpu > $OUT/pytest_s1.out 2>&1
rc=$?; echo "== S1 suite rc=$rc: $(tail -1 $OUT/pytest_s1.out)"; [ $rc -eq 0 ] || { tail -30 $OUT/pytest_s1.out; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('bench', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], {k:s[k] for k in ('bp_pixels','bp_voxel','bp_denoise','bp_query')}, d['roofline']['launches_timed'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_configs.py -x -v --timeout 800 --timeout-method thread -m gpu -k "c3 or c4" \
    > $OUT/pytest_c3c4.out 2>&1
rc=$?; echo "== C3/C4 E2E rc=$rc: $(tail -1 $OUT/pytest_c3c4.out)"; exit $rc
