#!/usr/bin/env bash
# Round 5, call n: the run-based voxel kernel (chunk-ordered sums, no per-pixel lists): S1 suite, C3
# end to end against the oracle on every frame (SKIP_C3=1: not), voxel phase stamps on the C3 window,
# default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5n}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_s1.out 2>&1
rc=$?; echo "== S1 suite rc=$rc: $(tail -1 $OUT/pytest_s1.out)"; [ $rc -eq 0 ] || { tail -30 $OUT/pytest_s1.out; exit $rc; }
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_stamps.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
    > $OUT/stamps_c3.txt 2>&1 || { tail -5 $OUT/stamps_c3.txt; exit 1; }
echo "== stamps: $(grep -E 'call ms|k_bp_voxel_lds' $OUT/stamps_c3.txt | head -3 | tr '\n' ' ')"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['config']['stage_ms'])"
[ "${SKIP_C3:-0}" = 1 ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -x -v --timeout 500 --timeout-method thread -m gpu -k "c3" \
    > $OUT/pytest_c3.out 2>&1
rc=$?; echo "== C3 E2E rc=$rc: $(tail -1 $OUT/pytest_c3.out)"; exit $rc
