#!/usr/bin/env bash
# Round 5, call q: the voxel kernel's chunk loop with the sums' stores waited for under the next
# chunk's points (prefetch behind the sums' loads): S1 suite, stamps, bench (against fold4: the
# round-5 r5n kernel with a 4-wide fold), C3 end to end on every frame; then the rank proxy (one
# rank's device work at N = 8: its S1 slice beside the whole scene's graph stages).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5q}
SKIP_C3=1 OUT=$OUT bash scripts/gpu_r5n.sh || exit $?
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_fold4.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench_fold4.json 2> $OUT/bench_fold4.err || { tail -20 $OUT/bench_fold4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench_fold4.json').read().strip().splitlines()[-1]); print('bench fold4', d['ms_per_step'], d['config']['stage_ms']['bp_voxel'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -x -v --timeout 500 --timeout-method thread -m gpu -k "c3" \
    > $OUT/pytest_c3.out 2>&1
rc=$?; echo "== C3 E2E rc=$rc: $(tail -1 $OUT/pytest_c3.out)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/rank_proxy.py c3 4 8 > $OUT/rank_proxy_c3.jsonl 2> $OUT/rank_proxy_c3.err
rc=$?; cat $OUT/rank_proxy_c3.jsonl; [ $rc -eq 0 ] || tail -20 $OUT/rank_proxy_c3.err; exit $rc
