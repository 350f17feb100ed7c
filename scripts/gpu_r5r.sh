#!/usr/bin/env bash
# Round 5, call r: the diagnostics-build invariants test (worker process on libmcgraph_dbg.so); then
# timing-only builds (results differ by design) that replace the voxel / cell floor divisions
# (ablfdiv), the world-point divisions (ablwdiv) or both (abldiv) by reciprocal multiplies: how much of
# S1 the f64 divisions cost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5r}
mkdir -p $OUT
L=$PWD/maskclustering_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 280 --timeout-method thread -m gpu -k "diagnostics_build or in_kernel" > $OUT/pytest_dbg.out 2>&1
rc=$?; echo "== dbg test rc=$rc: $(tail -1 $OUT/pytest_dbg.out)"; [ $rc -eq 0 ] || { tail -30 $OUT/pytest_dbg.out; exit $rc; }
for v in "" ablfdiv ablwdiv abldiv; do
  MCGRAPH_LIB=$L/libmcgraph${v:+_$v}.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline > $OUT/bench_${v:-def}.json 2> $OUT/bench_${v:-def}.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench_${v:-def}.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_${v:-def}.json').read().strip().splitlines()[-1]); s=d['config']['stage_ms']; print('bench ${v:-def}', d['ms_per_step'], d['config']['objects'], {k:s[k] for k in ('bp_pixels','bp_voxel','bp_denoise','bp_query')})"
done
MCGRAPH_LIB=$L/libmcgraph_stampsabldiv.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 > $OUT/stamps_abldiv.txt 2>&1 || { tail -5 $OUT/stamps_abldiv.txt; exit 1; }
grep -E "call ms|k_bp_voxel_lds|ncount|knn  |bbox|cells" $OUT/stamps_abldiv.txt | head -8
