#!/usr/bin/env bash
# Round 5, call p: the voxel kernel with a load wave (chunk 256, three workgroups per CU: default
# build; chunk 192, four per CU: vxl192) against the one without (fold4): S1 suite on the default
# and vxl192, voxel phase stamps on the C3 window for all three, bench for all three.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5p}
mkdir -p $OUT
L=$PWD/maskclustering_amd
for v in "" vxl192; do
  lib=$L/libmcgraph${v:+_$v}.so
  MCGRAPH_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_s1_${v:-def}.out 2>&1
  rc=$?; echo "== S1 suite ${v:-def} rc=$rc: $(tail -1 $OUT/pytest_s1_${v:-def}.out)"; [ $rc -eq 0 ] || { tail -30 $OUT/pytest_s1_${v:-def}.out; exit $rc; }
done
for v in stamps stamps192 stampsf4; do
  MCGRAPH_LIB=$L/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
      > $OUT/stamps_$v.txt 2>&1 || { tail -5 $OUT/stamps_$v.txt; exit 1; }
  echo "== $v: $(grep -E 'call ms|k_bp_voxel_lds' $OUT/stamps_$v.txt | head -3 | tr '\n' ' ')"
done
for v in "" vxl192 fold4; do
  MCGRAPH_LIB=$L/libmcgraph${v:+_$v}.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench_${v:-def}.json 2> $OUT/bench_${v:-def}.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench_${v:-def}.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_${v:-def}.json').read().strip().splitlines()[-1]); print('bench ${v:-def}', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['config']['stage_ms']['bp_voxel'])"
done
