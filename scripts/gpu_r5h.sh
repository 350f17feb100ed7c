#!/usr/bin/env bash
# Round 5, call h: k-NN fill by a 20-input sorting network (first 20 selected entries, then inserts)
# against the committed build (headstamps), stamps on the C3 window for both; S1 suite; bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5h}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_s1.out 2>&1
rc=$?; echo "== S1 suite rc=$rc: $(tail -1 $OUT/pytest_s1.out)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_s1.out | head -20; exit $rc; }
for v in stamps headstamps stamps headstamps; do
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
      > $OUT/stamps_$v.txt 2>&1 || { tail -5 $OUT/stamps_$v.txt; exit 1; }
  echo "== $v: $(grep -E 'call ms|ncount|union  |knn  ' $OUT/stamps_$v.txt | head -4 | tr '\n' ' ')"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "== bench rc=$rc: $(python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"; exit $rc
