#!/usr/bin/env bash
# Round 5, call e: the Afforest-style DBSCAN union (pair pass without speculative unions) on the S1
# suite, the diagnostics build (class diagnostic + invariants), the stamps of the C3 window, and the
# default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_s1.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_s1.out 2>&1
rc=$?; echo "== S1 suite rc=$rc: $(tail -1 $OUT/pytest_s1.out)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_s1.out | head -20; exit $rc; }
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 150 python -u scripts/diag_classes.py 2 > $OUT/diag_dbg.out 2>&1
rc=$?; echo "== dbg diag rc=$rc: $(grep -c 'bp dbg' $OUT/diag_dbg.out) dbg prints; $(head -2 $OUT/diag_dbg.out | tail -1 | cut -c1-200); $(tail -1 $OUT/diag_dbg.out)"; [ $rc -eq 0 ] || exit $rc
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 180 --timeout-method thread -m gpu -k "invariants" > $OUT/pytest_inv_dbg.out 2>&1
rc=$?; echo "== dbg invariants rc=$rc: $(tail -1 $OUT/pytest_inv_dbg.out)"; [ $rc -eq 0 ] || exit $rc
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_stamps.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 > $OUT/stamps_c3.txt 2>&1
rc=$?; echo "== stamps rc=$rc: $(grep -E 'call ms|ncount|union  |knn  ' $OUT/stamps_c3.txt | head -4 | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "== bench rc=$rc: $(python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('stage_ms'))")"; exit $rc
