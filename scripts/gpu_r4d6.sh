#!/usr/bin/env bash
# After moving the ring kernel's grid description to the top of the slot: the class diagnostic
# (non-dbg, 4 repeats; dbg) and the S1 GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4d6}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/diag_classes.py 4 > $OUT/diag.out 2>&1 || { tail -20 $OUT/diag.out; exit 1; }
tail -3 $OUT/diag.out
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/diag_classes.py 1 > $OUT/diag_dbg.out 2>&1 || { tail -20 $OUT/diag_dbg.out; exit 1; }
grep -E "bp dbg|differing" $OUT/diag_dbg.out | head -20
timeout -k 10 300 python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_s1.out 2>&1 || { tail -30 $OUT/pytest_s1.out; exit 1; }
tail -2 $OUT/pytest_s1.out
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 250 --timeout-method thread -m gpu -k "invariants" > $OUT/pytest_s1_dbg.out 2>&1 || { tail -30 $OUT/pytest_s1_dbg.out; exit 1; }
tail -2 $OUT/pytest_s1_dbg.out
