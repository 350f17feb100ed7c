#!/usr/bin/env bash
# Round 5, call a: which property of the MC_DBG_CHECK build makes its DBSCAN results differ from the
# oracle (verdict r4 item 1).  The same source built five ways (scripts/build_variant.sh):
#   dbg          the diagnostics build as shipped (noinline check functions with device printf)
#   dbginl       the checks inlined (no calls in the class kernels)
#   dbgnoprint   noinline checks, no printf (counters only)
#   dbgnospill   the class kernels at 2 waves per SIMD (256 VGPRs: no spills), checks as in dbg
#   relnospill   the release kernels at 2 waves per SIMD
# each on the class diagnostic (scripts/diag_classes.py: every size class and tail mode against the
# oracle), then the in-kernel invariant test on the ones whose diagnostic equals the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5a}
mkdir -p $OUT
for v in ${VARIANTS:-dbginl dbgnoprint dbgnospill relnospill}; do
    MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 150 \
        python -u scripts/diag_classes.py 1 > $OUT/diag_$v.out 2>&1
    rc=$?
    echo "== $v rc=$rc: $(grep -c 'vs oracle' $OUT/diag_$v.out) runs differing from the oracle; $(grep -c 'bp dbg' $OUT/diag_$v.out) dbg prints; $(tail -1 $OUT/diag_$v.out)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/diag_$v.out; exit $rc; fi
done
for v in dbginl dbgnoprint dbgnospill; do
    MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 \
        python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 180 --timeout-method thread -m gpu -k "invariants" \
        > $OUT/pytest_inv_$v.out 2>&1
    rc=$?
    echo "== invariants $v rc=$rc: $(tail -1 $OUT/pytest_inv_$v.out)"
    if [ $rc -gt 1 ]; then exit $rc; fi
done
exit 0
