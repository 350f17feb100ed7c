#!/usr/bin/env bash
# Round 5, call g: far links kept in registers + batched k-NN entry fetches, validated as in r5e (S1
# suite, diagnostics build, stamps, bench); then the pair pass's stamp in three timing-only builds
# (results wrong by design): no LDS atomics (ablnoatomic), no list stores (ablnostore), neither
# (ablnone).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5g}
OUT=$OUT bash scripts/gpu_r5e.sh || exit $?
for v in ablnoatomic ablnostore ablnone; do
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
      > $OUT/stamps_$v.txt 2>&1 || { tail -5 $OUT/stamps_$v.txt; exit 1; }
  echo "== $v: $(grep -E 'ncount' $OUT/stamps_$v.txt | head -1)"
done
