#!/usr/bin/env bash
# Round 5, call d (timing-only builds, results wrong by design): the denoise pair pass's stamp without
# its fused union (ablunion) and without its two scattered u16 list stores (ablstore), against the
# stamps build of the shipped source (r5c: 134.6 us per slot).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5d}
mkdir -p $OUT
for v in stamps ablunion ablstore; do
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
      > $OUT/stamps_$v.txt 2>&1 || { tail -5 $OUT/stamps_$v.txt; exit 1; }
  echo "== $v: $(grep -E 'call ms|ncount|knn  ' $OUT/stamps_$v.txt | tr '\n' ' ')"
done
