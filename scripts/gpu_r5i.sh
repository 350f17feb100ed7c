#!/usr/bin/env bash
# Round 5, call i: voxel-kernel phase stamps (stamps build) and the k-NN list pass without its
# fetch / insert loop (ablknnins, timing only) on the C3 window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5i}
mkdir -p $OUT
for v in ${VARIANTS:-stamps ablknnins}; do
  MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_$v.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
      > $OUT/stamps_$v.txt 2>&1 || { tail -5 $OUT/stamps_$v.txt; exit 1; }
  echo "== $v: $(grep -E 'call ms|knn  |k_bp_voxel_lds' $OUT/stamps_$v.txt | head -4 | tr '\n' ' ')"
done
