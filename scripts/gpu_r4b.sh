#!/usr/bin/env bash
# Round 4, call b: S1 group times, alternating builds (scripts/gpu_ab_s1.sh over bp_profile.py): the
# build before the denoise split, the split without / with the fused union (default), and the voxel
# variants (recompute, fused ranks, both); then the S1 tests on each voxel variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4b}
mkdir -p "$OUT"
export MCGRAPH_LIB_PARTIAL=1
L=maskclustering_amd
OUT=$OUT/ab_c3 SHAPES="c3:600:100" REPS=2 \
    LIBS="$L/libmcgraph_presplit.so $L/libmcgraph_nofuse.so $L/libmcgraph.so $L/libmcgraph_vxre.so $L/libmcgraph_vxfr.so $L/libmcgraph_vxfrre.so" \
    timeout -k 10 800 bash scripts/gpu_ab_s1.sh || { echo "A/B c3 failed"; exit 1; }
OUT=$OUT/ab_c2 SHAPES="c2:0:250" REPS=1 \
    LIBS="$L/libmcgraph_presplit.so $L/libmcgraph_nofuse.so $L/libmcgraph.so $L/libmcgraph_vxre.so $L/libmcgraph_vxfr.so $L/libmcgraph_vxfrre.so" \
    timeout -k 10 400 bash scripts/gpu_ab_s1.sh || { echo "A/B c2 failed"; exit 1; }
for v in vxre vxfr vxfrre; do
  timeout -k 10 300 env MCGRAPH_LIB=$PWD/$L/libmcgraph_$v.so python -u -m pytest tests/test_gpu_s1.py -x -q \
      --timeout 200 --timeout-method thread -m gpu -k "voxel or dense or stages or glue" > "$OUT/pytest_$v.out" 2>&1 \
      || { echo "$v tests failed"; tail -30 "$OUT/pytest_$v.out"; exit 1; }
  tail -1 "$OUT/pytest_$v.out"
done
