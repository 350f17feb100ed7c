#!/usr/bin/env bash
# Round 4, call b: S1 group times of the default build (denoise split) against the build before the
# split and the voxel-recompute variant, alternating (scripts/gpu_ab_s1.sh over bp_profile.py); then
# the S1 voxel / class tests on the recompute variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4b}
mkdir -p "$OUT"
export MCGRAPH_LIB_PARTIAL=1
OUT=$OUT/ab LIBS="maskclustering_amd/libmcgraph_presplit.so maskclustering_amd/libmcgraph_nofuse.so maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_vxre.so" \
    REPS=2 timeout -k 10 900 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
timeout -k 10 300 env MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_vxre.so python -u -m pytest tests/test_gpu_s1.py -x -q \
    --timeout 200 --timeout-method thread -m gpu -k "voxel or dense or classes or stages" > "$OUT/pytest_vxre.out" 2>&1 \
    || { echo "vxre tests failed"; tail -30 "$OUT/pytest_vxre.out"; exit 1; }
tail -3 "$OUT/pytest_vxre.out"
