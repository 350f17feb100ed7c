#!/usr/bin/env bash
# Round 4, call g: HEAD (joined denoise tails by default, grid description at the top of the slot,
# recycled set-order tables): every GPU test, the class diagnostic against the oracle, the default
# bench line, and the voxel phase ablations (timing-only builds) for the next voxel change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4g}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step diag 240 python -u scripts/diag_classes.py 2
step bench 600 python -u bench.py
L=maskclustering_amd
export MCGRAPH_LIB_PARTIAL=1
OUT=$OUT/ab_vx SHAPES="c3:600:100" REPS=2 \
    LIBS="$L/libmcgraph.so $L/libmcgraph_vxab1.so $L/libmcgraph_vxab2.so $L/libmcgraph_vxfr.so" \
    timeout -k 10 300 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
