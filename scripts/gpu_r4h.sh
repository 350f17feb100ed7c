#!/usr/bin/env bash
# Round 4, call h: the late k-NN set-up build (MC_BP_KNN_LATE_INIT=1, fewer spills) against HEAD:
# its S1 tests and class diagnostic against the oracle first, then the S1 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4h}
mkdir -p "$OUT"
L=$PWD/maskclustering_amd
export MCGRAPH_LIB_PARTIAL=1
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_s1_knnlate 300 env MCGRAPH_LIB=$L/libmcgraph_knnlate.so python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_bench_configs.py -x -q --timeout 250 --timeout-method thread -m gpu -k "not c4"
step diag_knnlate 240 env MCGRAPH_LIB=$L/libmcgraph_knnlate.so python -u scripts/diag_classes.py 2
OUT=$OUT/ab SHAPES="c3:600:100 c2:0:250" REPS=3 \
    LIBS="maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_knnlate.so" \
    timeout -k 10 400 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
