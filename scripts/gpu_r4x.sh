#!/usr/bin/env bash
# Round 4, call x (extras at HEAD): the reference-API path on C3 (uint16 depth frames through the
# get_depth_raw hook, reference container orders, no post_process), the C5 312-scene sweep, C4 E2E.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4x}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -2 "$OUT/$name.out"; }
export MCGRAPH_LIB_PARTIAL=1
L=$PWD/maskclustering_amd
step pytest_s1_fdiv 300 env MCGRAPH_LIB=$L/libmcgraph_fdiv.so python -u -m pytest tests/test_gpu_s1.py -x -q --timeout 250 --timeout-method thread -m gpu
step diag_fdiv 240 env MCGRAPH_LIB=$L/libmcgraph_fdiv.so python -u scripts/diag_classes.py 1
OUT=$OUT/ab SHAPES="c3:600:100 c2:0:250" REPS=3 \
    LIBS="maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_fdiv.so" \
    timeout -k 10 400 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
step sweep_c2 400 python -u bench.py --variant sweep --steps 1 --warmup 1 --no-cpu-baseline
step e2e_c4 300 python -u bench.py --shape c4 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
step api_c3 500 python -u bench.py --variant api --shape c3 --steps 2 --warmup 1
