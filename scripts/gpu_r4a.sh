#!/usr/bin/env bash
# Round 4, call a (the first box of the round; steps in order of importance, each with its own limit):
# S1 + reference-API GPU tests on the default build (denoise split, fused union, reference orders),
# a short default bench line, the S1 group A/B of the new builds against the build before the
# split, and the in-kernel invariant checks (libmcgraph_dbg.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4a}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_s1_api 420 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_api.py -x -v --timeout 200 \
    --timeout-method thread -m gpu
step bench_e2e_c3 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
L=maskclustering_amd
export MCGRAPH_LIB_PARTIAL=1
OUT=$OUT/ab_c3 SHAPES="c3:600:100" REPS=1 \
    LIBS="$L/libmcgraph_presplit.so $L/libmcgraph_nofuse.so $L/libmcgraph.so $L/libmcgraph_vxre.so $L/libmcgraph_vxfr.so $L/libmcgraph_vxfrre.so" \
    timeout -k 10 400 bash scripts/gpu_ab_s1.sh || { echo "A/B failed"; exit 1; }
step pytest_s1_dbg 400 env MCGRAPH_LIB=$PWD/$L/libmcgraph_dbg.so python -u -m pytest tests/test_gpu_s1.py \
    -v --timeout 300 --timeout-method thread -m gpu -k "invariants or glue or classes"
