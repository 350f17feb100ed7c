#!/usr/bin/env bash
# Round 4, call a: S1 GPU tests on the default build (list-cap and repeat tests included), the same
# suite on the in-kernel-check build (libmcgraph_dbg.so, scripts/build_variant.sh dbg), and a short
# default bench line as the round's starting point.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4a}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_s1 500 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_api.py -x -v --timeout 200 --timeout-method thread -m gpu
step bench_e2e_c3 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
step pytest_s1_dbg 600 env MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so python -u -m pytest tests/test_gpu_s1.py \
    -v --timeout 400 --timeout-method thread -m gpu
