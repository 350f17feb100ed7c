#!/usr/bin/env bash
# Lane-group ring search (MC_RING_PAIRS=2 / 4 builds): their S1 parity runs, then the A/B against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3g}
mkdir -p "$OUT"
echo "== pytest_pairs $(date +%T)"
timeout -k 10 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_pairs.so python -u -m pytest tests/test_gpu_s1.py \
    tests/test_gpu_bench_configs.py -x -q --timeout 200 --timeout-method thread -m gpu > "$OUT/pytest_pairs.out" 2> "$OUT/pytest_pairs.err"
rc=$?; tail -3 "$OUT/pytest_pairs.out"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
echo "== pytest_quads $(date +%T)"
timeout -k 10 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_quads.so python -u -m pytest tests/test_gpu_s1.py \
    tests/test_gpu_bench_configs.py -x -q --timeout 200 --timeout-method thread -m gpu > "$OUT/pytest_quads.out" 2> "$OUT/pytest_quads.err"
rc=$?; tail -3 "$OUT/pytest_quads.out"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
echo "== pairs A/B $(date +%T)"
OUT=$OUT/ab_pairs LIBS="maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_pairs.so maskclustering_amd/libmcgraph_quads.so" SHAPES="c3:600:100 c2:0:250" REPS=2 \
    timeout -k 10 480 bash scripts/gpu_ab_s1.sh || { echo "pairs A/B failed"; exit 1; }
