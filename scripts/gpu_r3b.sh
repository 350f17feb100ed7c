#!/usr/bin/env bash
# One box, in order of importance; each step has its own time limit and a failure ends the script:
# the S1 GPU tests (incl. the per-batch host staging), the reference-API path at C2 with per-batch
# staging, a C3 kernel trace (per-batch group / class spans), the frame-sharded bench with 2 ranks on
# the one GPU (gloo), the API path at C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3b}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -20 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_s1 300 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_frame_shard.py -x -v --timeout 120 --timeout-method thread -m gpu
step api_c2 300 python bench.py --variant api --shape c2 --steps 5 --warmup 2
echo "== ktrace $(date +%T)"
OUT=$OUT/kt timeout -k 10 700 bash scripts/gpu_ktrace_c3.sh || { echo "ktrace failed"; exit 1; }
step stamps 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so python scripts/bp_stamps.py c3 600 100
echo "== env A/B $(date +%T)"
OUT=$OUT/envab REPS=1 timeout -k 10 400 bash scripts/gpu_env_ab.sh || { echo "env A/B failed"; exit 1; }
step pytest_cull 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_cull.so python -u -m pytest tests/test_gpu_s1.py -x -q \
    --timeout 120 --timeout-method thread -m gpu
echo "== cull A/B $(date +%T)"
OUT=$OUT/ab_cull LIBS="maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_cull.so" REPS=1 \
    timeout -k 10 400 bash scripts/gpu_ab_s1.sh || { echo "cull A/B failed"; exit 1; }
