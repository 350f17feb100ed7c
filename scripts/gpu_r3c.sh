#!/usr/bin/env bash
# S1 tests on the default build (ring culling + split k-NN), the base / cull / default A/B, the API
# path's upload-batch count, and the 2-rank frame-sharded bench on the one GPU (gloo).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3c}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -20 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest_s1 300 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_bench_configs.py -x -v --timeout 200 --timeout-method thread -m gpu
echo "== knn A/B $(date +%T)"
OUT=$OUT/ab_knn LIBS="maskclustering_amd/libmcgraph_base.so maskclustering_amd/libmcgraph_cull.so maskclustering_amd/libmcgraph.so" REPS=1 \
    timeout -k 10 500 bash scripts/gpu_ab_s1.sh || { echo "knn A/B failed"; exit 1; }
for nb in 1 2 4 8; do
  step api_c2_ub$nb 200 env MC_BP_UPLOAD_BATCHES=$nb python bench.py --variant api --shape c2 --steps 5 --warmup 2
done
step n2_e2e_c2 420 env MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --shape c2 --steps 3 --warmup 1
