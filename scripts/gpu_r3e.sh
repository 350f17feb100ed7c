#!/usr/bin/env bash
# The S1-related GPU tests on the default build (union half-loads, ordered stats without compares),
# the reference-API path at C2 / C3 / replay, and the 2-rank frame-sharded bench on one GPU (gloo).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3e}
mkdir -p "$OUT"
# variant parity runs: a failing assertion (pytest rc 1) is recorded and the script goes on; any
# other failure (timeout, fault, abort) ends it
vstep() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?
    tail -3 "$OUT/$name.out"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "$name rc=$rc"; exit 1; }; echo "$name rc=$rc"; }
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -20 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -3 "$OUT/$name.out"; }
step pytest 400 python -u -m pytest tests/test_gpu_s1.py tests/test_gpu_bench_configs.py tests/test_gpu_api.py \
    tests/test_gpu_frame_shard.py -x -v --timeout 200 --timeout-method thread -m gpu
OUT=$OUT/api timeout -k 10 900 bash scripts/gpu_api.sh || { echo "api failed"; exit 1; }
step n2_e2e_c2 300 env MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --shape c2 --steps 3 --warmup 1 --no-secondary
step stamps 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so python scripts/bp_stamps.py c3 600 100
vstep pytest_vr 200 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_vr.so python -u -m pytest tests/test_gpu_s1.py -x -q \
    --timeout 120 --timeout-method thread -m gpu
vstep pytest_p1 200 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_p1.so python -u -m pytest tests/test_gpu_s1.py -x -q \
    --timeout 120 --timeout-method thread -m gpu
echo "== spread / minmax A/B $(date +%T)"
OUT=$OUT/ab_spread_mm LIBS="maskclustering_amd/libmcgraph_prev.so maskclustering_amd/libmcgraph_spread.so maskclustering_amd/libmcgraph.so maskclustering_amd/libmcgraph_vr.so maskclustering_amd/libmcgraph_vs.so maskclustering_amd/libmcgraph_p1.so" SHAPES="c3:600:100 c2:0:250" REPS=1 \
    timeout -k 10 540 bash scripts/gpu_ab_s1.sh || { echo "spread A/B failed"; exit 1; }
