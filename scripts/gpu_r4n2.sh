#!/usr/bin/env bash
# Round 4: the default bench (C3 E2E, frame-sharded, graph stages row-block sharded) with 2 ranks
# sharing the one GPU over gloo: the path the driver's multi-GPU runs take, minus RCCL (batches
# capped: two ranks share one device's HBM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4n2}
mkdir -p "$OUT"
timeout -k 10 600 env MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 MC_BP_BATCH_PIXELS=300000000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --no-secondary \
    > "$OUT/n2_e2e_c3.json" 2> "$OUT/n2_e2e_c3.err" || { tail -20 "$OUT/n2_e2e_c3.err"; exit 1; }
cat "$OUT/n2_e2e_c3.json"
