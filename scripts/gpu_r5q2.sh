#!/usr/bin/env bash
# Round 5, call q2: the four-rank rehearsal of the default bench over gloo on the one GPU (scene-owner
# graph stages, two S1 producers per rank from N = 4 on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5q2}
mkdir -p $OUT
timeout -k 10 700 env MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 4 --warmup 1 --no-secondary \
    > "$OUT/n4_e2e_c3.json" 2> "$OUT/n4_e2e_c3.err" || { tail -30 "$OUT/n4_e2e_c3.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/n4_e2e_c3.json').read().strip().splitlines()[-1]); print('n4 gloo one GPU', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['config']['parallelism'], d['config']['s1_producers'])"
