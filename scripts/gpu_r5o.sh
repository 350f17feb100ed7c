#!/usr/bin/env bash
# Round 5, call o: scene-owner graph stages.  One rank's device work at N = 8 (scripts/rank_proxy.py,
# now also in scene-owner form), the two-rank rehearsal of the default bench (scene-owner on) over gloo
# on the one GPU, and the 2-rank GPU frame-shard tests.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5o}
mkdir -p $OUT
[ "${SKIP_PROXY:-0}" = 1 ] || timeout -k 10 400 python scripts/rank_proxy.py c3 8 8 > "$OUT/rank_proxy_c3.jsonl" 2> "$OUT/rank_proxy_c3.err" \
    || { tail -20 "$OUT/rank_proxy_c3.err"; exit 1; }
[ "${SKIP_PROXY:-0}" = 1 ] || cat "$OUT/rank_proxy_c3.jsonl"
timeout -k 10 600 env MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --no-secondary \
    > "$OUT/n2_e2e_c3.json" 2> "$OUT/n2_e2e_c3.err" || { tail -20 "$OUT/n2_e2e_c3.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/n2_e2e_c3.json').read().strip().splitlines()[-1]); print('n2 gloo one GPU', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['config']['parallelism'])"
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame_shard.py -x -v --timeout 400 --timeout-method thread -m gpu > $OUT/pytest_shard.out 2>&1
rc=$?; echo "== shard tests rc=$rc: $(tail -1 $OUT/pytest_shard.out)"; exit $rc
