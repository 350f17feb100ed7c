#!/usr/bin/env bash
# Round 5, call m: the scene pipeline in the default bench (S1 of scene k + 1 under the graph stages
# of scene k): one GPU, pipeline on and off; then the two-rank rehearsal over gloo on the one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5m}
mkdir -p "$OUT"
MC_BENCH_PIPELINE=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench_pipe.json 2> $OUT/bench_pipe.err
rc=$?; echo "== pipeline rc=$rc: $(tail -c 300 $OUT/bench_pipe.json | head -c 300)"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_pipe.err; exit $rc; }
MC_BENCH_PIPELINE=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-secondary > $OUT/bench_seq.json 2> $OUT/bench_seq.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench_seq.err; exit $rc; }
python3 -c "
import json
for n in ('pipe','seq'):
    d=json.loads(open('$OUT/bench_'+n+'.json').read().strip().splitlines()[-1]); print(n, d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['roofline']['avg_launch_ms'])"
timeout -k 10 600 env MC_BENCH_PIPELINE=1 MC_BENCH_BACKEND=gloo MC_BENCH_DEVICE=0 MC_BP_BATCH_PIXELS=300000000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --no-secondary \
    > "$OUT/n2_e2e_c3.json" 2> "$OUT/n2_e2e_c3.err" || { tail -20 "$OUT/n2_e2e_c3.err"; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/n2_e2e_c3.json').read().strip().splitlines()[-1]); print('n2 gloo one GPU', d['ms_per_step'], d['config']['objects'], d['config']['iterations'], d['config']['scene_pipeline'])"
