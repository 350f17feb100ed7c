#!/usr/bin/env bash
# Final records of a round on one box, in two calls (each under gpurun's limit):
#   PART=records: every GPU test + smoke, the default bench line, the C4 line, the C5 sweep line;
#   PART=profiles: rocprofv3 kernel stats of the bench command, the HBM traffic passes (FETCH_SIZE /
#     WRITE_SIZE, one per run), the SQ counter passes of the denoise kernels over a C3 window
#     (bp_profile.py), the two-rank rehearsal of the N > 1 bench (gloo, one device) and the rank proxy.
# Each GPU step has its own limit; a failure ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final}
PART=${PART:-records}
mkdir -p "$OUT"
run() { echo "== $* $(date +%T)" >&2; "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ "$PART" = records ]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  run timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  run timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
  run timeout -k 10 300 python bench.py --shape c4 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary \
      > "$OUT/bench_e2e_c4.json" 2> "$OUT/bench_e2e_c4.err" || { tail -20 "$OUT/bench_e2e_c4.err"; exit 1; }
  run timeout -k 10 300 python bench.py --variant sweep > "$OUT/bench_sweep_c5.json" 2> "$OUT/bench_sweep_c5.err" \
      || { tail -20 "$OUT/bench_sweep_c5.err"; exit 1; }
  cat "$OUT/bench_sweep_c5.json"
  exit 0
fi
RAW=/tmp/mc_raw_$$
mkdir -p "$RAW"
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-latency > "$OUT/prof_bench.json" \
    2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
find "$RAW/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 scripts/kstats.py "$OUT/kernel_stats.csv" | head -40
for C in FETCH_SIZE WRITE_SIZE; do
  run timeout -s KILL 180 rocprofv3 --pmc "$C" --output-format csv -d "$RAW/pmc_$C" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-latency > "$OUT/pmc_$C.json" \
      2> "$OUT/pmc_$C.err" || { tail -20 "$OUT/pmc_$C.err"; exit 1; }
  find "$RAW/pmc_$C" -name "*counter_collection.csv" -exec cp {} "$RAW/pmc_$C.csv" \;
done
python3 scripts/pmc_summary.py "$RAW" "$OUT/pmc_traffic.json"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  run timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "k_bp_denoise|k_bp_knn_ring" --output-format csv \
      -d "$RAW/sq$i" -o run -- python3 scripts/bp_profile.py c3 600 100 1 > "$OUT/sq$i.log" 2>&1 \
      || { echo "SQ pass $i failed"; tail -5 "$OUT/sq$i.log"; exit 1; }
  find "$RAW/sq$i" -name "*counter_collection.csv" -exec cp {} "$RAW/sq$i.csv" \;
done
python3 scripts/pmc_kernel.py "k_bp_" "$RAW"/sq*.csv > "$OUT/denoise_sq_counters_c3.json"
rm -rf "$RAW"
run timeout -k 10 300 env MC_BENCH_DEVICE=0 MC_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 4 --warmup 1 \
    > "$OUT/n2_e2e_c3.json" 2> "$OUT/n2_e2e_c3.err" || { tail -20 "$OUT/n2_e2e_c3.err"; exit 1; }
run timeout -k 10 400 python scripts/rank_proxy.py c3 6 2 4 8 > "$OUT/rank_proxy_c3.jsonl" 2> "$OUT/rank_proxy_c3.err" \
    || { tail -20 "$OUT/rank_proxy_c3.err"; exit 1; }
ls -la "$OUT"
exit 0
