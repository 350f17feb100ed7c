mkdir -p gpurun_out/apithr2
# C2 reference-API path: the set-order replay's worker count (default: half the CPU share) against 12 / 16
for cfg in "0" "12" "16" "0" "12" "16"; do
  MC_SETORDER_THREADS=$cfg timeout -k 10 200 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 \
      > gpurun_out/apithr2/t$cfg.json 2> gpurun_out/apithr2/t$cfg.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/apithr2/t$cfg.json').read().strip().splitlines()[-1]); print('setorder threads $cfg', d['value'], d['config']['part_ms'])"
done
