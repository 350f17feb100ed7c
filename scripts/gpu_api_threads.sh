mkdir -p gpurun_out/apithr
for t in 16 8 4; do
  OMP_NUM_THREADS=$t timeout -k 10 200 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 > gpurun_out/apithr/t$t.json 2> gpurun_out/apithr/t$t.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/apithr/t$t.json').read().strip().splitlines()[-1]); print($t, d['value'], d['config']['part_ms'])"
done
