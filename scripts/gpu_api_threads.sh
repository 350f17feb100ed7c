mkdir -p gpurun_out/apithr
# C2 reference-API path: the set-order replay on a persistent worker pool (default) against a pool
# per call (MC_SETORDER_PERSIST=0), and at 16 / 8 host threads
for cfg in "16 1" "16 0" "8 1" "16 1" "16 0"; do
  set -- $cfg
  OMP_NUM_THREADS=$1 MC_SETORDER_PERSIST=$2 timeout -k 10 200 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 \
      > gpurun_out/apithr/t$1_p$2.json 2> gpurun_out/apithr/t$1_p$2.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/apithr/t$1_p$2.json').read().strip().splitlines()[-1]); print('threads $1 persist $2', d['value'], d['config']['part_ms'])"
done
