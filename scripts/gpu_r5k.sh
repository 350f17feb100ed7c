#!/usr/bin/env bash
# Round 5, call k: S6 components of levels >= 1 in one launch when N_1 is small (N_1 read back after
# level 0): the graph-stage GPU tests (parity, large scenes C3/C4 against the sparse oracle), then the
# default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5k}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_frame_shard.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_graph.out 2>&1
rc=$?; echo "== graph tests rc=$rc: $(tail -1 $OUT/pytest_graph.out)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_graph.out | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "== bench rc=$rc: $(python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);c=d['config'];print(d['ms_per_step'], {k:v for k,v in c['stage_ms'].items() if not k.startswith('bp')}, d['secondary']['c2_g'])")"; exit $rc
