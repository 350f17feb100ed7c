#!/usr/bin/env bash
# Reference-API boundary after the host-loop changes: the API / post-process GPU tests, then C2 (with a
# cProfile step) and C3 through the drop-in modules.  Each step has its own limit; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5api2
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_pp.py > "$OUT/pytest.out" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.out"; exit 1; }
tail -3 "$OUT/pytest.out"
run() { local name=$1; shift; timeout -k 10 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }; cat "$OUT/$name.json"; }
run api_c2 300 python bench.py --variant api --shape c2 --steps 5 --warmup 2 --profile
run api_c3 600 python bench.py --variant api --shape c3 --steps 3 --warmup 1
