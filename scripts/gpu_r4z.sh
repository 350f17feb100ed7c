#!/usr/bin/env bash
# Round 4, last check at HEAD (host-side set-order changes since r4f4): the reference-API GPU tests,
# the S1 suite, smoke, and the C2 API line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4z}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -2 "$OUT/$name.out"; }
step pytest_api_s1 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_s1.py tests/test_gpu_frame_shard.py -x -q --timeout 300 --timeout-method thread -m gpu
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step api_c2 300 python -u bench.py --variant api --shape c2 --steps 5 --warmup 2 --with-pp
