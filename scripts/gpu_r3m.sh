#!/usr/bin/env bash
# A repeat of every GPU test on the final tree (run-to-run stability of the parity results).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3m}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu.log"; exit $rc
