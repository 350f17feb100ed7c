#!/usr/bin/env bash
# Final round-3 measurement on the default build: every GPU test, smoke, bench, rocprofv3 stats, PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/v8} bash scripts/gpu_round.sh
