#!/usr/bin/env bash
# S1 batch size: the C3 E2E bench at the default batch cap (640 M pixels) and at 1 G pixels per batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3h}
OUT=$OUT ENVS="- MC_BP_BATCH_PIXELS=1000000000" REPS=2 timeout -k 10 700 bash scripts/gpu_env_ab.sh
