#!/usr/bin/env bash
# How much more batching would give: the default (5 batches of 300 C3 frames) against 4 batches of 375.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3l}
OUT=$OUT ENVS="- MC_BP_BATCH_PIXELS=1100000000" REPS=1 timeout -k 10 500 bash scripts/gpu_env_ab.sh
