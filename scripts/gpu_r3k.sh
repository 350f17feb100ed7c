#!/usr/bin/env bash
# Per-phase stamps of the final denoise build (C3 frames 600-699).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r3k}
mkdir -p "$OUT"
timeout -k 10 240 env MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so python scripts/bp_stamps.py c3 600 100 \
    > "$OUT/stamps.txt" 2> "$OUT/stamps.err" || { tail -5 "$OUT/stamps.err"; exit 1; }
cat "$OUT/stamps.txt"
