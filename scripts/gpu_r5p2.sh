#!/usr/bin/env bash
# Round 5, call p2: one rank's device work at N = 1 / 8 with two S1 producers (scripts/rank_proxy.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r5p2}
mkdir -p $OUT
timeout -k 10 500 python scripts/rank_proxy.py c3 8 8 > "$OUT/rank_proxy_c3.jsonl" 2> "$OUT/rank_proxy_c3.err" \
    || { tail -20 "$OUT/rank_proxy_c3.err"; exit 1; }
cat "$OUT/rank_proxy_c3.jsonl"
