#!/usr/bin/env bash
# Round 4, call d: the per-class denoise tails' parity failure (r4c) characterised before anything
# else runs: every class x both tail modes x repeats on the tiny dense scene, with the differing
# statistics printed; then the same under the in-kernel invariant build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r4d}
mkdir -p "$OUT"
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" \
    || { echo "$name failed"; tail -30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }; tail -12 "$OUT/$name.out"; }
step diag 240 python -u scripts/diag_classes.py 4
step diag_dbg 300 env DIAG_VERBOSE=1 MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so python -u scripts/diag_classes.py 1
