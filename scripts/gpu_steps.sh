#!/usr/bin/env bash
# Run a list of GPU steps, each under its own time limit, stopping at the first failure.
#   OUT=gpurun_out/x bash scripts/gpu_steps.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/steps}
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd" >&2
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "rc=$rc" >&2
  tail -3 "$OUT/$name.out"; tail -5 "$OUT/$name.err" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
exit 0
