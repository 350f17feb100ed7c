#!/usr/bin/env bash
# rocprofv3 --kernel-trace --stats over a python command; only the per-kernel stats CSV is copied
# to <out csv> (the per-dispatch trace stays in /tmp):  bash scripts/trace_pass.sh <out csv> <python args...>
set -u
dst=$1; shift
raw=/tmp/trace_raw_$$
mkdir -p "$raw"
timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --stats -d "$raw" -o trace --output-format csv -- python3 "$@"
rc=$?
f=$(find "$raw" -name "trace_kernel_stats.csv" | head -n 1)
if [ -z "$f" ]; then echo "no kernel stats (rocprofv3 rc=$rc)" >&2; exit 1; fi
cp "$f" "$dst"
