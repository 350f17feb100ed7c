#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ablate.jsonl
for lib in maskclustering_amd/libmcgraph.so $(ls build/variants/*.so 2>/dev/null); do
  MCGRAPH_LIB=$PWD/$lib timeout -k 10 300 python scripts/ablate.py ${SHAPE:-c2} >> gpurun_out/ablate.jsonl 2> gpurun_out/ablate.err
  rc=$?; [ $rc -eq 0 ] || { echo "ablate $lib rc=$rc"; tail -5 gpurun_out/ablate.err; exit $rc; }
done
cat gpurun_out/ablate.jsonl
