#!/usr/bin/env bash
# Builds a diagnostics / A-B variant of libmcgraph.so in-tree (here, on the CPU; the .so travels to the
# GPU box with the snapshot):  scripts/build_variant.sh NAME [-DFLAG=VALUE ...]
#   -> maskclustering_amd/libmcgraph_NAME.so, selected per process with MCGRAPH_LIB=<path>.
#   dbg:    scripts/build_variant.sh dbg -DMC_DBG_CHECK=1     (in-kernel invariant checks)
#   stamps: scripts/build_variant.sh stamps -DMC_BP_STAMPS     (per-phase clock shares)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall "$@" \
    -o "maskclustering_amd/libmcgraph_${name}.so" maskclustering_amd/csrc/mc_api.hip
# the same flags' device code must hold no spill store before an EXEC restore (such a
# build computes wrong results); a failing variant is removed rather than left to be run
if ! python3 scripts/spill_exec_check.py --build "$@" k_ > "/tmp/spill_check_${name}.txt"; then
    cat "/tmp/spill_check_${name}.txt" >&2
    rm -f "maskclustering_amd/libmcgraph_${name}.so"
    echo "spill placement check failed for ${name}: try other flags (e.g. -DMC_DBG_NOINLINE=0/1, -DMC_DBG_PRINT=0)" >&2
    exit 1
fi
echo "maskclustering_amd/libmcgraph_${name}.so"
