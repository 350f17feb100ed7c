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
echo "maskclustering_amd/libmcgraph_${name}.so"
