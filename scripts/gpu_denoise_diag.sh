#!/usr/bin/env bash
# Denoise diagnostics on one box: per-phase clock shares (a -DMC_BP_STAMPS build, built beforehand as
# maskclustering_amd/libmcgraph_stamps.so) and SQ / TCP counter passes over the LDS denoise classes
# on a C3 frame slice (scripts/bp_profile.py).  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/denoise_diag}
SHAPE=${SHAPE:-c3}
F0=${F0:-0}
NF=${NF:-100}
mkdir -p "$OUT"
if [ -f maskclustering_amd/libmcgraph_stamps.so ]; then
  MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so timeout -k 10 240 python3 scripts/bp_stamps.py "$SHAPE" "$F0" "$NF" \
      > "$OUT/stamps.txt" 2> "$OUT/stamps.err" || { tail -5 "$OUT/stamps.err"; exit 1; }
  cat "$OUT/stamps.txt"
fi
K=${K:-k_bp_denoise_lds}
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "$K" --output-format csv -d "$OUT/p$i" -o run -- \
      python3 scripts/bp_profile.py "$SHAPE" "$F0" "$NF" 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/p$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 scripts/pmc_kernel.py "$K" "$OUT"/p*.csv > "$OUT/summary.json"
rm -f "$OUT"/p*.csv
cat "$OUT/summary.json"
