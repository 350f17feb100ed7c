#!/usr/bin/env bash
# SQ/TCP counter passes for one kernel (default k_s3_masks) over graph builds
# (scripts/ablate.py), each pass its own run; summary via scripts/pmc_kernel.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_kernel}
K=${K:-k_s3_masks}
SHAPE=${SHAPE:-c2}
mkdir -p "$OUT"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES" \
           "SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_CYCLES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-include-regex "$K" --output-format csv -d "$OUT/p$i" -o run -- \
      python3 ${PROG:-scripts/ablate.py} "$SHAPE" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  find "$OUT/p$i" -name "*counter_collection.csv" -exec mv {} "$OUT/p$i.csv" \;
  rm -rf "$OUT/p$i"
done
python3 scripts/pmc_kernel.py "$K" "$OUT"/p*.csv | tee "$OUT/summary.json"
