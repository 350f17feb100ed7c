#!/usr/bin/env bash
# Round 5, call c: every C4 frame's S1 against the oracle (the full C4 E2E test), the denoise stamps
# and group times on a C3 window, and the L2 request-size counter passes of the S1 kernels on the same
# window (scripts/pmc_sizes.py: traffic without the blanket FETCH_SIZE doubling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5c}
mkdir -p $OUT
run() { echo "== $* $(date +%T)" >&2; "$@"; local rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
run timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -x -v --timeout 500 --timeout-method thread -m gpu -k "c4" \
    > $OUT/pytest_c4.out 2>&1 || { tail -30 $OUT/pytest_c4.out; exit 1; }
tail -2 $OUT/pytest_c4.out
fi
run timeout -k 10 200 python -u scripts/bp_profile.py c3 600 100 3 > $OUT/bp_profile_c3.json 2> $OUT/bp_profile_c3.err || { tail -5 $OUT/bp_profile_c3.err; exit 1; }
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_stamps.so MCGRAPH_LIB_PARTIAL=1 run timeout -k 10 200 python -u scripts/bp_stamps.py c3 600 100 \
    > $OUT/stamps_c3.txt 2>&1 || { tail -5 $OUT/stamps_c3.txt; exit 1; }
RAW=/tmp/mc_raw_$$
mkdir -p $RAW
i=0
for SET in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_BUBBLE_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"; do
  i=$((i+1))
  run timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "k_bp_" --output-format csv \
      -d $RAW/p$i -o run -- python3 scripts/bp_profile.py c3 600 100 1 > $OUT/sizes$i.log 2>&1 \
      || { echo "pass $i failed"; tail -5 $OUT/sizes$i.log; exit 1; }
  find $RAW/p$i -name "*counter_collection.csv" -exec cp {} $RAW/sizes$i.csv \;
done
python3 scripts/pmc_sizes.py $RAW $OUT/pmc_sizes_c3w.json "k_bp_" | tee $OUT/pmc_sizes_c3w.txt
rm -rf $RAW
