mkdir -p gpurun_out/r4d5
DIAG_VERBOSE=1 MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/diag_classes.py 1 > gpurun_out/r4d5/diag_dbg.out 2>&1 || exit 1
grep -E "dbg origin|dbg ring|a \(|run joined=./min_class=4" gpurun_out/r4d5/diag_dbg.out | head -30
