mkdir -p gpurun_out/r4d4
DIAG_VERBOSE=1 MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_dbg.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/diag_classes.py 1 > gpurun_out/r4d4/diag_dbg.out 2>&1 || exit 1
grep -A40 "dbg ring" gpurun_out/r4d4/diag_dbg.out | head -30
MCGRAPH_LIB=$PWD/maskclustering_amd/libmcgraph_r4f1.so MCGRAPH_LIB_PARTIAL=1 timeout -k 10 200 python -u scripts/diag_classes.py 2 > gpurun_out/r4d4/diag_r4f1.out 2>&1 || exit 1
tail -8 gpurun_out/r4d4/diag_r4f1.out
