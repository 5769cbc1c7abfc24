#!/bin/bash
# round 5 (e): Bluestein rows (odd M > 8192, M > 16384) against the oracle; the comm tests
# after the region_create / comm_barrier rewrite; the 1-rank ring without gather / pin.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_gpu_edge.py" tests/test_gpu_rccl_ring.py tests/test_gpu_comm_failure.py tests/test_gpu_rccl_multirank.py tests/test_gpu_multirank.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "bluestein or generic_rows_wide or wide_split or rccl or peer or ring or slab or silent or failure" > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|residuals" $O/tests.log | tail -60; tail -3 $O/tests.log; exit $rc
