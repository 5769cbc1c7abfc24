#!/bin/bash
# r06e: the F32 tests with the mechanism's bars, then the bench probe rehearsal (r06d)
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/r06e
O=gpurun_out/r06e
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_f32.py "tests/test_gpu_edge.py::test_bluestein_rows_f32" "tests/test_gpu_edge.py::test_wide_split_rows_f32" "tests/test_gpu_rccl_multirank.py::test_rccl_config_slabs_match_single_gpu" -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "config 5|RCCL|PASSED|FAILED|passed|failed|M=|psi_err" $O/tests.log | cut -c1-400
tools/r06/r06d.sh
