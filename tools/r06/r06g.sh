#!/bin/bash
# r06g: F32 solve error per path after SPL_U_F64, the F32 edge tests, then the probe rehearsal
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/r06g
O=gpurun_out/r06g
timeout -k 10 300 python tools/r06/f32_solve_err.py 8192:16 20000:4 20000:8 16384:32 9000:4 5000:32 1000:64 > $O/f32_solve_err.txt 2>&1 || exit 1
cat $O/f32_solve_err.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_f32.py -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "f32 or split or bluestein or wide" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log; grep -E "psi_err" $O/tests.log | cut -c1-300
tools/r06/r06d.sh
