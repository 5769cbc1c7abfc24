#!/bin/bash
# wide-row pass B1's recurrence coefficients formed from the twiddles (in-tree library) against
# the previous tree (lib/exp/orig.so): wide-row parity tests, then kernel times (8192^2 F32 x2, F64)
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/b1calc
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_edge.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "8192 or widest or wide or config5" > gpurun_out/b1calc/tests.log 2>&1 || { tail -30 gpurun_out/b1calc/tests.log; exit 1; }
tail -1 gpurun_out/b1calc/tests.log
for rep in 1 2; do
  tools/prof_lib.sh b1f$rep orig -- --n 8192 --dtype f32 --steps 20 > gpurun_out/b1calc/ab32_$rep.txt 2>&1 || exit 2
  grep -E "==|pass" gpurun_out/b1calc/ab32_$rep.txt
done
tools/prof_lib.sh b1d orig -- --n 8192 --steps 20 > gpurun_out/b1calc/ab64.txt 2>&1 || exit 3
grep -E "==|pass" gpurun_out/b1calc/ab64.txt
