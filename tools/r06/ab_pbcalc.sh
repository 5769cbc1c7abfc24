#!/bin/bash
# pass B's recurrence coefficients formed from the twiddles (in-tree library) against the
# previous tree (lib/exp/orig.so): spectral parity tests, then kernel times twice each
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/pbcalc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_multirank.py tests/test_gpu_f32.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not realisations and not smooth" > gpurun_out/pbcalc/tests.log 2>&1 || { tail -30 gpurun_out/pbcalc/tests.log; exit 1; }
tail -1 gpurun_out/pbcalc/tests.log
for rep in 1 2; do
  tools/prof_lib.sh pb$rep orig > gpurun_out/pbcalc/ab64_$rep.txt 2>&1 || exit 2
  grep -E "==|passB|passA" gpurun_out/pbcalc/ab64_$rep.txt
done
tools/prof_lib.sh pb32 orig -- --n 8192 --dtype f32 --steps 20 > gpurun_out/pbcalc/ab32.txt 2>&1 || exit 3
grep -E "==|pass" gpurun_out/pbcalc/ab32.txt
