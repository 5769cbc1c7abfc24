#!/bin/bash
# alternating strip walk (lib/exp/alt.so): bitwise parity tests on it, then A/B timing + PMC
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/alt
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/alt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tendency_kernels.py tests/test_gpu_multirank.py tests/test_gpu_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/alt/tests.log 2>&1 || { tail -30 gpurun_out/alt/tests.log; exit 1; }
tail -2 gpurun_out/alt/tests.log
tools/prof_lib.sh alt1 alt > gpurun_out/alt/ab.txt 2>&1 && tools/prof_lib.sh alt2 alt >> gpurun_out/alt/ab.txt 2>&1 || exit 2
cat gpurun_out/alt/ab.txt
cd /tmp && export TMPDIR=/tmp
for n in default alt; do
  L=""; [ $n != default ] && L=$R/julia-ocean-modelling_amd/lib/exp/$n.so
  QGMI355_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/alt/pmc_$n -o f -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --no-pmc-live --no-reference-runs --dropin-steps 0 > $R/gpurun_out/alt/pmc_$n.log 2>&1 || exit 3
  python3 -c "
import sys; sys.path.insert(0, '$R')
import bench, glob
f = glob.glob('$R/gpurun_out/alt/pmc_$n/**/*counter_collection.csv', recursive=True)[0]
m, k = bench.pmc_counter_mean(f, 'FETCH_SIZE')
print('$n tendency FETCH_SIZE x2 per launch: %.1f MB (%d launches)' % (2 * m * 1024 / 1e6, k))
"
done
