#!/bin/bash
# the alternating walk in both tendency kernels (in-tree library) against the previous tree
# (lib/exp/orig.so): parity tests, then kernel time and PMC reads at 4096^2 F64 and 8192^2 F32
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/alt2
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tendency_kernels.py tests/test_gpu_pair_bitwise.py tests/test_gpu_multirank.py tests/test_gpu_dropin.py tests/test_gpu_f32.py tests/test_gpu_rccl_ring.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/alt2/tests.log 2>&1 || { tail -30 gpurun_out/alt2/tests.log; exit 1; }
tail -1 gpurun_out/alt2/tests.log
tools/prof_lib.sh a64 orig > gpurun_out/alt2/ab64.txt 2>&1 || exit 2
tools/prof_lib.sh a32 orig -- --n 8192 --dtype f32 --steps 20 > gpurun_out/alt2/ab32.txt 2>&1 || exit 2
grep -E "==|tendency" gpurun_out/alt2/ab64.txt gpurun_out/alt2/ab32.txt
cd /tmp && export TMPDIR=/tmp
for cfg in "64 --n 4096" "32 --n 8192 --dtype f32"; do
  set -- $cfg; tag=$1; shift
  for n in default orig; do
    L=""; [ $n != default ] && L=$R/julia-ocean-modelling_amd/lib/exp/$n.so
    QGMI355_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/alt2/pmc_${tag}_$n -o f -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --no-pmc-live --no-reference-runs --dropin-steps 0 "$@" > $R/gpurun_out/alt2/pmc_${tag}_$n.log 2>&1 || exit 3
    python3 -c "
import sys; sys.path.insert(0, '$R')
import bench, glob
f = glob.glob('$R/gpurun_out/alt2/pmc_${tag}_$n/**/*counter_collection.csv', recursive=True)[0]
m, k = bench.pmc_counter_mean(f, 'FETCH_SIZE')
print('$tag $n tendency FETCH_SIZE x2 per launch: %.1f MB (%d launches)' % (2 * m * 1024 / 1e6, k))
"
  done
done
