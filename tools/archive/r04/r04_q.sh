#!/bin/bash
# round 4 (q): new tendency chip-full defaults: bitwise / parity tests, then the bench (driver
# flags) base (lib/exp/base.so, the old counts) vs current, 3 interleaved repeats, 4096^2 F64
# and 8192^2 F32 (config 5).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tendency_kernels.py tests/test_gpu_pair_bitwise.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in base cur; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    for cfg in 4096f64 8192f32; do
      A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"
      QGMI355_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $A --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b_${v}_${cfg}_$rep.json 2> $O/b_${v}_${cfg}_$rep.err || exit 5
      echo "== $v $cfg $rep $(grep -o '"value": [0-9.]*' $O/b_${v}_${cfg}_$rep.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_${cfg}_$rep.json | head -1)"
    done
  done
done
