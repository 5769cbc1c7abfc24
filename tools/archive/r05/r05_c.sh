#!/bin/bash
# round 5 (c): slot-ordered u / coefficients in the lane-exchange passes: quick parity
# subset, then base vs current (4096^2 F64, 8192^2 F32), kernel stats of current.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_f32.py tests/test_gpu_pcg.py tests/test_gpu_tendency_kernels.py tests/test_gpu_pair_bitwise.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base cur; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    for cfg in 8192f32 4096f64; do
      A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"
      QGMI355_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 10 $A --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b_${v}_${cfg}_$rep.json 2> $O/b_${v}_${cfg}_$rep.err || exit 5
      echo "== $v $cfg $rep $(grep -o '"value": [0-9.]*' $O/b_${v}_${cfg}_$rep.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_${cfg}_$rep.json | head -1)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for cfg in 8192f32 4096f64; do
  A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$cfg -o cur -- python3 $R/bench.py $A --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --steps 20 --warmup 5 > $R/$O/pb_$cfg.json 2> $R/$O/pb_$cfg.err || exit 6
  python3 $R/tools/kstats.py $R/$O/prof_$cfg/cur_kernel_stats.csv
done
