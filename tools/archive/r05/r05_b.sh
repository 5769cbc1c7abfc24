#!/bin/bash
# round 5 (b): lane-exchange transform in the wide-row passes (M = 8192): the 8192 parity
# tests, then base vs current at 8192^2 F32 (config 5) and 4096^2 F64, kernel stats of both.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_f32.py tests/test_gpu_configs.py "tests/test_gpu_multirank.py::test_slabs_match_single_gpu" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
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
for v in base cur; do
  L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
  QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof8_$v -o $v -- python3 $R/bench.py --n 8192 --dtype f32 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --steps 20 --warmup 5 > $R/$O/pb8_$v.json 2> $R/$O/pb8_$v.err || exit 6
  python3 $R/tools/kstats.py $R/$O/prof8_$v/${v}_kernel_stats.csv
done
