#!/bin/bash
# round 5 (g): where the wide-row pass A's time goes -- the transform microbench with the next
# row prefetched (one- vs two-buffer transform) and phase stamps of spec_passA_half at 8192^2 F32.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 120 ./tools/microbench/fft_lx > $O/fft_lx.txt 2>&1 || { tail -5 $O/fft_lx.txt; exit 2; }
grep -E "pf|one-buffer" $O/fft_lx.txt
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampAH.so timeout -k 10 200 python tools/stamps/stamps_passA_half.py 8192 f32 > $O/stampsAH_8192f32.txt 2>&1 || { tail -5 $O/stampsAH_8192f32.txt; exit 3; }
cat $O/stampsAH_8192f32.txt
# A/B: split twiddles from registers (current tree) vs LDS tables (base5 = HEAD), 8192^2 F32 and F64
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_edge.py -k "widest_rows_8192" tests/test_gpu_f32.py tests/test_gpu_configs.py > $O/tests_wide.log 2>&1 || { tail -20 $O/tests_wide.log; exit 4; }
tail -2 $O/tests_wide.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base5 cur; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so; [ $v = cur ] && L=$R/julia-ocean-modelling_amd/lib/libqgmi355.so
    for D in f32 f64; do
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${D}_$rep -o k -- python3 $R/bench.py --n 8192 --dtype $D --steps 20 --warmup 5 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_${D}_$rep.json 2> $R/$O/b_${v}_${D}_$rep.err || exit 5
      echo "== $v $D $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${D}_$rep.json | head -1)"
      python3 $R/tools/kstats.py $R/$O/p_${v}_${D}_$rep/k_kernel_stats.csv | grep -E "half|tendency"
    done
  done
done
