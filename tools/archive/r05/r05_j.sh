#!/bin/bash
# round 5 (j): cl2 = tw1 + the pass B coefficient tables in LDS with the one-buffer transform
# (4096-point pass B and both wide-row B passes) + stage-2 twiddle powers in SGPRs only where
# they measured faster (4096 pass A, wide-row B0).  Parity first, then a same-box A/B against
# tw1 and sg, three interleaved repeats.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05j; mkdir -p $O
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/cl2.so timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_f32.py tests/test_gpu_configs.py > $O/tests_cl2.log 2>&1 || { tail -20 $O/tests_cl2.log; exit 4; }
echo "cl2: $(tail -1 $O/tests_cl2.log)"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in tw1 sg cl2; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    for C in "8192 f32" "4096 f64"; do
      set -- $C; N=$1; D=$2
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${N}_$rep -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $R/$O/b_${v}_${N}_$rep.json 2> $R/$O/b_${v}_${N}_$rep.err || exit 5
      echo "== $v $N $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${N}_$rep.json | head -1) | $(python3 $R/tools/kstats.py $R/$O/p_${v}_${N}_$rep/k_kernel_stats.csv | grep -E 'pass|carry|tendency' | awk '{printf "%s %s; ", $1, $5}')"
    done
  done
done
