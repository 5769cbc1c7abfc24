#!/bin/bash
# round 5 (g): where the lane-exchange passes' time goes -- the transform microbench with the
# next row prefetched (one- vs two-buffer transform), phase stamps of the wide-row pass A and
# the 4096-point pass B -- then parity of the current tree and a same-box A/B:
#   base5 = HEAD before (split twiddles from LDS tables), tw1 = split twiddles from registers,
#   cur = tw1 + stage-2 twiddle powers in SGPRs + SGPR-base row addressing.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 120 ./tools/microbench/fft_lx > $O/fft_lx.txt 2>&1 || { tail -5 $O/fft_lx.txt; exit 2; }
grep -E "pf|one-buffer" $O/fft_lx.txt
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampAH.so timeout -k 10 200 python tools/stamps/stamps_phases.py 8192 f32 A > $O/stampsAH_8192f32.txt 2>&1 || { tail -5 $O/stampsAH_8192f32.txt; exit 3; }
cat $O/stampsAH_8192f32.txt
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampB4.so timeout -k 10 200 python tools/stamps/stamps_phases.py 4096 f64 B > $O/stampsB4_4096f64.txt 2>&1 || { tail -5 $O/stampsB4_4096f64.txt; exit 3; }
cat $O/stampsB4_4096f64.txt
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py::test_widest_rows_8192 tests/test_gpu_f32.py > $O/tests_par.log 2>&1 || { tail -20 $O/tests_par.log; exit 4; }
tail -2 $O/tests_par.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base5 tw1 cur; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so; [ $v = cur ] && L=$R/julia-ocean-modelling_amd/lib/libqgmi355.so
    for C in "8192 f32" "4096 f64"; do
      set -- $C; N=$1; D=$2
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${N}_$rep -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $R/$O/b_${v}_${N}_$rep.json 2> $R/$O/b_${v}_${N}_$rep.err || exit 5
      echo "== $v $N $D $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${N}_$rep.json | head -1)"
      python3 $R/tools/kstats.py $R/$O/p_${v}_${N}_$rep/k_kernel_stats.csv | grep -E "pass|carry"
    done
  done
done
