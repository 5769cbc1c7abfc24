#!/bin/bash
# round 5 (h): same-box A/B of the pass changes (kernel stats from rocprofv3 over the bench's steps):
#   tw1 = split twiddles from registers; ln = tw1 + SGPR-base row addressing; cur = ln + stage-2
#   twiddle powers in SGPRs; pbA / pbB = cur + the 4096 pass B's next coefficients loaded before the
#   row's stores / before its transform; e1 = pbB + the wide-row B1's coefficients loaded early.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05h; mkdir -p $O
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/e1.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py::test_widest_rows_8192 tests/test_gpu_f32.py > $O/tests_e1.log 2>&1 || { tail -20 $O/tests_e1.log; exit 4; }
tail -1 $O/tests_e1.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in tw1 ln cur pbA pbB e1; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    for C in "8192 f32" "4096 f64"; do
      set -- $C; N=$1; D=$2
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${N}_$rep -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $R/$O/b_${v}_${N}_$rep.json 2> $R/$O/b_${v}_${N}_$rep.err || exit 5
      echo "== $v $N $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${N}_$rep.json | head -1) | $(python3 $R/tools/kstats.py $R/$O/p_${v}_${N}_$rep/k_kernel_stats.csv | grep -E 'pass|carry|tendency' | awk '{printf "%s %s; ", $1, $5}')"
    done
  done
done
