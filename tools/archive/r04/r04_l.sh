#!/bin/bash
# round 4 (l): tendency with rotated ring slots / induction row pointers (scalar-unit load):
# bitwise tests, then interleaved kernel stats base (lib/exp/base.so) vs current, 4096^2 F64
# and 8192^2 F32, plus the SALU counters of the new build.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tendency_kernels.py tests/test_gpu_pair_bitwise.py tests/test_gpu_parity.py tests/test_gpu_pcg.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base cur; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    for cfg in 4096f64 8192f32; do
      A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${cfg}_$rep -o k -- python3 $R/bench.py $A --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_${cfg}_$rep.json 2> $R/$O/b_${v}_${cfg}_$rep.err || exit 5
      echo "== $v $cfg $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${cfg}_$rep.json | head -1)"
      python3 $R/tools/kstats.py $R/$O/p_${v}_${cfg}_$rep/k_kernel_stats.csv | sed -n 2,3p
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc -o k -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/pmc.log 2>&1 || exit 6
