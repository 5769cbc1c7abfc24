#!/bin/bash
# round 4 (p): chip-full count of the tendency (QG_TEND_WAVES) re-swept after the scalar-unit
# changes: 4096^2 F64 (one-point kernel, default 6) and 8192^2 F32 (pair kernel, default 6),
# two interleaved repeats, kernel stats.  CFGS / WS override the lists.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r04p; mkdir -p $O
for rep in ${REPS:-1 2}; do
  for cfg in ${CFGS:-4096f64 8192f32}; do
    A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"; [ $cfg = 8192f64 ] && A="--n 8192"
    for w in ${WS:-3 4 5 6 7 8 10}; do
      QG_TEND_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${cfg}_w${w}_$rep -o k -- python3 $R/bench.py $A --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b_${cfg}_w${w}_$rep.json 2> $O/b_${cfg}_w${w}_$rep.err || exit 5
      echo "== $cfg w$w $rep $(python3 $R/tools/kstats.py $O/p_${cfg}_w${w}_$rep/k_kernel_stats.csv | grep tendency | head -1)"
    done
  done
done
