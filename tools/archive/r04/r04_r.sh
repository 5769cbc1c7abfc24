#!/bin/bash
# round 4 (r): spec_passB<4096> experiments.  Phase stamps (tools/stamps) of the variants listed in
# STAMPS, then kernel stats of the current library vs the variants in VARS (lib/exp/NAME.so),
# 3 interleaved repeats at 4096^2 F64.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04r; mkdir -p $O
for v in ${STAMPS:-stampB stampB2}; do
  echo "## $v"; QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/$v.so timeout -k 10 200 python tools/stamps/stamps_passB.py 4096 > $O/$v.txt 2>&1 || { tail -5 $O/$v.txt; exit 4; }
  cat $O/$v.txt
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in cur ${VARS:-B2}; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_$rep -o k -- python3 $R/bench.py --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_$rep.json 2> $R/$O/b_${v}_$rep.err || exit 5
    echo "== $v $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_$rep.json | head -1)"
    python3 $R/tools/kstats.py $R/$O/p_${v}_$rep/k_kernel_stats.csv | sed -n 2,5p
  done
done
