#!/bin/bash
# round 4 (s): tendency tile sweep at 4096^2 F64 (QG_TEND_TILE = WxR: strip width x rows per
# workgroup) against the default geometry, two interleaved repeats, kernel stats.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r04s; mkdir -p $O
for rep in 1 2; do
  for t in default ${TILES:-128x8 128x16 256x8 256x11 256x16 512x8 512x16 512x32}; do
    E=""; [ $t != default ] && E="QG_TEND_TILE=$t"
    env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${t}_$rep -o k -- python3 $R/bench.py --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b_${t}_$rep.json 2> $O/b_${t}_$rep.err || exit 5
    echo "== $t $rep $(python3 $R/tools/kstats.py $O/p_${t}_$rep/k_kernel_stats.csv | grep tendency | head -1)"
  done
done
