#!/bin/bash
# round 5 (a): lane-exchange 4096-point transform in spec_passA/B<4096>: parity tests, then
# base (lib/exp/base.so = round-4 HEAD) vs current at 4096^2 F64, 2 interleaved repeats, and
# the kernel stats of both.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base cur; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    QGMI355_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 5
    echo "== $v $rep $(grep -o '"value": [0-9.]*' $O/b_${v}_$rep.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$rep.json | head -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base cur; do
  L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
  QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o $v -- python3 $R/bench.py --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --steps 30 --warmup 10 > $R/$O/pb_$v.json 2> $R/$O/pb_$v.err || exit 6
  python3 $R/tools/kstats.py $R/$O/prof_$v/${v}_kernel_stats.csv
done
