#!/bin/bash
# round 4 (c): overlap with the interior rows on a CU-masked stream (variants of the excluded
# CUs), its trace; tendency peel A/B (interior strips straight-line) at 8192^2 F32 / 4096^2
# F64; the whole GPU suite.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04c; mkdir -p $O
export QG_OCC_VERBOSE=1
summ() { python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], 'overlap', r['config']['halo_overlap'], round(r['value'],1), 'ab', r['overlap_ab'].get('halo_overlap'), round(r['overlap_ab'].get('value',0),1), 'halo_ms', round(r['comm']['halo_ms'],4))" $1; }
for k in 1 2; do
  for v in xcd1 lo8 xcd2 none; do
    case $v in
      xcd1) export QG_OV_CUS="0,32,64,96,128,160,192,224";;
      lo8) export QG_OV_CUS="0,1,2,3,4,5,6,7";;
      xcd2) export QG_OV_CUS="0,32,64,96,128,160,192,224,1,33,65,97,129,161,193,225";;
      none) export QG_OV_CUS="-1";;
    esac
    timeout -k 10 300 python bench.py --comm-self --overlap --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/ov_${v}_$k.json 2> $O/ov_${v}_$k.err || { tail -5 $O/ov_${v}_$k.err; exit 3; }
    summ $O/ov_${v}_$k.json
  done
done
grep -h "overlap:" $O/ov_*_1.err | sort | uniq
unset QG_OV_CUS QG_OCC_VERBOSE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o ov -- python3 $R/bench.py --comm-self --overlap --steps 30 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 --comm-probe-reps 0 > $R/$O/trace.log 2>&1 || exit 4
python3 $R/tools/timeline.py $R/$O/trace/ov_kernel_trace.csv spec_carry 3 > $R/$O/timeline.txt
head -24 $R/$O/timeline.txt
for v in nopeel coefearly cur; do
  L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
  for n in 8192f32 4096f64; do
    N=${n:0:4}; D=${n:4:3}
    QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_$n -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_$n.json 2> $R/$O/b_${v}_$n.err || exit 5
    echo "== $v $n $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_$n.json | head -1)"
    python3 $R/tools/kstats.py $R/$O/p_${v}_$n/k_kernel_stats.csv > $R/$O/k_${v}_$n.txt; head -6 $R/$O/k_${v}_$n.txt
  done
done
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/cg_floor.py 256 > $O/cg_floor.txt 2>&1
cat $O/cg_floor.txt
