#!/bin/bash
# round 4 (d): whole GPU suite (F32 transforms in the wide-row solver, CG stagnation rule);
# kernel stats 8192^2 F32 / 4096^2 F64; overlap A/B x3 + trace; plain-CG floor; PMC at 8192^2 F32.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
grep -E "config 5|F32|plain CG|vs C oracle" $O/tests.log | head -20
timeout -k 10 300 python tools/cg_floor.py 256 > $O/cg_floor.txt 2>&1; cat $O/cg_floor.txt
summ() { python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], 'overlap', r['config']['halo_overlap'], round(r['value'],1), 'ab', r['overlap_ab'].get('halo_overlap'), round(r['overlap_ab'].get('value',0),1), 'halo_ms', round(r['comm']['halo_ms'],4))" $1; }
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --comm-self --overlap --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/ov_$k.json 2> $O/ov_$k.err || { tail -5 $O/ov_$k.err; exit 3; }
  summ $O/ov_$k.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o ov -- python3 $R/bench.py --comm-self --overlap --steps 30 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 --comm-probe-reps 0 > $R/$O/trace.log 2>&1 || exit 4
python3 $R/tools/timeline.py $R/$O/trace/ov_kernel_trace.csv spec_carry 3 > $R/$O/timeline.txt
head -12 $R/$O/timeline.txt
for n in 8192f32 4096f64; do
  N=${n:0:4}; D=${n:4:3}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_$n -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_$n.json 2> $R/$O/b_$n.err || exit 5
  echo "== $n $(grep -o '"value": [0-9.]*' $R/$O/b_$n.json | head -1)"
  python3 $R/tools/kstats.py $R/$O/p_$n/k_kernel_stats.csv > $R/$O/k_$n.txt; head -6 $R/$O/k_$n.txt
done
cd $R
bash tools/pmc.sh r04d8 --n 8192 --dtype f32 --dropin-steps 0 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 6; }
python3 tools/pmc_summary.py r04d8 > $O/pmc_summary.txt; cat $O/pmc_summary.txt | head -60
