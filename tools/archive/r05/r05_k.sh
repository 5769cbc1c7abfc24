#!/bin/bash
# round 5 (k): the tree after the pass changes -- full GPU suite, smoke, the driver's bench command
# (with the live PMC traffic passes), the 1-rank-ring bench (peer transports + their check against
# RCCL), config 5, carry phase stamps, and a same-box A/B of the final passes against tw1.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 5; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -10 $O/bench_driver.err; exit 6; }
python3 -c "
import json; d=json.loads(open('$O/bench_driver.json').read().strip().splitlines()[-1]); r=d['roofline']
print('driver bench', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), 'traffic', r['traffic'], '|', r['traffic_source'])
print('dropin', d.get('dropin',{}).get('ratio_to_qg_run'), 'slot1', d.get('dropin_slot1',{}).get('ratio_to_qg_run'))"
timeout -k 10 300 python bench.py --comm-self --steps 50 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $O/bench_commself.json 2> $O/bench_commself.err || { tail -10 $O/bench_commself.err; exit 7; }
python3 -c "
import json; d=json.loads(open('$O/bench_commself.json').read().strip().splitlines()[-1]); c=d['config']
print('comm-self', round(d['value'],1), c['transport_choice'], '|', c.get('transport_check'))"
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampC.so timeout -k 10 200 python tools/stamps/stamps_carry.py 4096 f64 > $O/stampsC_4096.txt 2>&1 || { tail -5 $O/stampsC_4096.txt; exit 8; }
cat $O/stampsC_4096.txt
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampC.so timeout -k 10 200 python tools/stamps/stamps_carry.py 8192 f32 > $O/stampsC_8192.txt 2>&1 || { tail -5 $O/stampsC_8192.txt; exit 8; }
cat $O/stampsC_8192.txt
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in tw1 fin; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so; [ $v = fin ] && L=$R/julia-ocean-modelling_amd/lib/libqgmi355.so
    for C in "8192 f32" "4096 f64"; do
      set -- $C; N=$1; D=$2
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${N}_$rep -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $R/$O/b_${v}_${N}_$rep.json 2> $R/$O/b_${v}_${N}_$rep.err || exit 9
      echo "== $v $N $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${N}_$rep.json | head -1) | $(python3 $R/tools/kstats.py $R/$O/p_${v}_${N}_$rep/k_kernel_stats.csv | grep -E 'pass|carry|tendency' | awk '{printf "%s %s; ", $1, $5}')"
    done
  done
done
