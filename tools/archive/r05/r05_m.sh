#!/bin/bash
# round 5 (m): final evidence on the final tree -- full GPU suite, smoke, the driver's bench
# command (live PMC traffic), its rocprofv3 kernel stats, a 2-rank RCCL rehearsal on one GPU
# (peer transports + their bitwise check in a real multi-process run), config 5 three times.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -10 $O/bench_driver.err; exit 6; }
python3 -c "
import json; d=json.loads(open('$O/bench_driver.json').read().strip().splitlines()[-1]); r=d['roofline']
print('driver bench', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'frac', round(r['frac'],3), 'avg_launch_ms', round(r['avg_launch_ms'],4), 'traffic', r['traffic'], '|', r['traffic_source'])
print('dropin', round(d['dropin']['ms_per_step']/d['ms_per_step'],3), 'slot1', round(d['dropin_slot1']['ms_per_step']/d['ms_per_step'],3))"
timeout -k 10 400 python bench.py --gpus 2 --one-gpu --steps 20 --warmup 5 > $O/bench_2rank_onegpu.json 2> $O/bench_2rank_onegpu.err || { tail -10 $O/bench_2rank_onegpu.err; exit 7; }
python3 -c "
import json; d=json.loads(open('$O/bench_2rank_onegpu.json').read().strip().splitlines()[-1]); c=d['config']
print('2-rank one-GPU rehearsal', round(d['value'],1), c['transport_choice'], '|', c.get('transport_check'), '| ab', d.get('transport_ab',{}).get('value'))"
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --n 8192 --dtype f32 --steps 20 --warmup 5 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $O/b8k_$rep.json 2> $O/b8k_$rep.err || exit 8
  echo "== 8192 f32 $rep $(grep -o '"value": [0-9.]*' $O/b8k_$rep.json | head -1)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc-live > $R/$O/prof_bench.json 2> $R/$O/prof_bench.err || exit 9
python3 $R/tools/kstats.py $R/$O/prof/drv_kernel_stats.csv
