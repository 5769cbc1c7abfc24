#!/bin/bash
# round 4 (n): QG_KEEP_ORDER_SLOT1 (the lean drop-in mode): drop-in + multirank keep-order
# tests, then the bench's dropin / dropin_slot1 legs.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_multirank.py -k "keep_order or slot1 or reference_signatures" -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 2; }
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', round(r['value'],1), 'ms', round(r['ms_per_step'],4))
for k in ('dropin','dropin_slot1'): print(k, {x: r[k][x] for x in ('ms_per_step','vs_qg_run_step') if x in r[k]}, r[k].get('error'))"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur r16; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_$rep -o k -- python3 $R/bench.py --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_$rep.json 2> $R/$O/b_${v}_$rep.err || exit 5
    echo "== $v $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_$rep.json | head -1)"
    python3 $R/tools/kstats.py $R/$O/p_${v}_$rep/k_kernel_stats.csv | sed -n 2,5p
  done
done
