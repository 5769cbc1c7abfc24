#!/bin/bash
# round 5 (d): the full GPU suite on this tree; the bench with its drop-in legs; the 1-rank
# ring (--comm-self, default = automatic transports) against the plain path, 3 interleaved
# repeats (verdict r04 item 2: >= 0.98x).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-steps 0 --cpu-steps-1t 0 > $O/b_default.json 2> $O/b_default.err || exit 5
python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('default', round(r['value'],1), 'dropin', r['dropin'].get('vs_qg_run_step'), 'slot1', r['dropin_slot1'].get('vs_qg_run_step'))" $O/b_default.json
for rep in 1 2 3; do
  for v in plain self; do
    A=""; [ $v = self ] && A="--comm-self --no-transport-ab --comm-probe-reps 0"
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 $A > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 6
    echo "== $v $rep $(grep -o '"value": [0-9.]*' $O/b_${v}_$rep.json | head -1) $(grep -o '"transport_choice": "[^"]*"' $O/b_${v}_$rep.json) $(grep -o '"halo_overlap": [a-z]*' $O/b_${v}_$rep.json | head -1)"
  done
done
