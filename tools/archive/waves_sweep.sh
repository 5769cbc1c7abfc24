#!/bin/bash
# tendency chip-full sweep: tools/waves_sweep.sh "N:w1,w2,..;N:..." [reps]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
REPS=${2:-2}
IFS=';' read -ra CASES <<< "$1"
for rep in $(seq $REPS); do for c in "${CASES[@]}"; do
  n=${c%%:*}; ws=${c#*:}
  for w in ${ws//,/ }; do
    st=200; [ $n -ge 8192 ] && st=40
    QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n $n --warmup 20 --steps $st --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 6
    python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print($n, 'waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done; done
