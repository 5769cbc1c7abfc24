# A/B of the timed-region measurement on one box: qg_run (default) vs per-step events inside
# the timed loop (--events-in-timed) vs HIP-graph replay (--graph).  usage: tools/graph_vs_stream.sh
cd $GRAFT_REPO_ROOT
for n in 4096 1024; do
  for rep in 1 2; do
    for g in "" "--events-in-timed" "--graph"; do
      timeout -k 10 200 python bench.py --n $n --steps $([ $n = 4096 ] && echo 100 || echo 1000) --warmup 20 --cpu-steps 0 --pcg-steps 0 $g > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
      python -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print($n, '$g', round(d['value'],1), round(d['ms_per_step']*1e3,1), 'us/step; tend', round(d['roofline']['avg_launch_ms']*1e3,1))"
    done
  done
done
