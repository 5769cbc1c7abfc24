cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do for w in 2 3; do
  QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n 4096 --warmup 20 --steps 200 --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print(4096, 'waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
done; done
