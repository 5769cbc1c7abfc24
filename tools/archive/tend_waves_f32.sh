cd $GRAFT_REPO_ROOT
for w in 1 2 3 4; do
  QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n 8192 --dtype f32 --steps 30 --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print('f32 8192 waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
done
timeout -k 10 200 python bench.py --n 8192 --steps 30 --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print('f64 8192 default', round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
