# tendency launch geometry: QG_TEND_WAVES chip-fulls of strips (default 2 above ~3500^2).
# usage: tools/tend_waves.sh
cd $GRAFT_REPO_ROOT
for n in ${QG_WAVE_SIZES:-4096 8192}; do
  for w in 1 2 3 4; do
    QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n $n --warmup 20 --steps $([ $n = 8192 ] && echo 30 || echo 100) --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print($n, 'waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done
