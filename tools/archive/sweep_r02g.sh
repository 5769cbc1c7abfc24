#!/bin/bash
# after the batched prologue: certifying tendency (PCG leg) and F32 pair-kernel chip-fulls
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 2 3 4 6 8; do
  QG_CERT_WAVES=$w timeout -k 10 120 python bench.py --solver pcg --pcg-steps 0 --cpu-steps 0 --warmup 10 --steps 100 > gpurun_out/cs.json 2>gpurun_out/cs.err || exit 3
  echo "cert waves $w: $(grep -o '"value": [0-9.]*' gpurun_out/cs.json | head -1) $(grep -o '"tendency_ms": [0-9.]*' gpurun_out/cs.json)"
done
for n in 4096 8192; do for w in 2 4 6 8; do
  st=200; [ $n -ge 8192 ] && st=40
  QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n $n --dtype f32 --steps $st --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print('f32', $n, 'waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
done; done
