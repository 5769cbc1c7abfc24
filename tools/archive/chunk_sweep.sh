# spectral-solver chunk rows at small grids.  usage: tools/chunk_sweep.sh
cd $GRAFT_REPO_ROOT
for n in 512 1024 2048; do
  for L in 2 4 8 16; do
    timeout -k 10 200 python bench.py --n $n --chunk-rows $L --steps 1000 --cpu-steps 0 --pcg-steps 0 > gpurun_out/cs.json 2>gpurun_out/cs.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/cs.json').read().strip().splitlines()[-1]); r=d['step_roofline']; print($n, 'L', $L, round(d['value'],1), 'tend', round(r['tendency_ms']*1e3,1), 'solve', round(r['solve_ms']*1e3,1))"
  done
done
