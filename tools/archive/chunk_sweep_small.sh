# chunk-size sweep at small grids (latency-bound passes): bench.py --chunk-rows L per size.
# usage: tools/chunk_sweep_small.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/csweep
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --cpu-steps 0 --pcg-steps 0 --dropin-steps 0 --warmup 20 "$@" > gpurun_out/csweep/bench_$tag.json 2> gpurun_out/csweep/bench_$tag.err || return 1
  python -c "import json; d=json.loads(open('gpurun_out/csweep/bench_$tag.json').read().strip().splitlines()[-1]); r=d['step_roofline']; print('$tag', round(d['value'],1), round(d['ms_per_step']*1e3,1), round(r['tendency_ms']*1e3,1), round(r['solve_ms']*1e3,1))"
}
for n in 256 512 1024 2048; do
  for L in 0 8 4 2 1; do run n${n}_L$L --n $n --steps 1000 --chunk-rows $L || exit 1; done
done
