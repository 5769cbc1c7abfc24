# grid-size sweep on one GPU: bench.py per size, JSON lines under gpurun_out/sweep/.
# usage: tools/sweep.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live --warmup 20 "$@" > gpurun_out/sweep/bench_$tag.json 2> gpurun_out/sweep/bench_$tag.err || return 1
  python -c "import json; d=json.loads(open('gpurun_out/sweep/bench_$tag.json').read().strip().splitlines()[-1]); r=d['step_roofline']; print('$tag', round(d['value'],1), round(d['ms_per_step']*1e3,1), round(r['tendency_ms']*1e3,1), round(r['solve_ms']*1e3,1), round(r['frac']*100,1))"
}
for n in 128 256 512 1024 2048; do run n$n --n $n --steps 2000 || exit 1; done
run n4096 --n 4096 --steps 200 || exit 1
run n8192 --n 8192 --steps 50 || exit 1
run f32_n4096 --n 4096 --steps 200 --dtype f32 || exit 1
run f32_n8192 --n 8192 --steps 50 --dtype f32 || exit 1
run pcg_n1024 --n 1024 --steps 1000 --solver pcg || exit 1
run pcg_n4096 --n 4096 --steps 100 --solver pcg || exit 1
