#!/bin/bash
# chunk rows L of the direct solver's passes (pick_chunk) swept per grid: solve time by events
# usage: tools/r06/chunk_sweep.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/chunk
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 200 python bench.py --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live --warmup 20 --clock-warm-ms 500 "$@" > gpurun_out/chunk/b_$tag.json 2> gpurun_out/chunk/b_$tag.err || { echo "$tag failed"; return 0; }
  python -c "import json; d=json.loads(open('gpurun_out/chunk/b_$tag.json').read()); r=d['step_roofline']; print('$tag', round(d['value'],1), 'step', round(d['ms_per_step']*1e3,1), 'tend', round(r['tendency_ms']*1e3,1), 'solve', round(r['solve_ms']*1e3,1))"
}
for rep in 1 2; do
for L in 0 1 2 4 8; do run n512_L${L}_$rep --n 512 --steps 2000 --chunk-rows $L; done
for L in 0 1 2 4 8; do run n1024_L${L}_$rep --n 1024 --steps 2000 --chunk-rows $L; done
for L in 0 2 4 8 16; do run n2048_L${L}_$rep --n 2048 --steps 1000 --chunk-rows $L; done
for L in 0 8 16 32; do run n4096_L${L}_$rep --n 4096 --steps 200 --chunk-rows $L; done
for L in 0 16 32 64; do run f32n8192_L${L}_$rep --n 8192 --dtype f32 --steps 50 --chunk-rows $L; done
done
