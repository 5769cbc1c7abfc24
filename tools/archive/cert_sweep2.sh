#!/bin/bash
# PCG leg after the batched prologue: certifying tendency strip width x chip-fulls
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for tx in 128 256; do for w in 3 4 6; do
  QG_CERT_TX=$tx QG_CERT_WAVES=$w timeout -k 10 120 python bench.py --solver pcg --pcg-steps 0 --cpu-steps 0 --warmup 10 --steps 100 > gpurun_out/cs2.json 2>gpurun_out/cs2.err || exit 3
  echo "tx $tx waves $w: $(grep -o '"value": [0-9.]*' gpurun_out/cs2.json | head -1) $(grep -o '"tendency_ms": [0-9.]*' gpurun_out/cs2.json)"
done; done; done
