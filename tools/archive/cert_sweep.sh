#!/bin/bash
# PCG leg: the certifying tendency's strip width and chip-fulls (QG_CERT_TX, QG_CERT_WAVES)
cd $GRAFT_REPO_ROOT
for tx in 256 128; do for w in 1 2 3 4 6; do
  QG_CERT_VERBOSE=1 QG_CERT_TX=$tx QG_CERT_WAVES=$w timeout -k 10 120 python bench.py --solver pcg --pcg-steps 0 --cpu-steps 0 --warmup 10 --steps 40 > gpurun_out/cs_${tx}_$w.json 2>gpurun_out/cs_${tx}_$w.err || exit 3
  echo "tx $tx waves $w: $(grep -o '"value": [0-9.]*' gpurun_out/cs_${tx}_$w.json | head -1) $(grep -o '"tendency_ms": [0-9.]*' gpurun_out/cs_${tx}_$w.json) $(grep resident gpurun_out/cs_${tx}_$w.err)"
done; done
