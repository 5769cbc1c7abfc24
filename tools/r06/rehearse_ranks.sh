#!/bin/bash
# the multi-GPU bench path at 4 and 8 ranks, every rank on the one GPU of the box (RCCL over
# loopback; a rehearsal of the launch, the probe group and the transports -- not a measurement)
cd $GRAFT_REPO_ROOT; O=gpurun_out/ranks; mkdir -p $O
B="--cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --mg-steps 0 --dropin-steps 0 --no-pmc-live --no-reference-runs"
for G in 4 8; do
  timeout -k 10 500 python bench.py --gpus $G --one-gpu --n 1024 --steps 20 --warmup 5 $B > $O/g$G.json 2> $O/g$G.err || { tail -20 $O/g$G.err; exit $G; }
  python - <<PY
import json
d = json.loads(open("$O/g$G.json").read()); c = d["config"]
print($G, "ranks:", round(d["value"], 1), "steps/s aggregate (all ranks on one GPU);", c["transport_probe"], "| halo", c["halo_transport"], "gather", c["gather_transport"], "| check:", c["transport_check"])
PY
done
