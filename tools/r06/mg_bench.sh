#!/bin/bash
# the bench headline path with the multigrid-preconditioned PCG: one GPU, and 2 ranks on the one GPU
cd $GRAFT_REPO_ROOT; O=gpurun_out/mgbench; mkdir -p $O
B="--cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --mg-steps 0 --dropin-steps 0 --no-pmc-live --no-reference-runs"
timeout -k 10 300 python bench.py --solver pcg --precond mg --steps 10 --warmup 3 $B > $O/one.json 2> $O/one.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --one-gpu --solver pcg --precond mg --steps 10 --warmup 3 $B > $O/two.json 2> $O/two.err || exit 2
python - <<PY
import json
for f in ("one", "two"):
    d = json.load(open("$O/%s.json" % f))
    print(f, d["value"], d["ms_per_step"], d["config"]["solver"], d["config"].get("parallelism"), d.get("roofline", {}).get("frac"))
PY
