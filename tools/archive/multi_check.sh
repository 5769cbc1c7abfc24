#!/bin/bash
# multi-GPU path on one GPU: the launch rehearsal (2 and 4 ranks, host transport), the 1-rank
# RCCL ring at 4096^2 with and without --overlap, and the plain path, same call.
# usage: tools/multi_check.sh TAG
TAG=${1:-mc}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/bench_rehearsal.sh || exit 1
for v in plain commself overlap; do
  X=""; [ $v = commself ] && X="--comm-self"; [ $v = overlap ] && X="--comm-self --overlap"
  timeout -k 10 300 python bench.py --cpu-steps 0 --pcg-steps 0 --steps 50 --warmup 20 $X > gpurun_out/mc_${TAG}_$v.json 2> gpurun_out/mc_${TAG}_$v.err || exit 2
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/mc_${TAG}_$v.json | head -1)"
done
