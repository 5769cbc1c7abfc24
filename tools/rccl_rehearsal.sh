#!/bin/bash
# multi-rank bench over REAL RCCL on one GPU (bench.py --one-gpu: every rank declares its own
# host to RCCL, the network transport over loopback carries the collectives), both launch modes
# the driver may use.  Exercises the exact --transport rccl code path of the scaling run (not
# xGMI: the numbers are not a measurement).  usage: tools/rccl_rehearsal.sh [GRID] [N...]
cd $GRAFT_REPO_ROOT
G=${1:-1024}; shift; NS=${@:-2 4 8}
O=gpurun_out/rccl_rehearsal; mkdir -p $O
for N in $NS; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --one-gpu --grid $G --steps 10 --warmup 3 > $O/run_${G}_$N.json 2> $O/run_${G}_$N.err || { tail -20 $O/run_${G}_$N.err; exit 1; }
  tail -1 $O/run_${G}_$N.json | cut -c1-400
  timeout -k 10 300 python bench.py --gpus $N --one-gpu --grid $G --steps 10 --warmup 3 > $O/plain_${G}_$N.json 2> $O/plain_${G}_$N.err || { tail -20 $O/plain_${G}_$N.err; exit 1; }
  tail -1 $O/plain_${G}_$N.json | cut -c1-400
done
