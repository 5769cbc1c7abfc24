# multi-rank bench rehearsal on ONE GPU: the driver's torch.distributed.run launch of bench.py
# with N ranks, over the host transport (RCCL refuses several ranks on one device).
# usage: tools/bench_rehearsal.sh
cd $GRAFT_REPO_ROOT
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --transport host --grid 256 --steps 5 --warmup 3 > gpurun_out/rehearsal_$N.json 2> gpurun_out/rehearsal_$N.err || { tail -20 gpurun_out/rehearsal_$N.err; exit 1; }
  tail -1 gpurun_out/rehearsal_$N.json | cut -c1-400
done
