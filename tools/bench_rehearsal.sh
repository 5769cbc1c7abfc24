# multi-rank bench rehearsal on ONE GPU over the host transport (RCCL refuses several ranks
# on one device), in both launch modes the driver may use: torch.distributed.run, and a plain
# `python bench.py --gpus N` (bench.py then starts the rank processes itself).
# usage: tools/bench_rehearsal.sh
cd $GRAFT_REPO_ROOT
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --transport host --grid 256 --steps 5 --warmup 3 > gpurun_out/rehearsal_$N.json 2> gpurun_out/rehearsal_$N.err || { tail -20 gpurun_out/rehearsal_$N.err; exit 1; }
  tail -1 gpurun_out/rehearsal_$N.json | cut -c1-300
  timeout -k 10 300 python bench.py --gpus $N --transport host --grid 256 --steps 5 --warmup 3 > gpurun_out/rehearsal_plain_$N.json 2> gpurun_out/rehearsal_plain_$N.err || { tail -20 gpurun_out/rehearsal_plain_$N.err; exit 1; }
  tail -1 gpurun_out/rehearsal_plain_$N.json | cut -c1-300
done
