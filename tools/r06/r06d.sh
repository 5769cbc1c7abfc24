#!/bin/bash
# r06d: the multi-GPU bench's peer-transport probe on one GPU (2 ranks over RCCL loopback):
# self-launched, under torch.distributed.run, and with a probe rank killed by SIGSEGV; each
# stdout must hold exactly the one JSON line (strict parse)
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/r06d
O=gpurun_out/r06d
A="--gpus 2 --one-gpu --steps 20 --warmup 5 --cpu-steps 0 --comm-probe-reps 5"
timeout -k 10 400 python bench.py $A > $O/self.json 2> $O/self.err || { tail -20 $O/self.err; exit 1; }
python -c "import json; d=json.loads(open('$O/self.json').read()); c=d['config']; print('self', d['value'], c['transport_probe'], c['transport_choice'], c['halo_transport'], c['gather_transport'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py $A > $O/torchrun.json 2> $O/torchrun.err || { tail -20 $O/torchrun.err; exit 2; }
python -c "import json; d=json.loads(open('$O/torchrun.json').read()); c=d['config']; print('torchrun', d['value'], c['transport_probe'], c['transport_choice'], c['halo_transport'], c['gather_transport'])"
QG_BENCH_PROBE_KILL=1 timeout -k 10 400 python bench.py $A > $O/killed.json 2> $O/killed.err || { tail -20 $O/killed.err; exit 3; }
python -c "import json; d=json.loads(open('$O/killed.json').read()); c=d['config']; print('killed', d['value'], c['transport_probe'], c['transport_choice'], c['halo_transport'], c['gather_transport'])"
