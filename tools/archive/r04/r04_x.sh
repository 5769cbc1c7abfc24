#!/bin/bash
# round 4 (x): the bench's transport_ab leg in the launch modes the driver may use (self-launched
# ranks on one GPU, 2 ranks), and the 1-rank ring at config 5's size (8192^2 F32).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04x
mkdir -p $O
show() { python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r['config']
print(sys.argv[1], c.get('halo_transport'), c.get('gather_transport'), c.get('halo_overlap'), round(r['value'],1), round(r['ms_per_step'],4))
print('  overlap_ab', {k: v for k, v in r.get('overlap_ab', {}).items() if k != 'note'})
print('  transport_ab', {k: v for k, v in r.get('transport_ab', {}).items() if k != 'note'})
print('  comm', r.get('comm'))" $1; }
timeout -k 10 300 python bench.py --gpus 2 --one-gpu --n 1024 --steps 50 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/og2.json 2> $O/og2.err || exit 3
show $O/og2.json
timeout -k 10 300 python bench.py --comm-self --n 8192 --dtype f32 --steps 50 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs8k.json 2> $O/cs8k.err || exit 4
show $O/cs8k.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || exit 5
show $O/drv.json
