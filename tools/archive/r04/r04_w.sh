#!/bin/bash
# round 4 (w): end-of-round evidence on this tree (tools/round_evidence.sh), then the 1-rank
# ring bench with the transport A/B leg as the bench now records it.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
bash tools/round_evidence.sh r04w || exit $?
O=gpurun_out/r04w_cs
mkdir -p $O
timeout -k 10 300 python bench.py --comm-self --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs.json 2> $O/cs.err || exit 7
python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r['config']
print('headline', c['halo_transport'], c['gather_transport'], c['halo_overlap'], round(r['value'],1))
print('overlap_ab', r['overlap_ab']); print('transport_ab', r['transport_ab'])" $O/cs.json
