#!/bin/bash
# round 4 (v): peer transports after the fail-fast fix -- tests (ring, rank processes, silent
# peer in both transports), 1-rank-ring bench A/B in one process (transport_ab), 4 ranks on
# the one GPU with the peer transports.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04v
mkdir -p $O
export QG_COMM_TIMEOUT=20
export QG_VERIFY_PUT=1
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_rccl_ring.py "tests/test_gpu_rccl_multirank.py::test_peer_transports_across_processes_bit_identical" \
  "tests/test_gpu_rccl_multirank.py::test_rccl_silent_peer_returns_rccl_error" > $O/tests.log 2>&1
rc=$?; tail -22 $O/tests.log | grep -E "PASS|FAIL|passed|failed|Error"
[ $rc -ne 0 ] && exit $rc
show() { python3 -c "
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r['config']; ab=r.get('transport_ab',{}); ov=r.get('overlap_ab',{})
print(sys.argv[1], c.get('halo_transport'), c.get('gather_transport'), round(r['value'],1), '| ab', ab.get('halo_transport'), ab.get('gather_transport'), round(ab.get('value',0),1), ab.get('error',''), '| ov', ov.get('halo_overlap'), round(ov.get('value',0),1), '| halo_ms', round(r['comm'].get('halo_ms',0),4), 'gather_ms', round(r['comm'].get('allgather_ms',0),4))" $1; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --comm-self --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs_rccl_$k.json 2> $O/cs_rccl_$k.err || exit 3
  show $O/cs_rccl_$k.json
  timeout -k 10 300 python bench.py --comm-self --halo peer --gather peer --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs_peer_$k.json 2> $O/cs_peer_$k.err || exit 3
  show $O/cs_peer_$k.json
  timeout -k 10 300 python bench.py --comm-self --halo put --gather peer --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs_put_$k.json 2> $O/cs_put_$k.err || exit 3
  show $O/cs_put_$k.json
  timeout -k 10 300 python bench.py --comm-self --halo put --gather peer --no-overlap --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 --no-transport-ab > $O/cs_putno_$k.json 2> $O/cs_putno_$k.err || exit 3
  show $O/cs_putno_$k.json
done
timeout -k 10 300 python bench.py --gpus 4 --one-gpu --n 1024 --halo put --gather peer --steps 50 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/og4.json 2> $O/og4.err || exit 5
show $O/og4.json
timeout -k 10 300 python bench.py --gpus 2 --one-gpu --n 4096 --steps 30 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/og2_4096.json 2> $O/og2_4096.err || exit 6
show $O/og2_4096.json
