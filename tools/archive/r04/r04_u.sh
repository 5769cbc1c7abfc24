#!/bin/bash
# round 4 (u): the peer-copy halo transport -- bitwise tests (one-rank ring, rank processes on
# the one GPU, silent peer), same-process A/B of the 1-rank ring bench (rccl vs peer halo,
# overlap on), and a kernel + memory-copy trace of the peer schedule.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04u
mkdir -p $O
export QG_COMM_TIMEOUT=20
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_rccl_ring.py "tests/test_gpu_rccl_multirank.py::test_peer_transports_across_processes_bit_identical" \
  "tests/test_gpu_rccl_multirank.py::test_rccl_silent_peer_returns_rccl_error" > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log
for k in 1 2; do
  for h in rccl peer; do
    timeout -k 10 300 python bench.py --comm-self --halo $h --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs_${h}_$k.json 2> $O/cs_${h}_$k.err || exit 3
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], r['config'].get('halo_transport'), 'overlap', r['config']['halo_overlap'], round(r['value'],1), 'ab', r['overlap_ab'].get('halo_overlap'), round(r['overlap_ab'].get('value',0),1), 'halo_ms', round(r['comm']['halo_ms'],4))" $O/cs_${h}_$k.json
  done
done
for g in rccl peer; do
  timeout -k 10 300 python bench.py --gpus 4 --one-gpu --n 1024 --halo $g --gather $g --steps 50 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/og4_$g.json 2> $O/og4_$g.err || exit 5
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], r['config'].get('halo_transport'), r['config'].get('gather_transport'), round(r['value'],1), round(r['ms_per_step'],3), 'comm', r.get('comm'))" $O/og4_$g.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/trace -o pe -- python3 $R/bench.py --comm-self --halo peer --steps 30 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 --comm-probe-reps 0 > $R/$O/trace.log 2>&1 || exit 4
ls $R/$O/trace
python3 $R/tools/timeline.py $R/$O/trace/pe_kernel_trace.csv spec_carry 3 $R/$O/trace/pe_memory_copy_trace.csv > $R/$O/timeline.txt
head -60 $R/$O/timeline.txt
exit $rc
