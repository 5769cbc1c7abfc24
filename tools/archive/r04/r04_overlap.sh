#!/bin/bash
# round 4: overlap A/B on the 1-rank RCCL ring (3 repeats each order), a kernel trace of the
# overlap schedule, and the targeted parity tests of this round's changes.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out/r04a
O=gpurun_out/r04a
export QG_OCC_VERBOSE=1
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_rccl_ring.py tests/test_gpu_pcg.py "tests/test_gpu_multirank.py::test_failed_certificate_stops_every_rank_at_the_same_step" \
  tests/test_gpu_multirank.py::test_overlap_is_bit_identical tests/test_gpu_dropin.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  for ov in "" "--overlap"; do
    timeout -k 10 300 python bench.py --comm-self $ov --steps 200 --warmup 20 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 > $O/cs${ov}_$k.json 2> $O/cs${ov}_$k.err || exit 3
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], 'overlap', r['config']['halo_overlap'], round(r['value'],1), 'ab', r['overlap_ab'].get('halo_overlap'), round(r['overlap_ab'].get('value',0),1), 'halo_ms', round(r['comm']['halo_ms'],4))" $O/cs${ov}_$k.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o ov -- python3 $R/bench.py --comm-self --overlap --steps 30 --warmup 10 --pcg-steps 0 --dropin-steps 0 --cpu-steps 0 --comm-probe-reps 0 > $R/$O/trace.log 2>&1 || exit 4
python3 $R/tools/timeline.py $R/$O/trace/ov_kernel_trace.csv spec_carry 3 > $R/$O/timeline.txt
head -30 $R/$O/timeline.txt
cd $R
timeout -k 10 300 python tools/cg_floor.py 256 > $O/cg_floor.txt 2>&1
cat $O/cg_floor.txt
