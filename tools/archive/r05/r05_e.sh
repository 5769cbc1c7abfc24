#!/bin/bash
# round 5 (e): Bluestein rows (odd M > 8192, M > 16384) against the oracle; the comm tests
# after the region_create / comm_barrier rewrite; the 1-rank ring without gather / pin.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_gpu_edge.py" tests/test_gpu_rccl_ring.py tests/test_gpu_comm_failure.py tests/test_gpu_rccl_multirank.py tests/test_gpu_multirank.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "bluestein or generic_rows_wide or two_row or small_and_ragged or rccl or peer or ring or slab or silent or failure" > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|residuals" $O/tests.log | tail -60; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in plain self; do
  A=""; [ $v = self ] && A="--comm-self --no-transport-ab --comm-probe-reps 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o $v -- python3 $R/bench.py --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 $A > $R/$O/pb_$v.json 2> $R/$O/pb_$v.err || exit 6
  python3 $R/tools/kstats.py $R/$O/prof_$v/${v}_kernel_stats.csv
  python3 $R/tools/timeline.py $R/$O/prof_$v/${v}_kernel_trace.csv tendency 2 > $R/$O/timeline_$v.txt
  cat $R/$O/timeline_$v.txt
done
cd $R
for rep in 1 2 3; do
  for v in plain self; do
    A=""; [ $v = self ] && A="--comm-self --no-transport-ab --comm-probe-reps 0"
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 $A > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 7
    echo "== $v $rep $(grep -o '"value": [0-9.]*' $O/b_${v}_$rep.json | head -1)"
  done
done
