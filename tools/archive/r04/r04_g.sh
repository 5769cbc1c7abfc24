#!/bin/bash
# round 4 (g): pass B with its recurrence coefficients in LDS (lib/exp/ctab.so: in-place
# inverse transform at 4096) vs current, 3 alternating repeats at 4096^2 F64 (kernel stats +
# driver-flag bench); the tests touched since (f).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -s tests/test_gpu_pcg.py tests/test_gpu_rccl_ring.py "tests/test_gpu_multirank.py::test_overlap_is_bit_identical" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep "plain CG" $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for k in 1 2 3; do
  for v in ctab cur; do
    L=""; [ $v != cur ] && L=$R/julia-ocean-modelling_amd/lib/exp/$v.so
    QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_$k -o k -- python3 $R/bench.py --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/b_${v}_$k.json 2> $R/$O/b_${v}_$k.err || exit 5
    python3 $R/tools/kstats.py $R/$O/p_${v}_$k/k_kernel_stats.csv > $R/$O/k_${v}_$k.txt
    QGMI355_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/$O/d_${v}_$k.json 2> $R/$O/d_${v}_$k.err || exit 6
    echo "== $v $k prof $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_$k.json | head -1) drv $(grep -o '"value": [0-9.]*' $R/$O/d_${v}_$k.json | head -1) $(grep passB $R/$O/k_${v}_$k.txt)"
  done
done
cd $R
QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/ctab.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py > $O/tests_ctab.log 2>&1; echo "ctab parity rc $?"; tail -2 $O/tests_ctab.log
