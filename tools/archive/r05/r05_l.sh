#!/bin/bash
# round 5 (l): the carry kernel -- packed grid (the real line k = M/2 in the k = 0 lane: 512
# workgroups at M = 8192, one round), the extra column folded into k-block 0, the singular
# line's scans in registers, unrolled segment combines.  Parity (incl. multi-rank), carry phase
# stamps, then a same-box A/B against fin (HEAD), three interleaved repeats.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05l; mkdir -p $O
for C in "1024 f64" "4096 f64" "8192 f32" "8192 f64"; do
  set -- $C
  for v in fin cp; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so; [ $v = cp ] && L=$R/julia-ocean-modelling_amd/lib/libqgmi355.so
    echo "$v $(QGMI355_LIB=$L timeout -k 10 200 python tools/r05/state_digest.py $1 $2 5 2>/dev/null | tail -1)"
  done
done
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_f32.py tests/test_gpu_multirank.py tests/test_gpu_rccl_multirank.py tests/test_gpu_pcg.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 4; }
tail -1 $O/tests.log
for C in "4096 f64" "8192 f32"; do
  set -- $C
  QGMI355_LIB=$R/julia-ocean-modelling_amd/lib/exp/stampC.so timeout -k 10 200 python tools/stamps/stamps_carry.py $1 $2 > $O/stampsC_$1.txt 2>&1 || { tail -5 $O/stampsC_$1.txt; exit 8; }
  cat $O/stampsC_$1.txt
done
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in fin cp; do
    L=$R/julia-ocean-modelling_amd/lib/exp/$v.so; [ $v = cp ] && L=$R/julia-ocean-modelling_amd/lib/libqgmi355.so
    for C in "8192 f32" "4096 f64"; do
      set -- $C; N=$1; D=$2
      QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_${v}_${N}_$rep -o k -- python3 $R/bench.py --n $N --dtype $D --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --no-pmc-live > $R/$O/b_${v}_${N}_$rep.json 2> $R/$O/b_${v}_${N}_$rep.err || exit 9
      echo "== $v $N $rep $(grep -o '"value": [0-9.]*' $R/$O/b_${v}_${N}_$rep.json | head -1) | $(python3 $R/tools/kstats.py $R/$O/p_${v}_${N}_$rep/k_kernel_stats.csv | grep -E 'pass|carry|tendency' | awk '{printf "%s %s; ", $1, $5}')"
    done
  done
done
