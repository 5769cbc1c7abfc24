#!/bin/bash
# one GPU round: parity tests, bench (driver flags and defaults), rocprof kernel stats.
# usage: tools/gpu_check.sh TAG [extra bench args]
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --warmup 5 --steps 20 "$@" > gpurun_out/bench_${TAG}_drv.json 2> gpurun_out/bench_${TAG}_drv.err || exit 3
cat gpurun_out/bench_${TAG}_drv.json
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 3
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o $TAG -- python3 $R/bench.py --steps 50 --warmup 20 --cpu-steps 0 --pcg-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 4
cut -d, -f1-4 $R/gpurun_out/prof_$TAG/${TAG}_kernel_stats.csv | head -8
