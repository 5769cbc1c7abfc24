#!/bin/bash
# the whole -m gpu suite as the driver runs it (one process), with per-test durations
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 1140 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25 > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -32 gpurun_out/tests_$TAG.log
exit $rc
