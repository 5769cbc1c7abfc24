#!/bin/bash
# run selected GPU test files: tools/r06/gtest.sh TAG file-or-nodeid...
TAG=$1; shift
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/t_$TAG.log | tail -3
exit $rc
