#!/bin/bash
# pass A A/B (lib/exp/coefrow.so: coefficients reloaded per row): solver parity tests, kernel
# stats at 4096^2 (twice) and 2048^2.  usage: tools/passa_ab.sh TAG
set -o pipefail
TAG=${1:-paab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pcg.py tests/test_gpu_f32.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a coefrow || exit 3
bash tools/prof_lib.sh ${TAG}b coefrow || exit 4
bash tools/prof_lib.sh ${TAG}2k coefrow -- --n 2048 --steps 100 || exit 5
