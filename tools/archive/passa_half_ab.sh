#!/bin/bash
# wide-row pass A (M = 8192) A/B: F32 rows' r issued before the next row's loads (default) vs
# after them (lib/exp/pahlate.so); F32 parity tests, kernel stats at 8192^2 F32 twice and F64.
# usage: tools/passa_half_ab.sh TAG
set -o pipefail
TAG=${1:-pah}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_f32.py tests/test_gpu_configs.py -k "f32 or config5 or F32" > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a pahlate -- --n 8192 --dtype f32 --steps 20 --warmup 5 || exit 3
bash tools/prof_lib.sh ${TAG}b pahlate -- --n 8192 --dtype f32 --steps 20 --warmup 5 || exit 4
bash tools/prof_lib.sh ${TAG}d pahlate -- --n 8192 --steps 10 --warmup 3 || exit 5
