#!/bin/bash
# pass B set-up A/B (lib/exp/l2first.so: coefficient / closure loads first, then UIN / WIN):
# solver parity tests, kernel stats at 4096^2 twice and 2048^2.  usage: tools/passb_setup_ab.sh TAG
set -o pipefail
TAG=${1:-pbs}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pcg.py tests/test_gpu_f32.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
QGMI355_LIB=$GRAFT_REPO_ROOT/julia-ocean-modelling_amd/lib/exp/l2first.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py > gpurun_out/t2_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t2_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a l2first || exit 3
bash tools/prof_lib.sh ${TAG}b l2first || exit 4
bash tools/prof_lib.sh ${TAG}2k l2first -- --n 2048 --steps 100 || exit 5
