#!/bin/bash
# carry kernel: UIN re-read in the forward pass (lib/exp/uinreload.so, no spill) vs held in
# registers (default); solver parity with the variant, kernel stats at 4096^2 twice and 1024^2.
set -o pipefail
TAG=${1:-cr}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
QGMI355_LIB=$GRAFT_REPO_ROOT/julia-ocean-modelling_amd/lib/exp/uinreload.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pcg.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a uinreload || exit 3
bash tools/prof_lib.sh ${TAG}b uinreload || exit 4
bash tools/prof_lib.sh ${TAG}1k uinreload -- --n 1024 --steps 200 || exit 5
