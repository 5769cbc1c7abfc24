#!/bin/bash
# pass A / B set-up A/B: full GPU tests, then kernel stats of the default library,
# lib/exp/serialcarry.so (pass B's per-line carry set-up) and lib/exp/head.so (the previous
# commit), twice.  usage: tools/solve_ab.sh TAG
set -o pipefail
TAG=${1:-sab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a serialcarry head || exit 3
bash tools/prof_lib.sh ${TAG}b head serialcarry || exit 4
bash tools/prof_lib.sh ${TAG}1k serialcarry head -- --n 1024 --steps 200 || exit 5
