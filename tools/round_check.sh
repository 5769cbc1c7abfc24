#!/bin/bash
# end-of-round evidence in one call: GPU tests, bench (driver flags and defaults), rocprof
# kernel stats (tools/gpu_check.sh), PMC passes (tools/pmc.sh), grid-size sweep (tools/sweep.sh).
# usage: tools/round_check.sh TAG
TAG=${1:-rc}
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh $TAG || exit $?
bash tools/pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || exit 5
bash tools/sweep.sh > gpurun_out/sweep_$TAG.txt 2>&1 || exit 6
cat gpurun_out/sweep_$TAG.txt
