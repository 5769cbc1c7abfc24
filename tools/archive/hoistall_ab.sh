#!/bin/bash
# pass A coefficient hoist below N = 2048 (lib/exp/hoistall.so) vs the default, kernel stats at
# 1024^2, 512^2, 256^2.  usage: tools/hoistall_ab.sh TAG
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1024 512 256; do bash tools/prof_lib.sh ${1:-ha}$n hoistall -- --n $n --steps 400 || exit 1; done
