#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python tools/r05/f32_global_grid.py > $O/f32_global.txt 2>&1 || { tail -5 $O/f32_global.txt; exit 4; }
cat $O/f32_global.txt
