#!/bin/bash
# multigrid PCG after the host-transport copy fix: convergence curves over 8 steps (slabs),
# then the multigrid tests and the in-process slab tests
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/r06/mg_probe2.py 256 1,4,8 8 20 > gpurun_out/mg_probe6.txt 2>&1 || exit 1
timeout -k 10 300 python tools/r06/mg_probe2.py 512 4 8 20 >> gpurun_out/mg_probe6.txt 2>&1 || exit 1
tools/r06/gtest.sh mg4 tests/test_gpu_mg.py tests/test_gpu_configs.py -s
