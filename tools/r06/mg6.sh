#!/bin/bash
# earlier agglomeration of the slab multigrid levels: slab tests (in-process and RCCL), then the 2-rank bench
cd $GRAFT_REPO_ROOT
tools/r06/gtest.sh mg6 tests/test_gpu_mg.py tests/test_gpu_rccl_multirank.py -k "slabs or kw" -s || exit 1
timeout -k 10 300 python tools/r06/mg_probe2.py 256 1,2,4,8 2 10 > gpurun_out/mg_probe8.txt 2>&1 || exit 2
bash tools/r06/mg_bench.sh
