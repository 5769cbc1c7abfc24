#!/bin/bash
# fused multigrid passes: tests (one GPU, in-process slabs, RCCL slabs incl. config 4), then the bench leg
cd $GRAFT_REPO_ROOT
tools/r06/gtest.sh mg5 tests/test_gpu_mg.py tests/test_gpu_rccl_multirank.py -k "mg or MG or kw or config_slabs" -s || exit 1
timeout -k 10 300 python tools/r06/mg_probe2.py 256 1,4 3 8,10,12 > gpurun_out/mg_probe7.txt 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pmc-live --no-reference-runs --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --mg-steps 10 > gpurun_out/mg5_bench.json 2> gpurun_out/mg5_bench.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/mg5_bench.json')); print(d['value'], json.dumps(d['mg_pcg_solver']))"
