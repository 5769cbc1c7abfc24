cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/r06/mg_probe2.py 256 1,4 4 10,12,14,20 > gpurun_out/mg_probe4.txt 2>&1 || exit 1
timeout -k 10 300 python tools/r06/mg_probe.py 256 > gpurun_out/mg_probe5.txt 2>&1 || exit 2
tools/r06/gtest.sh mg3 tests/test_gpu_mg.py tests/test_gpu_pcg.py -s
