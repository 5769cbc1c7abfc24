#!/bin/bash
# r06c: solve precision on the weak-scaling grids, F32 decomposition, new config tests, pass-B A/B
R=$GRAFT_REPO_ROOT; cd $R || exit 1; mkdir -p gpurun_out/r06c
O=gpurun_out/r06c
timeout -k 10 400 python -u tools/r06/solve_precision.py --device 4096:8192 4096:16384 4096:32768 > $O/solve_precision.txt 2>&1 || exit 1
cat $O/solve_precision.txt
timeout -k 10 300 python -u tools/r06/f32_decompose.py 8192 8192 10 16 > $O/f32_8192_10.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/r06/f32_decompose.py 8192 8192 3 16 > $O/f32_8192_3.txt 2>&1 || exit 2
timeout -k 10 400 python -u tools/r06/f32_decompose.py 8192 65536 3 8 > $O/f32_65536_3.txt 2>&1 || exit 2
tail -n 20 $O/f32_*.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -k "weak_scaling or longdouble or g8" -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 3; }
grep -E "vs C oracle|long double|slabs vs|passed|failed" $O/configs.log
tools/prof_lib.sh r06c pbcoef > $O/ab_pbcoef.txt 2>&1 || exit 4
cat $O/ab_pbcoef.txt
