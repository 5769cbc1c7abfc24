# A/B of tendency-kernel variants (lib/variants/*.so): bitwise tests, then kernel stats at
# 4096^2, 2048^2, 8192^2 F64
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_tendency_kernels.py tests/test_gpu_parity.py > gpurun_out/t_tend.log 2>&1; rc=$?; tail -3 gpurun_out/t_tend.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_variants.sh t4k --warmup 20 || exit 3
bash tools/prof_variants.sh t2k --n 2048 --warmup 20 --steps 100 || exit 4
bash tools/prof_variants.sh t8k --n 8192 --warmup 5 || exit 5
exit 0
