# A/B of the pass B pin-sum variants (lib/variants/*.so) at 4096^2, 1024^2, 8192^2 F64
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_edge.py > gpurun_out/t_pin.log 2>&1; rc=$?; tail -3 gpurun_out/t_pin.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_variants.sh pin4k --warmup 20 || exit 3
bash tools/prof_variants.sh pin1k --n 1024 --warmup 20 --steps 200 || exit 4
bash tools/prof_variants.sh pin8k --n 8192 --warmup 5 || exit 5
exit 0
