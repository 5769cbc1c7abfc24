# A/B of solver-pass variants (lib/variants/*.so), twice each, at 4096^2 and 1024^2 F64
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_edge.py > gpurun_out/t_pb.log 2>&1; rc=$?; tail -1 gpurun_out/t_pb.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
bash tools/prof_variants.sh b4k$r --warmup 20 || exit 3
bash tools/prof_variants.sh b1k$r --n 1024 --warmup 20 --steps 200 || exit 4
done
exit 0
