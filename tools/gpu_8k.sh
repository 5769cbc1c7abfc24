# wide-row (M = 8192) checks: parity tests, F64 / F32 benches, kernel stats.  usage: tools/gpu_8k.sh TAG
set -o pipefail
TAG=${1:-8k}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_edge.py tests/test_gpu_f32.py "tests/test_gpu_multirank.py::test_slabs_match_single_gpu" > gpurun_out/t$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --n 8192 --steps 20 --cpu-steps 0 --cpu-steps-1t 0 > gpurun_out/b${TAG}_f64.json 2>&1 || exit 3
timeout -k 10 200 python bench.py --n 8192 --steps 20 --cpu-steps 0 --cpu-steps-1t 0 --dtype f32 > gpurun_out/b${TAG}_f32.json 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o p$TAG -- python3 $GRAFT_REPO_ROOT/bench.py --n 8192 --steps 10 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --dtype f32 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}d -o p${TAG}d -- python3 $GRAFT_REPO_ROOT/bench.py --n 8192 --steps 10 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}d.log 2>&1 || exit 6
