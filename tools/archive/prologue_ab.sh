#!/bin/bash
# tendency prologue A/B (batched vs serial ring-fill loads, lib/exp/serial.so) + chip-full
# sweep with the batched prologue.  usage: tools/prologue_ab.sh TAG
set -o pipefail
TAG=${1:-pro}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_tendency_kernels.py tests/test_gpu_parity.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}4k serial || exit 3
bash tools/prof_lib.sh ${TAG}2k serial -- --n 2048 --steps 100 || exit 4
bash tools/prof_lib.sh ${TAG}8k serial -- --n 8192 --steps 10 --warmup 3 || exit 5
for rep in 1 2; do for w in 2 3 4 6; do
  QG_TEND_WAVES=$w timeout -k 10 200 python bench.py --n 4096 --warmup 20 --steps 200 --cpu-steps 0 --pcg-steps 0 > gpurun_out/tw.json 2>gpurun_out/tw.err || exit 6
  python -c "import json; d=json.loads(open('gpurun_out/tw.json').read().strip().splitlines()[-1]); print(4096, 'waves', $w, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
done; done
