#!/bin/bash
# tendency walk-direction A/B: parity tests touching the tendency, kernel stats of the default
# library vs lib/exp/uponly.so (4096^2 twice, 8192^2), FETCH_SIZE of both.  usage: tools/walk_ab.sh TAG
set -o pipefail
TAG=${1:-wab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_tendency_kernels.py tests/test_gpu_parity.py tests/test_gpu_pcg.py tests/test_gpu_multirank.py tests/test_gpu_configs.py tests/test_gpu_rccl_ring.py tests/test_gpu_edge.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_lib.sh ${TAG}a uponly || exit 3
bash tools/prof_lib.sh ${TAG}b uponly || exit 4
bash tools/prof_lib.sh ${TAG}8k uponly -- --n 8192 --steps 10 --warmup 3 || exit 5
bash tools/prof_lib.sh ${TAG}pcg uponly -- --solver pcg || exit 6
bash tools/pmc_traffic.sh ${TAG}d || exit 7
QGMI355_LIB=$GRAFT_REPO_ROOT/julia-ocean-modelling_amd/lib/exp/uponly.so bash tools/pmc_traffic.sh ${TAG}u || exit 8
python3 tools/pmc_to_json.py ${TAG}d 4096 gpurun_out/pmc_${TAG}d.json > /dev/null && python3 tools/pmc_to_json.py ${TAG}u 4096 gpurun_out/pmc_${TAG}u.json > /dev/null
python3 -c "
import json
for t in ('${TAG}d','${TAG}u'):
    d=json.load(open('gpurun_out/pmc_%s.json'%t))['kernels']['tendency']; print(t, 'tendency read', round(d['read_bytes']/1e6,1), 'write', round(d['write_bytes']/1e6,1))"
