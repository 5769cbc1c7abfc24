#!/bin/bash
# round 4 (i): multi-rank RCCL on one GPU (--one-gpu / NCCL_HOSTID): the RCCL slab tests incl.
# configs 4 and 5 at full size, then the bench's rccl code path at 2/4/8 ranks (both launch
# modes) and at the config-4 / config-5 sizes.  SKIP_TESTS=1: the bench part only.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04i; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl_multirank.py -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; grep -E "PASS|FAIL|RCCL|passed|failed|Error" $O/tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 bash tools/rccl_rehearsal.sh 1024 2 4 8 > $O/rehearsal_1024.log 2>&1; rc=$?; cut -c1-300 $O/rehearsal_1024.log; [ $rc -ne 0 ] && exit $rc
D=gpurun_out/rccl_rehearsal
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 4 --one-gpu --steps 10 --warmup 3 --clock-warm-ms 300 > $D/run_4096_4.json 2> $D/run_4096_4.err || { tail -20 $D/run_4096_4.err; exit 2; }
tail -1 $D/run_4096_4.json | cut -c1-600
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 8 --one-gpu --grid 8192 --dtype f32 --steps 10 --warmup 3 --clock-warm-ms 300 > $D/run_8192f32_8.json 2> $D/run_8192f32_8.err || { tail -20 $D/run_8192f32_8.err; exit 3; }
tail -1 $D/run_8192f32_8.json | cut -c1-600
