#!/bin/bash
# finished carry-ins in spec_carry (default) vs pass B finishing them (QG_NO_FINAL_CARRY=1):
# solver parity tests, bit-identity of the two forms (zeta hash after the tune_tend steps),
# kernel stats at 4096^2 (two pairs) and 1024^2.  usage: tools/final_carry_ab.sh TAG
set -o pipefail
TAG=${1:-fc}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_pcg.py tests/test_gpu_edge.py tests/test_gpu_f32.py tests/test_gpu_checkpoint.py tests/test_gpu_graph.py > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
for n in 256 1024 4096; do
  a=$(timeout -k 10 120 python tools/tune_tend.py $n | grep -o '"zeta_sha1": "[0-9a-f]*"')
  b=$(QG_NO_FINAL_CARRY=1 timeout -k 10 120 python tools/tune_tend.py $n | grep -o '"zeta_sha1": "[0-9a-f]*"')
  echo "n $n final $a nofinal $b"; [ "$a" = "$b" ] || { echo "HASH MISMATCH"; exit 2; }
done
bash tools/prof_lib.sh ${TAG}a || exit 3
QG_NO_FINAL_CARRY=1 bash tools/prof_lib.sh ${TAG}an || exit 4
bash tools/prof_lib.sh ${TAG}b || exit 5
QG_NO_FINAL_CARRY=1 bash tools/prof_lib.sh ${TAG}bn || exit 6
bash tools/prof_lib.sh ${TAG}1k -- --n 1024 --steps 200 || exit 7
QG_NO_FINAL_CARRY=1 bash tools/prof_lib.sh ${TAG}1kn -- --n 1024 --steps 200 || exit 8
