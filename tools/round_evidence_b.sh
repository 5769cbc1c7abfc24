#!/bin/bash
# End-of-round evidence, part B: grid-size sweep, 8192^2 (config 5) kernel stats and PMC, the
# multi-rank launch rehearsal and the 1-rank RCCL ring with the comm probe.
# usage: tools/round_evidence_b.sh TAG
TAG=${1:-rc}
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash tools/sweep.sh > gpurun_out/sweep_$TAG.txt 2>&1 || exit 6
cat gpurun_out/sweep_$TAG.txt
bash tools/prof_8k.sh ${TAG}8k > gpurun_out/prof8k_$TAG.txt 2>&1 || exit 7
bash tools/pmc.sh ${TAG}8 --n 8192 --dtype f32 --dropin-steps 0 --clock-warm-ms 200 > gpurun_out/pmc8_$TAG.log 2>&1 || exit 8
bash tools/bench_rehearsal.sh > gpurun_out/rehearsal_$TAG.txt 2>&1 || exit 9
timeout -k 10 300 python bench.py --comm-self --steps 20 --warmup 5 --cpu-steps 0 --pcg-steps 0 > gpurun_out/bench_${TAG}_commself.json 2> gpurun_out/bench_${TAG}_commself.err || exit 10
echo done
