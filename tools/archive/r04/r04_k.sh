#!/bin/bash
# round 4 (k): scalar-unit load of the tendency kernels (PMC), 4096^2 F64 and 8192^2 F32.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for cfg in 4096f64 8192f32; do
  A=""; [ $cfg = 8192f32 ] && A="--n 8192 --dtype f32"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r04k/pmc_$cfg -o k -- python3 $R/bench.py $A --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/gpurun_out/r04k/pmc_$cfg.log 2>&1 || exit 1
done
ls -R $R/gpurun_out/r04k | head
