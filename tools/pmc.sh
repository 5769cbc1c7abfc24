#!/bin/bash
# PMC passes (counters only with --kernel-trace, never with sys/runtime traces).
# usage: tools/pmc.sh TAG [extra bench.py args]
TAG=$1; shift
EXTRA="$@"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o $name -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --mg-steps 0 --no-pmc-live --no-reference-runs --dropin-steps 0 $EXTRA > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_LDS || exit 1
run fetch FETCH_SIZE || exit 2
run write WRITE_SIZE || exit 3
run sq2 SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM || exit 4
ls $R/gpurun_out/pmc_${TAG}_*
