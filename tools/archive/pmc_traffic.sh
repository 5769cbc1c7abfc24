#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes only (per-kernel HBM traffic), for the library in
# $QGMI355_LIB (default build if unset).  usage: tools/pmc_traffic.sh TAG [extra bench.py args]
TAG=$1; shift
EXTRA="$@"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o $name -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 $EXTRA > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1
}
run fetch FETCH_SIZE || exit 2
run write WRITE_SIZE || exit 3
