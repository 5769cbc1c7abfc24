#!/bin/bash
# kernel stats of the default library and of the given experiment libraries (lib/exp/NAME.so)
# usage: tools/prof_lib.sh TAG NAME... [-- extra bench args]
TAG=$1; shift
NAMES=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done; [ "$1" = "--" ] && shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for n in default "${NAMES[@]}"; do
  L=""; [ $n != default ] && L=$R/julia-ocean-modelling_amd/lib/exp/$n.so
  QGMI355_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_$n -o $n -- python3 $R/bench.py --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --mg-steps 0 --dropin-steps 0 --no-pmc-live --no-reference-runs --steps 30 --warmup 10 "$@" > $R/gpurun_out/b_${TAG}_$n.json 2> $R/gpurun_out/b_${TAG}_$n.err || exit 1
  echo "== $n $(grep -o '"value": [0-9.]*' $R/gpurun_out/b_${TAG}_$n.json | head -1)"
  python3 $R/tools/kstats.py $R/gpurun_out/prof_${TAG}_$n/${n}_kernel_stats.csv | tail -n +2 | head -5
done
