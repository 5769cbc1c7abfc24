#!/bin/bash
# kernel stats of the default library and of each lib/variants/*.so.
# usage: tools/prof_variants.sh TAG [extra bench.py args]
TAG=$1; shift
EXTRA="$@"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
prof() {  # name [lib]
  local name=$1 lib=$2
  QGMI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_$name -o $name -- python3 $R/bench.py --cpu-steps 0 --pcg-steps 0 --steps 20 $EXTRA > $R/gpurun_out/bench_${TAG}_$name.json 2> $R/gpurun_out/bench_${TAG}_$name.err || return 1
  echo "== $name"; cut -c1-200 $R/gpurun_out/bench_${TAG}_$name.json | cut -d, -f2,7
}
prof default "" || exit 1
for v in $R/julia-ocean-modelling_amd/lib/variants/*.so; do
  [ -e "$v" ] || continue
  prof $(basename $v .so) $v || exit 2
done
