#!/bin/bash
# multigrid PCG leg at 4096^2: the bench line's mg_pcg_solver record and rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT; R=$GRAFT_REPO_ROOT; O=gpurun_out/mgprof; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pmc-live --no-reference-runs --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --mg-steps 10 > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['mg_pcg_solver']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o mg -- python3 $R/bench.py --steps 5 --warmup 3 --no-pmc-live --no-reference-runs --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --mg-steps 10 > $R/$O/prof.log 2>&1 || exit 2
cut -d, -f1-6 $R/$O/prof/mg_kernel_stats.csv | head -30
