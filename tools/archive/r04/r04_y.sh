#!/bin/bash
# round 4 (y): the driver's GPU commands on the final tree (GPU suite, smoke, bench).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_drv.json 2> $O/bench_drv.err || exit 3
python3 -c "import json; d=json.loads(open('$O/bench_drv.json').read().strip().splitlines()[-1]); print(round(d['value'],1), 'steps/s', round(d['ms_per_step'],4), 'ms; tendency frac', round(d['roofline']['frac'],3))"
